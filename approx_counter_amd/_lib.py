"""ctypes binding of include/approx_counter_amd.h.

The shared library is built in-tree (``make`` at the repo root) into
``approx_counter_amd/lib/libapprox_counter_amd.so``.  There is deliberately no
fallback: if the library is missing, importing the binding raises.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libapprox_counter_amd.so")
# Kernel-tuning experiments (tools/variants.sh) point this at another build of the same sources.
LIB_PATH = os.environ.get("APPROX_COUNTER_AMD_LIB", LIB_PATH)
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "approx_counter_amd.h")
# test-only entry points of the same library (never used by the product path)
TESTING_HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "approx_counter_amd_testing.h")

AC_OK, AC_ERR_INVALID, AC_ERR_DEVICE, AC_ERR_NOMEM, AC_ERR_INTERNAL = 0, 1, 2, 3, 4
AC_MAX_SEGS = 4
AC_MAX_JOBS = 4

p32 = ctypes.POINTER(ctypes.c_uint32)
p64 = ctypes.POINTER(ctypes.c_uint64)
p8 = ctypes.POINTER(ctypes.c_uint8)


class ACWindows(ctypes.Structure):
    _fields_ = [("codes", p32), ("nmask", p32), ("start", p64), ("length", p32),
                ("n_windows", ctypes.c_uint32), ("n_bases", ctypes.c_uint64)]


class ACSegment(ctypes.Structure):
    _fields_ = [("kmers", p64), ("n_kmers", ctypes.c_uint32), ("sample", ACWindows),
                ("counts", p32)]


class ACDna5Windows(ctypes.Structure):
    _fields_ = [("bases", p8), ("offset", p64), ("length", p32), ("n_windows", ctypes.c_uint32)]


class ACJob(ctypes.Structure):
    _fields_ = [("kmers", p64), ("n_kmers", ctypes.c_uint32), ("sample", ACDna5Windows), ("counts", p64)]


class ACSampleJob(ctypes.Structure):
    _fields_ = [("kmers", p64), ("n_kmers", ctypes.c_uint32), ("sample", ACWindows), ("counts", p64)]


class ApproxCounterError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"[ac_status {status}] {message}")
        self.status = status


_lib = None


def load():
    """Load the in-tree library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `make` (hipcc, gfx950)")
    # torch ships its own libamdhip64.so.7.  Whichever runtime is loaded first
    # serves the whole process (same soname); if ours (/opt/rocm) comes first,
    # torch's later CUDA init fails with "No HIP GPUs are available".  So when
    # torch is present, let it load its runtime first and share it.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    L.ac_abi_version.restype = ctypes.c_int
    L.ac_device_count.restype = ctypes.c_int
    L.ac_comm_id_bytes.restype = ctypes.c_int
    L.ac_comm_unique_id.argtypes = [vp, vp]
    L.ac_comm_unique_id.restype = ctypes.c_int
    L.ac_comm_init.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
    L.ac_comm_init.restype = ctypes.c_int
    L.ac_allreduce_counts.argtypes = [vp, vp, ctypes.c_uint64, vp]
    L.ac_allreduce_counts.restype = ctypes.c_int
    L.ac_last_error.argtypes = [vp]
    L.ac_last_error.restype = ctypes.c_char_p
    L.ac_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    L.ac_create.restype = ctypes.c_int
    L.ac_destroy.argtypes = [vp]
    L.ac_destroy.restype = None
    L.ac_error_count.argtypes = [vp, ctypes.c_uint32, p64, ctypes.c_uint32,
                                 ctypes.POINTER(ACWindows), p64]
    L.ac_error_count.restype = ctypes.c_int
    L.ac_error_count_device.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ACSegment), ctypes.c_uint32, p32,
                                        ctypes.c_uint32, vp]
    L.ac_error_count_device.restype = ctypes.c_int
    L.ac_image_bases.argtypes = [p32, ctypes.c_uint32]
    L.ac_image_bases.restype = ctypes.c_uint64
    L.ac_pack_windows.argtypes = [p8, p64, p32, ctypes.c_uint32, p32, p32, p64, p32,
                                  ctypes.c_uint64]
    L.ac_pack_windows.restype = ctypes.c_int
    L.ac_last_launch.argtypes = [vp, p64, p32, p32]
    L.ac_last_launch.restype = ctypes.c_int
    L.ac_sample_upload.argtypes = [vp, ctypes.POINTER(ACWindows), ctypes.POINTER(ACWindows)]
    L.ac_sample_upload.restype = ctypes.c_int
    exact = [vp, ctypes.c_uint32, ctypes.POINTER(ACWindows), ctypes.c_float, p64, ctypes.c_uint32, ctypes.c_uint64,
             ctypes.c_uint64, p64, p64, ctypes.c_uint64, p64, p64, p64]
    for fn in (L.ac_exact_count, L.ac_exact_count_device):
        fn.argtypes = exact
        fn.restype = ctypes.c_int
    L.ac_sample_upload_slot.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ACWindows), ctypes.POINTER(ACWindows)]
    L.ac_sample_upload_slot.restype = ctypes.c_int
    for fn in (L.ac_error_count_samples, L.ac_error_count_images):
        fn.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ACSampleJob), ctypes.c_uint32]
        fn.restype = ctypes.c_int
    L.ac_create_multi.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    L.ac_create_multi.restype = ctypes.c_int
    L.ac_count.argtypes = [vp, ctypes.c_uint32, p64, ctypes.c_uint32, p32, p32, p64,
                           ctypes.POINTER(ctypes.c_uint16), ctypes.c_uint32, p64]
    L.ac_count.restype = ctypes.c_int
    L.ac_error_count_jobs.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ACJob), ctypes.c_uint32]
    L.ac_error_count_jobs.restype = ctypes.c_int
    L.ac_error_count_jobs_submit.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ACJob), ctypes.c_uint32, p32, vp]
    L.ac_error_count_jobs_submit.restype = ctypes.c_int
    L.ac_check.argtypes = [vp, vp]
    L.ac_check.restype = ctypes.c_int
    L.ac_stage_mode.argtypes = [vp]
    L.ac_stage_mode.restype = ctypes.c_int
    if hasattr(L, "ac_testing_stage_hooks"):  # (an A/B build of an older ABI may lack it)
        L.ac_testing_stage_hooks.argtypes = [ctypes.c_uint32]
        L.ac_testing_stage_hooks.restype = ctypes.c_uint32
    if hasattr(L, "ac_host_alloc"):  # (ABI >= 7; A/B builds of older ABIs lack it)
        L.ac_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(vp)]
        L.ac_host_alloc.restype = ctypes.c_int
        L.ac_host_free.argtypes = [vp]
        L.ac_host_free.restype = ctypes.c_int
    L.ac_exact_path.argtypes = [vp]
    L.ac_exact_path.restype = ctypes.c_int
    pint = ctypes.POINTER(ctypes.c_int)
    L.ac_set_host_cpus.argtypes = [pint, ctypes.c_int, ctypes.c_int]
    L.ac_set_host_cpus.restype = ctypes.c_int
    L.ac_host_pool_cpus.argtypes = [pint, pint, ctypes.c_int]
    L.ac_host_pool_cpus.restype = ctypes.c_int
    L.ac_plan_host_cpus.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                    pint, ctypes.c_int, pint, ctypes.c_int]
    L.ac_plan_host_cpus.restype = ctypes.c_int
    _lib = L
    return L


def header_functions():
    """Names of the functions declared in include/approx_counter_amd.h and the
    test-only include/approx_counter_amd_testing.h."""
    text = open(HEADER_PATH).read() + open(TESTING_HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ac_[a-z_]+)\s*\(", text)))


def check(status: int, ctx=None) -> None:
    if status != AC_OK:
        msg = load().ac_last_error(ctx)
        raise ApproxCounterError(status, msg.decode() if msg else "unknown error")
