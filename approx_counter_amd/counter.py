"""Host-side mirror of the reference's approximate-count interface.

``error_count(sequences, exact_count, nb_thread, k, v)`` has the argument
meaning of ``errorCount`` (approx_counter.cpp:531): ``sequences`` is the
sampled window set, ``exact_count`` the (k-mer, exact count) pairs kept by
get_most_frequent / get_solid_kmers (887-899), and the result maps every
candidate k-mer to its approximate count (``results[kmer] = total``, 596).
``nb_thread`` and ``v`` are accepted for signature parity; the work runs on the
GPU through the C ABI of include/approx_counter_amd.h.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import ACDna5Windows, ACJob, ACSampleJob, ACSegment, ACWindows, check

_DNA5 = np.full(256, 4, dtype=np.uint8)
for _c, _v in ((b"A", 0), (b"C", 1), (b"G", 2), (b"T", 3), (b"U", 3)):
    _DNA5[_c[0]] = _v
    _DNA5[_c.lower()[0]] = _v


def to_dna5(seq) -> np.ndarray:
    """Dna5 ordinal bytes (A0 C1 G2 T3, anything else 4), as SeqAn's Dna5String."""
    if isinstance(seq, np.ndarray):
        return np.ascontiguousarray(seq, dtype=np.uint8)
    if isinstance(seq, str):
        seq = seq.encode()
    return _DNA5[np.frombuffer(bytes(seq), dtype=np.uint8)]


def _ptr(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


class PackedSample:
    """Host window image (see ac_windows in include/approx_counter_amd.h)."""

    def __init__(self, codes, nmask, start, length, n_bases):
        self.codes, self.nmask, self.start, self.length = codes, nmask, start, length
        self.n_bases = int(n_bases)

    @property
    def n_windows(self) -> int:
        return int(self.length.size)

    @property
    def total_bases(self) -> int:
        return int(self.length.sum(dtype=np.uint64))

    def as_struct(self) -> ACWindows:
        return ACWindows(_ptr(self.codes, ctypes.c_uint32), _ptr(self.nmask, ctypes.c_uint32),
                         _ptr(self.start, ctypes.c_uint64), _ptr(self.length, ctypes.c_uint32),
                         self.n_windows, self.n_bases)

    def equal_window_len(self):
        """The common window length when every window has it and window w starts at base
        w * ceil32(length) (the layout ac_error_count_device reads without descriptors when given window_len),
        else None."""
        n = self.n_windows
        if n == 0:
            return None
        ln = int(self.length[0])
        stride = (ln + 31) // 32 * 32
        if not np.all(self.length == ln):
            return None
        if not np.array_equal(self.start, np.arange(n, dtype=np.uint64) * np.uint64(stride)):
            return None
        return ln


def pack_windows(windows) -> PackedSample:
    """Pack Dna5 windows into the 2-bit + N-mask image with ac_pack_windows.
    `windows` is a sequence of strings / byte strings / Dna5 ordinal arrays, or a
    2-D uint8 array of equal-length windows (Dna5 ordinals, one per row)."""
    L = _lib.load()
    if isinstance(windows, np.ndarray) and windows.ndim == 2:
        n, wl = windows.shape
        arrs = [None] * n
        lengths = np.full(n, wl, dtype=np.uint32)
        starts = np.arange(n, dtype=np.uint64) * np.uint64(wl)
        flat = np.ascontiguousarray(windows, dtype=np.uint8).reshape(-1)
        if flat.size == 0:
            flat = np.zeros(1, np.uint8)
    else:
        arrs = [to_dna5(w) for w in windows]
        lengths = np.array([a.size for a in arrs], dtype=np.uint32)
        starts = np.zeros(len(arrs), dtype=np.uint64)
        if len(arrs) > 1:
            starts[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
        flat = np.concatenate(arrs) if arrs and lengths.sum() else np.zeros(1, np.uint8)
    flat = np.ascontiguousarray(flat, dtype=np.uint8)
    lens_c = lengths if lengths.size else np.zeros(1, np.uint32)
    n_bases = int(L.ac_image_bases(_ptr(lens_c, ctypes.c_uint32), len(arrs)))
    codes = np.zeros(n_bases // 16, dtype=np.uint32)
    nmask = np.zeros(n_bases // 32, dtype=np.uint32)
    out_start = np.zeros(max(len(arrs), 1), dtype=np.uint64)
    out_len = np.zeros(max(len(arrs), 1), dtype=np.uint32)
    st = L.ac_pack_windows(_ptr(flat, ctypes.c_uint8),
                           _ptr(starts if starts.size else np.zeros(1, np.uint64), ctypes.c_uint64),
                           _ptr(lens_c, ctypes.c_uint32), len(arrs),
                           _ptr(codes, ctypes.c_uint32), _ptr(nmask, ctypes.c_uint32),
                           _ptr(out_start, ctypes.c_uint64), _ptr(out_len, ctypes.c_uint32), n_bases)
    check(st)
    return PackedSample(codes, nmask, out_start[: len(arrs)], out_len[: len(arrs)], n_bases)


class _PinnedBlock:
    """One ac_host_alloc block, released when the last array viewing it goes (numpy keeps this
    object as the arrays' base)."""

    def __init__(self, nbytes: int):
        L = _lib.load()
        p = ctypes.c_void_p()
        check(L.ac_host_alloc(max(int(nbytes), 1), ctypes.byref(p)))
        self._L, self.ptr, self.nbytes = L, p.value, max(int(nbytes), 1)
        self.__array_interface__ = {"shape": (self.nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                    "version": 3}

    def __del__(self):
        if getattr(self, "ptr", None):
            self._L.ac_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = None


def pinned_empty(n: int, dtype) -> np.ndarray:
    """An uninitialised array of n elements in pinned, device-mapped host memory (ac_host_alloc)."""
    dt = np.dtype(dtype)
    return np.asarray(_PinnedBlock(n * dt.itemsize)).view(dt)[:n]


def pinned_copy(a) -> np.ndarray:
    """A copy of `a` in ac_host_alloc memory."""
    a = np.ascontiguousarray(a)
    out = pinned_empty(max(a.size, 1), a.dtype)[: a.size]
    out[...] = a.reshape(-1)
    return out.reshape(a.shape)


class Dna5Sample:
    """A sample as errorCount receives it: a StringSet<Dna5String>
    (approx_counter.cpp:38), i.e. Dna5 ordinal bytes concatenated, with each
    window's offset and length (ac_dna5_windows)."""

    def __init__(self, bases, offset, length):
        self.bases = np.ascontiguousarray(bases, dtype=np.uint8)
        self.offset = np.ascontiguousarray(offset, dtype=np.uint64)
        self.length = np.ascontiguousarray(length, dtype=np.uint32)
        if self.offset.shape != self.length.shape:
            raise ValueError("Dna5Sample: offset and length differ in size")
        # ac_dna5_windows carries no size for `bases`: the packer would read past the buffer
        if self.length.size and int((self.offset + self.length.astype(np.uint64)).max()) > self.bases.size:
            raise ValueError("Dna5Sample: a window reaches past the end of `bases`")
        if self.bases.size == 0:
            self.bases = np.zeros(1, np.uint8)

    @classmethod
    def from_windows(cls, windows) -> "Dna5Sample":
        """From a sequence of strings / Dna5 arrays, or a 2-D uint8 array of
        equal-length windows (one per row)."""
        if isinstance(windows, np.ndarray) and windows.ndim == 2:
            n, wl = windows.shape
            return cls(windows.reshape(-1), np.arange(n, dtype=np.uint64) * np.uint64(wl),
                       np.full(n, wl, dtype=np.uint32))
        arrs = [to_dna5(w) for w in windows]
        length = np.array([a.size for a in arrs], dtype=np.uint32)
        offset = np.zeros(len(arrs), dtype=np.uint64)
        if len(arrs) > 1:
            offset[1:] = np.cumsum(length[:-1], dtype=np.uint64)
        bases = np.concatenate(arrs) if arrs and length.sum() else np.zeros(1, np.uint8)
        return cls(bases, offset, length)

    def pinned(self) -> "Dna5Sample":
        """The same sample with its bytes and offsets in ac_host_alloc memory: ac_error_count_jobs
        then packs it on the device when its windows have one length of 1..256 bases."""
        return Dna5Sample(pinned_copy(self.bases), pinned_copy(self.offset), pinned_copy(self.length))

    def subset(self, lo: int, hi: int) -> "Dna5Sample":
        """Windows [lo, hi) (a shard), sharing the bases."""
        return Dna5Sample(self.bases, self.offset[lo:hi], self.length[lo:hi])

    @property
    def n_windows(self) -> int:
        return int(self.length.size)

    @property
    def total_bases(self) -> int:
        return int(self.length.sum(dtype=np.uint64))

    def as_struct(self) -> ACDna5Windows:
        one = lambda a, t: _ptr(a if a.size else np.zeros(1, a.dtype), t)  # noqa: E731
        return ACDna5Windows(_ptr(self.bases, ctypes.c_uint8), one(self.offset, ctypes.c_uint64),
                             one(self.length, ctypes.c_uint32), self.n_windows)


class Jobs:
    """A reusable ac_job array (both read ends of one run, or shards): the
    k-mer and count arrays are kept alive with it."""

    def __init__(self, parts):
        """`parts`: sequence of (kmers, Dna5Sample)."""
        self.kmers = [np.ascontiguousarray(np.asarray(km, dtype=np.uint64)) for km, _ in parts]
        self.samples = [smp for _, smp in parts]
        self.counts = [np.zeros(max(k.size, 1), dtype=np.uint64) for k in self.kmers]
        self.n_counts = sum(int(k.size) for k in self.kmers)
        self.array = (ACJob * len(parts))(*[
            ACJob(_ptr(km if km.size else np.zeros(1, np.uint64), ctypes.c_uint64), int(km.size), smp.as_struct(),
                  _ptr(c, ctypes.c_uint64))
            for km, smp, c in zip(self.kmers, self.samples, self.counts)])

    def results(self):
        return [c[: k.size] for c, k in zip(self.counts, self.kmers)]


class ApproxCounter:
    """One device context (ac_create / ac_destroy), or with n_gpus a context
    whose host-buffer counts are sharded over that many devices (ac_create_multi)."""

    def __init__(self, device: int = -1, n_gpus: int = 0):
        L = _lib.load()
        self._L = L
        h = ctypes.c_void_p()
        if n_gpus:
            check(L.ac_create_multi(ctypes.byref(h), int(n_gpus)))
        else:
            check(L.ac_create(ctypes.byref(h), device))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.ac_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._h

    def count(self, k: int, kmers, sample: PackedSample) -> np.ndarray:
        """ac_error_count: host arrays in, uint64 counts out (input order)."""
        kmers = np.ascontiguousarray(np.asarray(kmers, dtype=np.uint64))
        counts = np.zeros(max(kmers.size, 1), dtype=np.uint64)
        ws = sample.as_struct()
        st = self._L.ac_error_count(self._h, int(k),
                                    _ptr(kmers if kmers.size else np.zeros(1, np.uint64), ctypes.c_uint64),
                                    int(kmers.size), ctypes.byref(ws), _ptr(counts, ctypes.c_uint64))
        check(st, self._h)
        return counts[: kmers.size]

    def count_words(self, k: int, kmers, win_bits, win_nmask, win_word_offset, win_len) -> np.ndarray:
        """ac_count (SURVEY.md 8(b) layout): 2-bit words, N bitmap, per-window word offset
        (even) and uint16 length."""
        kmers = np.ascontiguousarray(np.asarray(kmers, dtype=np.uint64))
        bits = np.ascontiguousarray(win_bits, dtype=np.uint32)
        nm = np.ascontiguousarray(win_nmask, dtype=np.uint32)
        off = np.ascontiguousarray(win_word_offset, dtype=np.uint64)
        ln = np.ascontiguousarray(win_len, dtype=np.uint16)
        counts = np.zeros(max(kmers.size, 1), dtype=np.uint64)
        one = lambda a, t: _ptr(a if a.size else np.zeros(1, a.dtype), t)  # noqa: E731
        st = self._L.ac_count(self._h, int(k), one(kmers, ctypes.c_uint64), int(kmers.size), one(bits, ctypes.c_uint32),
                              one(nm, ctypes.c_uint32), one(off, ctypes.c_uint64), one(ln, ctypes.c_uint16),
                              int(ln.size), _ptr(counts, ctypes.c_uint64))
        check(st, self._h)
        return counts[: kmers.size]

    def count_jobs(self, k: int, jobs) -> list:
        """ac_error_count_jobs: the whole stage from Dna5 host buffers (pack, one DMA, one
        fused launch, counts back), up to 4 jobs.  `jobs` is a Jobs object or a sequence of
        (kmers, Dna5Sample / windows); returns the uint64 counts of every job."""
        if not isinstance(jobs, Jobs):
            jobs = Jobs([(km, w if isinstance(w, Dna5Sample) else Dna5Sample.from_windows(w)) for km, w in jobs])
        st = self._L.ac_error_count_jobs(self._h, int(k), jobs.array, len(jobs.array))
        check(st, self._h)
        return jobs.results()

    def submit_jobs(self, k: int, jobs: "Jobs", d_counts, stream=None) -> None:
        """ac_error_count_jobs_submit: pack + send + launch; uint32 counts (jobs concatenated)
        go to the device tensor `d_counts` on `stream` (asynchronous)."""
        ptr = ctypes.cast(ctypes.c_void_p(d_counts.data_ptr()), ctypes.POINTER(ctypes.c_uint32))
        st = self._L.ac_error_count_jobs_submit(self._h, int(k), jobs.array, len(jobs.array), ptr,
                                                ctypes.c_void_p(stream or 0))
        if st:
            check(st, self._h)

    def _sample_jobs(self, fn, k, parts):
        keep, arr = [], []
        for km, ws in parts:
            km = np.ascontiguousarray(np.asarray(km, dtype=np.uint64))
            c = np.zeros(max(km.size, 1), dtype=np.uint64)
            keep.append((km, c))
            arr.append(ACSampleJob(_ptr(km if km.size else np.zeros(1, np.uint64), ctypes.c_uint64), int(km.size), ws,
                                   _ptr(c, ctypes.c_uint64)))
        a = (ACSampleJob * len(arr))(*arr)
        check(fn(self._h, int(k), a, len(arr)), self._h)
        return [c[: km.size] for km, c in keep]

    def count_images(self, k: int, parts) -> list:
        """ac_error_count_images: host images [(kmers, PackedSample), ...] (up to 4 jobs) in one
        fused launch per device (sharded over the devices of an n_gpus context)."""
        return self._sample_jobs(self._L.ac_error_count_images, k, [(km, smp.as_struct()) for km, smp in parts])

    def upload_sample(self, sample: PackedSample, slot: int = 0) -> ACWindows:
        """ac_sample_upload_slot: the device copy of a host image (valid until the slot's next upload)."""
        dev = ACWindows()
        hw = sample.as_struct()
        check(self._L.ac_sample_upload_slot(self._h, int(slot), ctypes.byref(hw), ctypes.byref(dev)), self._h)
        return dev

    def count_samples(self, k: int, parts) -> list:
        """ac_error_count_samples: [(kmers, device sample from upload_sample), ...], one fused launch."""
        return self._sample_jobs(self._L.ac_error_count_samples, k, parts)

    def exact_path(self) -> int:
        """ac_exact_path: 1 partitioned, 0 hash table, -1 no exact count yet."""
        return int(self._L.ac_exact_path(self._h))

    def stage_mode(self) -> int:
        """ac_stage_mode: the last jobs call's stage -- 2 early launch (the count kernel copies each
        job in as the host flags it), 0 copy kernel / copy engine ahead of the launch, -1 no call yet."""
        return int(self._L.ac_stage_mode(self._h))

    # ---- multi-process data parallelism: the count all-reduce over RCCL (ac_comm_*) ----
    def comm_unique_id(self) -> bytes:
        """ac_comm_unique_id: a fresh RCCL unique id (rank 0 sends it to every rank)."""
        buf = ctypes.create_string_buffer(self._L.ac_comm_id_bytes())
        check(self._L.ac_comm_unique_id(self._h, buf), self._h)
        return buf.raw

    def comm_init(self, n_ranks: int, rank: int, unique_id: bytes) -> None:
        """ac_comm_init: join the n_ranks-rank RCCL communicator as `rank`."""
        buf = ctypes.create_string_buffer(bytes(unique_id), self._L.ac_comm_id_bytes())
        check(self._L.ac_comm_init(self._h, int(n_ranks), int(rank), buf), self._h)

    def allreduce_counts(self, d_counts, stream=None) -> None:
        """ac_allreduce_counts: in-place uint32 sum of a device count tensor over the ranks."""
        check(self._L.ac_allreduce_counts(self._h, ctypes.c_void_p(d_counts.data_ptr()),
                                          ctypes.c_uint64(d_counts.numel()), ctypes.c_void_p(stream or 0)),
              self._h)

    def check(self, stream=None) -> None:
        """ac_check: raise if a device launch since the last check skipped a malformed window."""
        check(self._L.ac_check(self._h, ctypes.c_void_p(stream or 0)), self._h)

    def exact_count(self, k: int, sample: PackedSample, lc_threshold: float, forbidden=(), limit: int = 500,
                    solid: int = 0):
        """ac_exact_count: count_kmers (approx_counter.cpp:487-519) + get_most_frequent /
        get_solid_kmers on the GPU.  Returns ([(kmer, count), ...] in CompareCount order,
        n_distinct, had_n)."""
        fb = np.ascontiguousarray(np.asarray(list(forbidden) or [0], dtype=np.uint64))
        cap = max(1, int(limit) if not solid else 1024)
        ws = sample.as_struct()
        while True:
            km = np.zeros(cap, np.uint64)
            ct = np.zeros(cap, np.uint64)
            n_out, n_dist, had_n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
            st = self._L.ac_exact_count(self._h, int(k), ctypes.byref(ws), float(lc_threshold),
                                        _ptr(fb, ctypes.c_uint64), len(forbidden), int(limit), int(solid),
                                        _ptr(km, ctypes.c_uint64), _ptr(ct, ctypes.c_uint64), cap,
                                        ctypes.byref(n_out), ctypes.byref(n_dist), ctypes.byref(had_n))
            if st == _lib.AC_ERR_INVALID and n_out.value > cap:
                cap = int(n_out.value)
                continue
            check(st, self._h)
            n = int(n_out.value)
            return [(int(a), int(b)) for a, b in zip(km[:n], ct[:n])], int(n_dist.value), int(had_n.value)

    @staticmethod
    def segment_array(segments):
        """The ac_segment array of DeviceSegment objects, built once and reusable with
        count_device (saves the per-call ctypes marshalling in launch loops)."""
        return (ACSegment * len(segments))(*[s.as_struct() for s in segments])

    def count_device(self, k: int, segments, stream=None, accumulate: bool = False, window_len=None) -> None:
        """ac_error_count_device over DeviceSegment objects, or an array from
        segment_array (asynchronous).  window_len (one per segment): the samples'
        windows all have that length and sit back to back at ceil32 strides
        (start / length are not read).  accumulate: AC_DEVICE_ACCUMULATE."""
        arr = segments if isinstance(segments, ctypes.Array) else self.segment_array(segments)
        wp = None
        if window_len is not None:
            wl = np.ascontiguousarray(window_len, dtype=np.uint32)
            if wl.size != len(arr):
                raise ValueError("one window_len per segment")
            wp = _ptr(wl, ctypes.c_uint32)
        st = self._L.ac_error_count_device(self._h, int(k), arr, len(arr), wp, 1 if accumulate else 0,
                                           ctypes.c_void_p(stream or 0))
        if st:
            check(st, self._h)

    def last_launch(self):
        w, wpw, g = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
        check(self._L.ac_last_launch(self._h, ctypes.byref(w), ctypes.byref(wpw), ctypes.byref(g)), self._h)
        return {"waves": w.value, "windows_per_wave": wpw.value, "groups": g.value}


class DeviceSegment:
    """A segment whose arrays live in device memory (torch tensors on cuda)."""

    def __init__(self, kmers, codes, nmask, start, length, counts, n_bases: int):
        self.kmers, self.codes, self.nmask = kmers, codes, nmask
        self.start, self.length, self.counts = start, length, counts
        self.n_bases = int(n_bases)

    @classmethod
    def upload(cls, kmers, sample: PackedSample, device="cuda"):
        import torch

        def t(a):
            # uint64 / uint32 views through int64 / int32 tensors (same bytes)
            a = np.ascontiguousarray(a)
            view = {np.dtype(np.uint64): np.int64, np.dtype(np.uint32): np.int32}[a.dtype]
            return torch.from_numpy(a.view(view) if a.size else np.zeros(1, view)).to(device)

        km = np.asarray(kmers, dtype=np.uint64)
        counts = torch.zeros(max(km.size, 1), dtype=torch.int32, device=device)
        seg = cls(t(km), t(sample.codes), t(sample.nmask), t(sample.start), t(sample.length),
                  counts, sample.n_bases)
        seg.n_kmers = int(km.size)
        seg.n_windows = sample.n_windows
        return seg

    def as_struct(self) -> ACSegment:
        def p(tensor, typ):
            return ctypes.cast(ctypes.c_void_p(tensor.data_ptr()), ctypes.POINTER(typ))

        ws = ACWindows(p(self.codes, ctypes.c_uint32), p(self.nmask, ctypes.c_uint32),
                       p(self.start, ctypes.c_uint64), p(self.length, ctypes.c_uint32),
                       self.n_windows, self.n_bases)
        return ACSegment(p(self.kmers, ctypes.c_uint64), self.n_kmers, ws,
                         p(self.counts, ctypes.c_uint32))

    def counts_numpy(self) -> np.ndarray:
        return self.counts[: self.n_kmers].cpu().numpy().view(np.uint32).astype(np.uint64)


def plan_host_cpus(rank_cpulists, rank: int, allowed: str, core_of=None) -> list:
    """ac_plan_host_cpus: the host-pool CPUs of local rank `rank`, given every local
    rank's GPU cpulist (sysfs text such as "0-63,128-191"), the CPUs the process may
    use and optionally each CPU's physical core (index = CPU)."""
    L = _lib.load()
    arr = (ctypes.c_char_p * len(rank_cpulists))(*[s.encode() for s in rank_cpulists])
    core = None
    if core_of is not None:
        core = np.ascontiguousarray(np.asarray(core_of, dtype=np.int32))
    cap = 4096
    out = np.zeros(cap, np.int32)
    n = L.ac_plan_host_cpus(arr, len(rank_cpulists), int(rank), allowed.encode(),
                            _ptr(core, ctypes.c_int) if core is not None else None,
                            int(core.size) if core is not None else 0, _ptr(out, ctypes.c_int), cap)
    if n < 0:
        raise ValueError("ac_plan_host_cpus: bad arguments")
    return [int(c) for c in out[: min(n, cap)]]


def host_pool_cpus():
    """ac_host_pool_cpus: (participants, [CPUs]) of the host pool plan in force."""
    L = _lib.load()
    part = ctypes.c_int()
    out = np.zeros(4096, np.int32)
    n = L.ac_host_pool_cpus(ctypes.byref(part), _ptr(out, ctypes.c_int), out.size)
    return int(part.value), [int(c) for c in out[: min(n, out.size)]]


_default_counter = None


def _counter() -> ApproxCounter:
    global _default_counter
    if _default_counter is None:
        _default_counter = ApproxCounter()
    return _default_counter


def error_count(sequences, exact_count, nb_thread: int = 4, k: int = 16, v: int = 0) -> dict:
    """errorCount (approx_counter.cpp:531-601): {kmer: approximate count}."""
    del nb_thread, v  # OpenMP thread count / verbosity of the CPU reference
    kmers = [int(km) for km, _ in exact_count]
    if not kmers:
        return {}
    # the sample as a StringSet<Dna5String>: packed, sent and counted by ac_error_count_jobs
    counts = _counter().count_jobs(k, [(np.array(kmers, dtype=np.uint64), Dna5Sample.from_windows(sequences))])[0]
    return {km: int(c) for km, c in zip(kmers, counts)}
