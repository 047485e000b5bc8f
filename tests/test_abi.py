"""CPU tests of the C ABI library: it loads, exports every declared symbol, and the
host-only entry points (packing, argument checks) behave; no kernel calls here."""
import ctypes
import subprocess

import numpy as np
import pytest

import approx_counter_amd as ac
from approx_counter_amd import _lib


def test_library_exports_every_header_symbol():
    L = _lib.load()
    names = _lib.header_functions()
    assert "ac_error_count" in names and "ac_error_count_device" in names
    for n in names:
        assert hasattr(L, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    assert set(names) <= exported


def test_library_targets_gfx950():
    out = subprocess.run(["strings", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_abi_version():
    assert _lib.load().ac_abi_version() == 8  # ABI 8: one ac_error_count_device (window_len, flags)


def test_pack_layout():
    wins = ["ACGTN", "A" * 40, "", "acgtRYgt", "T" * 32]
    s = ac.pack_windows(wins)
    assert s.n_bases % 32 == 0
    assert list(s.length) == [5, 40, 0, 8, 32]
    assert all(int(x) % 32 == 0 for x in s.start)
    for w, st, ln in zip(wins, s.start, s.length):
        d5 = ac.to_dna5(w)
        for j in range(int(ln)):
            b = int(st) + j
            code = (int(s.codes[b // 16]) >> (2 * (b % 16))) & 3
            isn = (int(s.nmask[b // 32]) >> (b % 32)) & 1
            assert isn == int(d5[j] >= 4)
            if not isn:
                assert code == d5[j]
    assert s.start[-1] + s.length[-1] <= s.n_bases


def test_dna5_mapping():
    assert list(ac.to_dna5("ACGTUacgtuNRYX-")) == [0, 1, 2, 3, 3, 0, 1, 2, 3, 3, 4, 4, 4, 4, 4]


def test_null_ctx_is_rejected():
    L = _lib.load()
    st = L.ac_error_count(None, 16, None, 0, None, None)
    assert st == _lib.AC_ERR_INVALID
    assert b"ctx" in L.ac_last_error(None)


def test_comm_entry_points_without_a_context():
    """The RCCL entry points reject a NULL context before touching RCCL; the id size is
    RCCL's 128 bytes (ncclUniqueId)."""
    L = _lib.load()
    assert L.ac_comm_id_bytes() == 128
    assert L.ac_comm_unique_id(None, None) == _lib.AC_ERR_INVALID
    assert L.ac_comm_init(None, 1, 0, None) == _lib.AC_ERR_INVALID
    assert L.ac_allreduce_counts(None, None, 0, None) == _lib.AC_ERR_INVALID


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="only meaningful without a GPU")
def test_no_device_fails_loudly():
    with pytest.raises(ac.ApproxCounterError) as ei:
        ac.ApproxCounter()
    assert ei.value.status == _lib.AC_ERR_DEVICE


def test_image_too_small_rejected():
    L = _lib.load()
    lens = np.array([40], np.uint32)
    codes = np.zeros(2, np.uint32)
    nmask = np.zeros(1, np.uint32)
    dna = np.zeros(40, np.uint8)
    st = L.ac_pack_windows(dna.ctypes.data_as(_lib.p8), np.zeros(1, np.uint64).ctypes.data_as(_lib.p64),
                           lens.ctypes.data_as(_lib.p32), 1, codes.ctypes.data_as(_lib.p32),
                           nmask.ctypes.data_as(_lib.p32), np.zeros(1, np.uint64).ctypes.data_as(_lib.p64),
                           np.zeros(1, np.uint32).ctypes.data_as(_lib.p32), ctypes.c_uint64(32))
    assert st == _lib.AC_ERR_INVALID


def test_pack_matches_reference_packing_random():
    """ac_pack_windows (the AVX2 packer shared with the jobs stage) against a
    plain numpy packing: random lengths 0..200, ordinals 0..255 (> 3 = N)."""
    rng = np.random.default_rng(3)
    wins = [rng.choice(np.array([0, 1, 2, 3, 0, 1, 2, 3, 4, 5, 200], np.uint8), size=int(n))
            for n in rng.integers(0, 200, size=300)]
    s = ac.pack_windows(wins)
    exp_codes = np.zeros_like(s.codes)
    exp_nmask = np.zeros_like(s.nmask)
    pos = 0
    for w in wins:
        b = pos + np.arange(w.size)
        isn = w > 3
        np.bitwise_or.at(exp_nmask, b[isn] // 32, (np.uint32(1) << (b[isn] % 32).astype(np.uint32)))
        np.bitwise_or.at(exp_codes, b // 16, ((w & 3).astype(np.uint32) << (2 * (b % 16)).astype(np.uint32)))
        pos += (w.size + 31) // 32 * 32
    assert np.array_equal(s.nmask, exp_nmask)
    assert np.array_equal(s.codes, exp_codes)


def test_dna5_sample_rejects_windows_past_the_buffer():
    """ac_dna5_windows has no size for `bases`: the Python side checks that no
    window reaches past the buffer before the packer could read beyond it."""
    import numpy as np
    import pytest

    import approx_counter_amd as ac

    ok = ac.Dna5Sample(np.zeros(10, np.uint8), np.array([0, 5], np.uint64), np.array([5, 5], np.uint32))
    assert ok.n_windows == 2
    with pytest.raises(ValueError):
        ac.Dna5Sample(np.zeros(10, np.uint8), np.array([0, 6], np.uint64), np.array([5, 5], np.uint32))
    with pytest.raises(ValueError):
        ac.Dna5Sample(np.zeros(10, np.uint8), np.array([0], np.uint64), np.array([5, 5], np.uint32))


def test_removed_entry_points_are_gone():
    """ABI 7 removed ac_idle (a no-op since ABI 6's removal of the armed launch) and
    ac_error_count_sample (ac_error_count_samples with one job); round 4's test-only arm statistics
    went with the armed launch; ABI 8 folded ac_error_count_device_accumulate / _equal into
    ac_error_count_device's window_len and flags (ABI sprawl)."""
    L = _lib.load()
    for name in ("ac_idle", "ac_error_count_sample", "ac_testing_arm_stats", "ac_error_count_device_accumulate",
                 "ac_error_count_device_equal"):
        assert not hasattr(L, name), name


def test_device_count_null_ctx_is_rejected():
    """ac_error_count_device (ABI 8 signature) checks its arguments before it touches the device."""
    L = _lib.load()
    st = L.ac_error_count_device(None, 16, None, 0, None, 0, None)
    assert st == _lib.AC_ERR_INVALID and b"ctx" in L.ac_last_error(None)
