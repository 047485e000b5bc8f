"""MI355X-native approximate k-mer counter (drop-in for qbonenfant/approx_counter's
approximate-count stage, ``errorCount`` at approx_counter.cpp:531-601).

The compute path is the HIP kernel behind the C ABI in
include/approx_counter_amd.h; this package is the host-side mirror of the
reference interface for that path (see counter.error_count).
"""
from .counter import (ApproxCounter, DeviceSegment, Dna5Sample, Jobs, PackedSample, error_count,
                      pack_windows, pinned_copy, pinned_empty, to_dna5)
from ._lib import ApproxCounterError

__all__ = ["ApproxCounter", "ApproxCounterError", "DeviceSegment", "Dna5Sample", "Jobs", "PackedSample",
           "error_count", "pack_windows", "pinned_copy", "pinned_empty", "to_dna5"]
