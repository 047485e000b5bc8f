#!/bin/bash
# per-wave timelines of the resident cfg2 launch and of a 4x longer one (stamps build)
set -e
export APPROX_COUNTER_AMD_LIB=build/var/${1:-stamps_nop}/libapprox_counter_amd.so
timeout -k 10 120 python3 tools/stamps.py
timeout -k 10 120 python3 tools/stamps.py --sn 40000
