#!/bin/bash
# PMC passes over the exact-count benchmark, one rocprofv3 run per pass:
#   bash tools/pmc_exact.sh OUTDIR "COUNTERS1" ["COUNTERS2" ...]
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for c in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -d $out/pass$i -o run -- python3 tools/bench_exact.py --reads 100000 --lim 2000 --steps 3 > $out/pass$i.log 2>&1 || exit 1
done
python3 tools/pmc_kernels.py $out --match part_
