#!/bin/bash
# SQ issue / LDS counters of the exact count's kernels at cfg4 (tools/bench_exact.py, 3 calls), one
# rocprofv3 run per pass:  bash tools/pmc_exact_sq.sh <outdir> [library]
out=$1; lib=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$lib" ] && export APPROX_COUNTER_AMD_LIB=$lib
mkdir -p $out; i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
         "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVES SQ_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/pass$i -o run -- python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 3 --warmup 1 --no-host > $out/pass$i.log 2>&1 || exit 1
done
python3 tools/pmc_kernels.py $out --match part_
