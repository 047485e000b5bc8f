#!/bin/bash
# One GPU-box pass for a round's evidence: parity tests, the default bench line,
# a rocprofv3 kernel-trace of the bench, and the two PMC passes for HBM traffic.
# usage (on the box, from the repo root): tools/gpu_profile.sh TAG [bench args...]
TAG=$1; shift
D=$GRAFT_REPO_ROOT/gpurun_out/$TAG
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-pipelined $*"
P="cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3"
exec tools/gpu_run.sh $TAG \
  "timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 300 python bench.py $*" \
  "$P --kernel-trace --stats -d $D/trace -o run -- $B" \
  "$P --kernel-trace --pmc FETCH_SIZE -d $D/pmc_fetch -o run -- $B" \
  "$P --kernel-trace --pmc WRITE_SIZE -d $D/pmc_write -o run -- $B"
