# rocprofv3 passes for one config's count kernel (device-resident launches, tools/kernel_run.py):
# FETCH_SIZE, WRITE_SIZE and SQ_INSTS_VALU each in a run of its own, then a kernel trace + stats.
# usage: bash tools/pmc_passes.sh <config> <tag>
set -e
cfg=$1; tag=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS"; do
  d=gpurun_out/${tag}_$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $c -d $d -o run -- python3 tools/kernel_run.py --config $cfg --launches 20
done
# (trace: 150 warm-up launches first; summarise with tools/prof_summary.py --skip 150)
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run -- python3 tools/kernel_run.py --config $cfg --launches 50 --warmup 150
