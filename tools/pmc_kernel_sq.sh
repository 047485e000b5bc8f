#!/bin/bash
# SQ issue counters of the count kernel (device-resident launches), one rocprofv3 run per pass:
#   bash tools/pmc_kernel_sq.sh <config> <outdir> [library]
cfg=$1; out=$2; lib=${3:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$lib" ] && export APPROX_COUNTER_AMD_LIB=$lib
mkdir -p $out; i=0
for c in "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_CYCLES" \
         "SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -d $out/pass$i -o run -- python3 tools/kernel_run.py --config $cfg --launches 20 > $out/pass$i.log 2>&1 || exit 1
done
python3 tools/pmc_kernels.py $out --match wm2_count
