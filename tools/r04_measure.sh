#!/bin/bash
# HISTORICAL: the round-4 batch as it ran.  Parts naming AC_ARM_US (armed launches) or AC_SLOT_STREAMS
# measure options removed in round 5 (ABI 6): on today's library both arms run the same code.
# Round-4 measurement batch on the GPU box (one box acquisition per call).  Every step has its
# own time limit; a test failure (rc 1) lets the next step run, anything else stops the batch.
# usage: tools/r04_measure.sh OUTDIR part...
#   tests     the GPU test files touched this round (early launch, bench path, scale)
#   suite     the whole -m gpu suite
#   configs   bench lines at cfg2-cfg5 (stage traces on)
#   shard     one rank's 1/8 cfg4 shard alone, pool capped at 2 and at 16 participants
#   copiers   copier-workgroup count A/B at cfg4 and on the shard
#   cfg2      cfg2 bench x3 (400 steps) with stage trace
#   stamps    per-wave timelines (resident cfg2 launch, staged calls)
#   ab        same-box A/B of the cfg2 stage (round-3 library, copier modes, packer stores, copy-ahead)
#   cli       CLI end to end at 10^4 / 10^5 reads
#   rehearse  1/2/4-rank cfg4 rehearsal on one GPU (gloo)
#   prof      kernel trace of bench.py at cfg2
#   pmc       SQ issue/wait counters, WRITE/FETCH_SIZE and a kernel trace of the resident cfg2 kernel
set -u
OUT=$1; shift
case $OUT in /*) ;; *) OUT=${GRAFT_REPO_ROOT:-$(pwd)}/$OUT ;; esac
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a "$OUT/summary.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/summary.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$OUT/$name.log"; exit $rc; fi
  grep -h 'passed\|failed\|stage trace\|"ms_per_step"' "$OUT/$name.log" \
    | sed -e 's/.*"value": \([0-9.e+]*\).*"ms_per_step": \([0-9.]*\).*"step_ms": \({[^}]*}\).*"kernel_ms": \([0-9.]*\).*/value \1 ms_per_step \2 \3 kernel_ms \4/' \
    | cut -c1-400 | tee -a "$OUT/summary.log"
}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --no-pipelined"
for part in "$@"; do
case $part in
tests)
  run tests_bench_path 400 $PYT -m gpu tests/test_gpu_bench_path.py
  run tests_parity 400 $PYT -m gpu tests/test_gpu_parity.py
  run tests_jobs 400 $PYT -m gpu tests/test_gpu_jobs.py
  run tests_scale 600 $PYT -m gpu tests/test_gpu_scale.py ;;
suite)
  run suite 1100 $PYT -m gpu tests ;;
configs)
  for c in cfg2 cfg3 cfg5 cfg4; do
    run bench_$c 300 env AC_STAGE_TRACE=1 python3 bench.py --config $c --steps 20 --warmup 5 $BQ
  done ;;
shard)
  for t in 2 16 2; do
    run shard_t$t 300 env AC_HOST_THREADS=$t AC_STAGE_TRACE=1 python3 bench.py --config cfg4 --shard 0/8 --steps 30 --warmup 5 $BQ
  done ;;
copiers)
  for w in 8 16 32 64; do
    run shard_t2_cw$w 300 env AC_COPIER_WGS=$w AC_HOST_THREADS=2 python3 bench.py --config cfg4 --shard 0/8 --steps 30 --warmup 5 $BQ --no-kernel-leg
    run cfg4_cw$w 300 env AC_COPIER_WGS=$w python3 bench.py --config cfg4 --steps 10 --warmup 3 $BQ --no-kernel-leg
  done ;;
stamps)  # per-wave timelines of a -DAC_STAMPS build (tools/variants.sh stamps "-DAC_STAMPS")
  run stamps_resident 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python3 tools/stamps.py
  run stamps_staged 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python3 tools/stage_stamps.py --calls 40 ;;
pmc)  # issue-time attribution of the resident cfg2 count kernel (20 launches of tools/kernel_run.py per pass)
  for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES" \
           "WRITE_SIZE" "FETCH_SIZE"; do
    n=$(echo $c | cut -d' ' -f1)
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc $c -d "$OUT/pmc_$n" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/kernel_run.py" --config cfg2 --launches 20 ) > "$OUT/pmc_$n.log" 2>&1 || { echo "pmc $n failed"; exit 3; }
    echo "== pmc $n ok" | tee -a "$OUT/summary.log"
  done
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$OUT/trace_cfg2" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/kernel_run.py" --config cfg2 --launches 50 --warmup 150 ) > "$OUT/trace_cfg2.log" 2>&1 || exit 4
  echo "== trace ok" | tee -a "$OUT/summary.log" ;;
ab)  # same-box A/B of the cfg2 stage (400 steps each, interleaved twice): round-3 library, this tree,
    # copier workgroups for small calls too, plain stores in the packer, 64 chunks of copy-ahead
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2; do
    run ab_r03_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so $B
    run ab_main_$rep 120 $B
    for w in 16 32 64; do run ab_cw${w}_$rep 120 env AC_COPIER_MIN_TICKETS=0 AC_COPIER_WGS=$w $B; done
    run ab_nostream_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/nostream/libapprox_counter_amd.so $B
    run ab_ahead64_cw32_$rep 120 env AC_COPIER_MIN_TICKETS=0 AC_COPIER_WGS=32 APPROX_COUNTER_AMD_LIB=build/var/ahead64/libapprox_counter_amd.so $B
  done ;;
ab2)  # same-box A/B: round-3 library vs this tree (small calls all-workgroup or copier staging), cfg2; cfg3 / cfg5
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2; do
    run ab_r03_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so $B
    run ab_main_$rep 120 $B
    for w in 8 16 32; do run ab_cw${w}_$rep 120 env AC_COPIER_MIN_TICKETS=0 AC_COPIER_WGS=$w $B; done
  done
  for c in cfg3 cfg5; do
    for rep in 1 2; do
      run ab_${c}_r03_$rep 200 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so python3 bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-pipelined --no-kernel-leg
      for w in 16 32; do run ab_${c}_cw${w}_$rep 200 env AC_COPIER_WGS=$w python3 bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-pipelined --no-kernel-leg; done
    done
  done ;;
cli)  # the drop-in CLI end to end (approximate-count interval from its own log), 10^4 and 10^5 reads, twice
  for rep in 1 2; do
    run cli_10000_$rep 300 python3 tools/cli_e2e.py --reads 10000 --lim 500
    run cli_100000_$rep 400 python3 tools/cli_e2e.py --reads 100000 --lim 2000
  done ;;
rehearse)  # the N > 1 bench path with 1 / 2 / 4 ranks sharing this GPU (gloo all-reduce), cfg4 strong
  ( bash tools/rehearse_ranks.sh "$OUT/rehearsal" cfg4 ) > "$OUT/rehearsal.log" 2>&1 || { echo "rehearsal failed"; tail -20 "$OUT/rehearsal.log"; exit 5; }
  tail -12 "$OUT/rehearsal.log" | cut -c1-300 ;;
prof)  # kernel trace of the bench's own run (stage + kernel leg) at cfg2
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-pipelined --kernel-launches 100 ) \
    > "$OUT/prof_bench.log" 2>&1 || { echo "prof failed"; exit 6; }
  tail -2 "$OUT/prof_bench.log" | cut -c1-300 ;;
ab3)  # packing teams: same-box cfg2 stage A/B vs the round-3 library (400 steps), then 2,000-step runs for the
     # step-time tail, and the host packer alone with teams of 2 / 4 / 8 / 16 of the 16-thread pool
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2 3; do
    run ab_r03_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so $B
    run ab_main_$rep 120 $B
    run ab_cw16_$rep 120 env AC_COPIER_MIN_TICKETS=0 AC_COPIER_WGS=16 $B
  done
  run long_r03 200 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so python3 bench.py --steps 2000 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg
  run long_main 200 python3 bench.py --steps 2000 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg
  g++ -O3 -std=c++17 -pthread -Iapprox_counter_amd/csrc tools/pack_bench.cpp approx_counter_amd/csrc/host_pack.cpp -o "$OUT/pack_bench" || exit 2
  for t in 2 4 8 16; do run pack_threads$t 60 env AC_HOST_THREADS=$t "$OUT/pack_bench" 10000 2000 0 1; done ;;
ab4)  # packing-task size (windows per task; the 16-participant pool's claims contend on one line) vs round 3
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2; do
    run ab_r03_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so $B
    for tw in 256 640 1280 2560; do run ab_task${tw}_$rep 120 env AC_TASK_WINDOWS=$tw $B; done
    run ab_task1280_cw16_$rep 120 env AC_TASK_WINDOWS=1280 AC_COPIER_MIN_TICKETS=0 AC_COPIER_WGS=16 $B
  done
  run long_main 200 python3 bench.py --steps 2000 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg ;;
ab5)  # around the new defaults (copier workgroups always, 1,280-window tasks): copier count, task size
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2; do
    run ab_r03_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so $B
    run ab_main_$rep 120 $B
    for w in 8 32; do run ab_cw${w}_$rep 120 env AC_COPIER_WGS=$w $B; done
    for tw in 960 1664; do run ab_task${tw}_$rep 120 env AC_TASK_WINDOWS=$tw $B; done
    run ab_ahead64_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/ahead64/libapprox_counter_amd.so $B
  done ;;
ab6)  # copier tickets of 1 / 4 (default) / 8 chunks vs round 3
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2; do
    run ab_r03_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so $B
    run ab_main_$rep 120 $B
    run ab_group1_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/group1/libapprox_counter_amd.so $B
    run ab_group8_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/group8/libapprox_counter_amd.so $B
  done ;;
ab7)  # two lane words at 5 resident waves per SIMD (w5 build) vs 4: kernel leg and stage at cfg2, kernel at cfg3
  for rep in 1 2; do
    run ab_k4_$rep 120 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pipelined --kernel-launches 300
    run ab_k5_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/w5/libapprox_counter_amd.so python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pipelined --kernel-launches 300
    run ab_k4_cfg3_$rep 200 python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined
    run ab_k5_cfg3_$rep 200 env APPROX_COUNTER_AMD_LIB=build/var/w5/libapprox_counter_amd.so python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined
  done ;;
ab8)  # half items (the queue's last round split by lane word): AC_SPLIT_ROUNDS 0 / 1 / 2, kernel leg + stage
  for rep in 1 2; do
    for r in 0 1 2; do
      run ab_split${r}_$rep 120 env AC_SPLIT_ROUNDS=$r python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pipelined --kernel-launches 300
    done
  done
  run ab_split1_cfg3 200 env AC_SPLIT_ROUNDS=1 python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined
  run ab_split0_cfg3 200 env AC_SPLIT_ROUNDS=0 python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined ;;
ab9)  # the kernel launched by a pool worker (task 0) while the caller publishes, vs the caller launching
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2 3; do
    run ab_r03_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/r03/libapprox_counter_amd.so $B
    run ab_task1_$rep 120 env AC_LAUNCH_TASK=1 $B
    run ab_task0_$rep 120 env AC_LAUNCH_TASK=0 $B
  done
  run ab_task1_shard_t2 200 env AC_HOST_THREADS=2 python3 bench.py --config cfg4 --shard 0/8 --steps 30 --warmup 5 --no-cpu-baseline --no-pipelined --no-kernel-leg
  run ab_task0_shard_t2 200 env AC_LAUNCH_TASK=0 AC_HOST_THREADS=2 python3 bench.py --config cfg4 --shard 0/8 --steps 30 --warmup 5 --no-cpu-baseline --no-pipelined --no-kernel-leg ;;
ab10)  # fewer resident waves for the cfg2 launch (AC_WAVE_CAP: 3 or 3.5 per SIMD instead of 4), kernel + stage
  for rep in 1 2; do
    for c in 0 3072 3584; do
      run ab_cap${c}_$rep 120 env AC_WAVE_CAP=$c python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pipelined --kernel-launches 300
    done
  done ;;
ab11)  # the first windows read from the host's pinned block before their chunk is copied, vs not
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2 3 4 5 6; do
    run ab_host_$rep 120 $B
    run ab_nohost_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/nohost/libapprox_counter_amd.so $B
  done
  for c in cfg5 cfg4; do
    run ab_host_$c 200 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined --no-kernel-leg
    run ab_nohost_$c 200 env APPROX_COUNTER_AMD_LIB=build/var/nohost/libapprox_counter_amd.so python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined --no-kernel-leg
  done ;;
ab12)  # the early-counting gate looking 62 chunks ahead vs 16 vs only the window's own chunks (kept: r04_m17)
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2 3; do
    run ab_ahead62_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/ahead62/libapprox_counter_amd.so $B
    run ab_ahead16_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/ahead16/libapprox_counter_amd.so $B
    run ab_ahead1_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/ahead1/libapprox_counter_amd.so $B
  done
  for c in cfg5 cfg4; do
    run ab_ahead62_$c 200 env APPROX_COUNTER_AMD_LIB=build/var/ahead62/libapprox_counter_amd.so python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined --no-kernel-leg
    run ab_ahead1_$c 200 env APPROX_COUNTER_AMD_LIB=build/var/ahead1/libapprox_counter_amd.so python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined --no-kernel-leg
  done ;;
tests_arm)  # the armed-launch tests first (a hang shows here, not in the suite)
  run tests_armed 400 $PYT -m gpu tests/test_gpu_armed.py ;;
arm)  # armed launches (AC_ARM_US=100; the default until r04_m21) vs none (AC_ARM_US=0): cfg2 stage 400 steps x3 interleaved; cfg3/5/4
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2 3; do
    run ab_arm_$rep 120 env AC_ARM_US=100 $B
    run ab_noarm_$rep 120 env AC_ARM_US=0 $B
  done
  for c in cfg3 cfg5 cfg4; do
    run ab_arm_$c 200 env AC_ARM_US=100 python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg
    run ab_noarm_$c 200 env AC_ARM_US=0 python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg
  done ;;
arm2)  # armed launches with a 256-window head task (default) / no head task / no arming, cfg2, x3
  B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
  for rep in 1 2 3; do
    run ab_head256_$rep 120 env AC_ARM_US=100 $B
    run ab_head128_$rep 120 env AC_ARM_US=100 AC_HEAD_WINDOWS=128 $B
    run ab_head0_$rep 120 env AC_ARM_US=100 AC_HEAD_WINDOWS=0 $B
    run ab_noarm_$rep 120 env AC_ARM_US=0 $B
  done ;;
armstamps)  # in-kernel timelines from segment 0's first sight of the call: armed (the next kernel waiting
           # through the read-back) vs not
  S="env APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so"
  run stamps_armed 120 $S AC_ARM_US=100000 python3 tools/stage_stamps.py --calls 40 --t0 progress
  run stamps_noarm 120 $S AC_ARM_US=0 python3 tools/stage_stamps.py --calls 40 --t0 progress
  run trace_arm 120 env AC_STAGE_TRACE=1 AC_ARM_US=100000 python3 bench.py --steps 400 --warmup 20 $BQ --no-kernel-leg ;;
armprof)  # kernel traces of the cfg2 stage, armed and not (tools/kernel_gaps.py: duration, idle gap, period)
  for m in arm noarm; do
    a=$([ $m = noarm ] && echo 0 || echo 100)
    ( cd /tmp && export TMPDIR=/tmp && AC_ARM_US=$a timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/prof_$m" -o run -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 300 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg ) \
      > "$OUT/prof_$m.log" 2>&1 || { echo "prof $m failed"; exit 6; }
    python3 tools/kernel_gaps.py "$(find "$OUT/prof_$m" -name '*.db' | head -1)" "wm2_count_kernel<2, true" | tee -a "$OUT/summary.log"
  done ;;
armtrace)  # host phases (AC_STAGE_TRACE) of the cfg2 stage with and without armed launches
  for rep in 1 2; do
    run trace_arm_$rep 120 env AC_STAGE_TRACE=1 AC_ARM_US=100 python3 bench.py --steps 400 --warmup 20 $BQ --no-kernel-leg
    run trace_noarm_$rep 120 env AC_STAGE_TRACE=1 AC_ARM_US=0 python3 bench.py --steps 400 --warmup 20 $BQ --no-kernel-leg
  done ;;
cfg2)
  for i in 1 2 3; do
    run cfg2_$i 200 env AC_STAGE_TRACE=1 python3 bench.py --steps 400 --warmup 10 $BQ
  done ;;
esac
done
