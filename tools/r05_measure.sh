#!/bin/bash
# Round-5 measurement batch on the GPU box (one box acquisition per call).  Every step has its
# own time limit; a test failure (rc 1) lets the next step run, anything else stops the batch.
# usage: tools/r05_measure.sh OUTDIR part...
#   slots     HISTORICAL (round 5, profiles/r05_m1): AC_SLOT_STREAMS=1 vs default.  The slot streams were
#             removed after that run, so the variable is no longer read and both arms now run the same
#             code; the part refuses to run rather than log a meaningless A/B.
#   long      2,000 cfg2 steps with the host pool at 16 / 15 / 14 participants (step-time tail)
#   stamps    per-wave timelines of the resident cfg2 launch (-DAC_STAMPS build in build/var/stamps)
#   suite     the whole -m gpu suite
#   configs   bench lines at cfg2-cfg5 (stage traces on)
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
  grep -h 'passed\|failed\|"ms_per_step"' "$OUT/$name.log" \
    | sed -e 's/.*"value": \([0-9.e+]*\).*"ms_per_step": \([0-9.]*\).*"step_ms": \({[^}]*}\).*/value \1 ms_per_step \2 \3/' \
    | cut -c1-300 | tee -a "$OUT/summary.log"
}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --no-pipelined"
B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
for part in "$@"; do
case $part in
slots)
  echo "slots: historical A/B of the removed AC_SLOT_STREAMS (profiles/r05_m1); nothing to compare now" | tee -a "$OUT/summary.log" ;;
long)
  for t in 16 15 14; do
    run long_t$t 200 env AC_HOST_THREADS=$t python3 bench.py --steps 2000 --warmup 20 $BQ --no-kernel-leg
  done ;;
stamps)
  run stamps_resident 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python3 tools/stamps.py
  run stamps_staged 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python3 tools/stage_stamps.py --calls 40 ;;
suite)
  run suite 1100 $PYT -m gpu tests ;;
tests)
  run tests_bench_path 400 $PYT -m gpu tests/test_gpu_bench_path.py
  run tests_jobs 400 $PYT -m gpu tests/test_gpu_jobs.py ;;
ptests)  # the launch tail's pieces: their tests and the parity / bench-path / jobs suites
  run tests_pieces 600 $PYT -m gpu tests/test_gpu_pieces.py
  run tests_parity 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_path.py tests/test_gpu_jobs.py ;;
pieces)  # kernel and stage A/B of the launch tail's pieces against variants
  for rep in 1 2; do
    for v in main nopieces pieces2 pieceshalf; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ksweep_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 10000,100000 --launches 200
    done
  done
  for v in main nopieces; do
    L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
    run kcfg3_$v 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 2000 --launches 30 --warmup 10
    run kcfg5_$v 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 1000 --k 22 --sl 150 --launches 30 --warmup 10
    run stage_$v 200 env $L $B
  done
  run stage_cfg5_early 200 python3 bench.py --config cfg5 --steps 20 --warmup 5 $BQ --no-kernel-leg
  run stage_cfg5_dma 200 env AC_STAGE_EARLY=0 python3 bench.py --config cfg5 --steps 20 --warmup 5 $BQ --no-kernel-leg ;;
sweep)  # kernel time against windows per wave (sample size), default item sizes and forced 2 / 4 windows per item
  for v in main chunk2 chunk4; do
    L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
    run sweep_$v 300 env $L python3 tools/kernel_sweep.py --sn 10000,20000,40000,100000
  done ;;
configs)
  for c in cfg2 cfg3 cfg5 cfg4; do
    run bench_$c 300 env AC_STAGE_TRACE=1 python3 bench.py --config $c --steps 20 --warmup 5 $BQ
  done ;;
prof)
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-pipelined --kernel-launches 100 ) \
    > "$OUT/prof_bench.log" 2>&1 || { echo "prof failed"; exit 6; }
  tail -2 "$OUT/prof_bench.log" | cut -c1-300 ;;
pmc)
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
tail)  # late claims in the launch tail x pieces: tests of the new default, then cfg2 kernel A/B, cfg3 / cfg5
  run tests_tail 600 $PYT -m gpu tests/test_gpu_pieces.py tests/test_gpu_parity.py tests/test_gpu_bench_path.py
  for rep in 1 2 3; do
    for v in main latenop nopieces piecesonly; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ksweep_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 10000 --launches 300
    done
  done
  for v in main latenop nopieces; do
    L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
    run kcfg3_$v 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 2000 --launches 30 --warmup 10
  done ;;
stamps2)  # per-wave timelines: the default and the round-4 item order
  run stamps_main 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python3 tools/stamps.py
  run stamps_nop 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps_nop/libapprox_counter_amd.so python3 tools/stamps.py ;;
handoff)  # the one-atomic count hand-off: tests, then cfg2 kernel / stage A/B against the previous commit
  run tests_handoff 900 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_path.py tests/test_gpu_jobs.py tests/test_gpu_scale.py
  for rep in 1 2 3; do
    for v in main prev; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ksweep_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 10000 --launches 300
    done
  done
  for rep in 1 2; do
    for v in main prev; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run stage_${v}_$rep 200 env $L $B
    done
  done ;;
pack8)  # eight concurrent pack-only processes on their planned CPU shares (the 8-GPU host side)
  run pack8 600 python3 tools/pack8.py
  run pack8_again 600 python3 tools/pack8.py ;;
shard)  # one rank's 1/8 cfg4 shard alone, pool at 2 (a 16-CPU quota split 8 ways) and at 16 participants
  for t in 2 16; do
    run shard_t$t 300 env AC_HOST_THREADS=$t AC_STAGE_TRACE=1 python3 bench.py --config cfg4 --shard 0/8 --steps 30 --warmup 5 $BQ
  done ;;
prio)  # raised priority for the holders of the last round's items: tests, kernel and stage A/B
  run tests_prio 900 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_path.py
  for rep in 1 2 3; do
    for v in main noprio prio2; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ksweep_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 10000 --launches 300
    done
  done
  for rep in 1 2; do
    for v in main noprio; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run stage_${v}_$rep 200 env $L $B
    done
  done
  for v in main noprio; do
    L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
    run kcfg3_$v 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 2000 --launches 30 --warmup 10
  done ;;
p1)  # k = 22 (P = 1): the early launch's staged kernel with one lane word (default) or two, and the DMA path
  for rep in 1 2; do
    run cfg5_stage_main_$rep 200 python3 bench.py --config cfg5 --steps 20 --warmup 5 $BQ --no-kernel-leg
    run cfg5_stage_words2_$rep 200 env APPROX_COUNTER_AMD_LIB=build/var/words2/libapprox_counter_amd.so python3 bench.py --config cfg5 --steps 20 --warmup 5 $BQ --no-kernel-leg
    run cfg5_stage_dma_$rep 200 env AC_STAGE_EARLY=0 python3 bench.py --config cfg5 --steps 20 --warmup 5 $BQ --no-kernel-leg
  done
  run kcfg5_main 300 python3 tools/kernel_sweep.py --sn 100000 --lim 1000 --k 22 --sl 150 --launches 30 --warmup 10
  run kcfg5_words2 300 env APPROX_COUNTER_AMD_LIB=build/var/words2/libapprox_counter_amd.so python3 tools/kernel_sweep.py --sn 100000 --lim 1000 --k 22 --sl 150 --launches 30 --warmup 10
  for rep in 1 2; do
    run cfg2_sync_$rep 200 $B
    run cfg2_submitform_$rep 200 $B --step-form submit
  done
  run tests_words2 600 env APPROX_COUNTER_AMD_LIB=build/var/words2/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_parity.py -k "every_k or equal or edge" ;;
p1b)  # the staged P = 1 kernel on two words (the new default): tests, cfg5 stage; the N > 1 step form
  run tests_p1b 900 $PYT -m gpu tests/test_gpu_jobs.py tests/test_gpu_scale.py tests/test_gpu_bench_path.py
  for rep in 1 2; do
    run cfg5_stage_main_$rep 200 python3 bench.py --config cfg5 --steps 20 --warmup 5 $BQ --no-kernel-leg
    run cfg5_stage_dma_$rep 200 env AC_STAGE_EARLY=0 python3 bench.py --config cfg5 --steps 20 --warmup 5 $BQ --no-kernel-leg
    run cfg2_sync_$rep 200 $B
    run cfg2_submitform_$rep 200 $B --step-form submit
  done ;;
chunks)  # windows per claim at cfg2: 1 (default) / 2 / 4, kernel x3 and stage x2
  for rep in 1 2 3; do
    for v in main chunk2 chunk4; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ksweep_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 10000 --launches 300
    done
  done
  for rep in 1 2; do
    for v in main chunk2 chunk4; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run stage_${v}_$rep 200 env $L $B
    done
  done ;;
final)  # what the driver runs at round end: the GPU suite, smoke, the default bench line
  run suite 1100 $PYT -m gpu tests
  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
  run bench_default 600 python3 bench.py ;;
stepform)  # the N > 1 step's way back, rehearsed on one GPU (one-rank RCCL communicator)
  for rep in 1 2 3; do
    run sf_sync_$rep 200 $B
    run sf_submit_$rep 200 $B --step-form submit
    run sf_host0_$rep 200 $B --step-form submit-host0
    run sf_host1_$rep 200 $B --step-form submit-host1
  done ;;
staged)  # the staged instantiation on resident input (every job sent ahead) against the plain kernel, cfg2-cfg5 kernel traces
  for c in cfg2 cfg3 cfg5 cfg4; do
    for m in plain staged; do
      F=""; [ $m = staged ] && F="--staged"
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/tr_${c}_$m" -o run -- \
        python3 "$GRAFT_REPO_ROOT/tools/kernel_run.py" --config $c --launches 20 --warmup 10 $F ) > "$OUT/tr_${c}_$m.log" 2>&1 \
        || { echo "trace $c $m failed"; tail -5 "$OUT/tr_${c}_$m.log"; exit 5; }
      echo "== tr $c $m ok" | tee -a "$OUT/summary.log"
    done
  done ;;
profcfg)  # kernel traces of bench.py's stage at cfg3 / cfg5 / cfg4 (the staged kernel inside the timed step)
  for c in cfg3 cfg5 cfg4; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined --kernel-launches 10 ) \
      > "$OUT/prof_$c.log" 2>&1 || { echo "prof $c failed"; exit 6; }
    echo "== prof $c ok" | tee -a "$OUT/summary.log"
  done ;;
stagedpmc)  # SQ instruction / wait counters of the staged instantiation on resident input against the plain kernel, cfg3
  for m in plain staged; do
    F=""; [ $m = staged ] && F="--staged"
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM \
      -d "$OUT/pmc3_$m" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_run.py" --config cfg3 --launches 10 --warmup 5 $F ) > "$OUT/pmc3_$m.log" 2>&1 \
      || { echo "pmc $m failed"; tail -5 "$OUT/pmc3_$m.log"; exit 3; }
    echo "== pmc3 $m ok" | tee -a "$OUT/summary.log"
  done ;;
pin)  # staged kernel's loop-read segment fields pinned in SGPRs (main) vs HEAD (prev): tests, stage cfg2-cfg5, staged-on-resident traces
  run tests_pin 900 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_path.py tests/test_gpu_jobs.py
  for rep in 1 2; do
    for v in main prev; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run stage_${v}_$rep 200 env $L $B
      for c in cfg3 cfg5 cfg4; do
        run ${c}_${v}_$rep 300 env $L python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg
      done
    done
  done
  for v in main prev; do
    ( cd /tmp && export TMPDIR=/tmp && { [ $v = main ] || export APPROX_COUNTER_AMD_LIB=$GRAFT_REPO_ROOT/build/var/$v/libapprox_counter_amd.so; } && \
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trs_cfg3_$v" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/kernel_run.py" --config cfg3 --launches 20 --warmup 10 --staged ) > "$OUT/trs_cfg3_$v.log" 2>&1 \
      || { echo "trace $v failed"; tail -5 "$OUT/trs_cfg3_$v.log"; exit 5; }
    echo "== trs cfg3 $v ok" | tee -a "$OUT/summary.log"
  done ;;
icache)  # instruction-cache counters of the staged instantiation on resident input against the plain kernel, cfg3 / cfg4
  for c in cfg3 cfg4; do
    for m in plain staged; do
      F=""; [ $m = staged ] && F="--staged"
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_REQ SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES \
        -d "$OUT/ic_${c}_$m" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_run.py" --config $c --launches 6 --warmup 4 $F ) > "$OUT/ic_${c}_$m.log" 2>&1 \
        || { echo "icache $c $m failed"; tail -5 "$OUT/ic_${c}_$m.log"; exit 3; }
      echo "== ic $c $m ok" | tee -a "$OUT/summary.log"
    done
  done ;;
copiers)  # copier workgroups per staged launch (AC_COPIER_WGS) at cfg3 / cfg4 / cfg5 and cfg2, x2
  for rep in 1 2; do
    for w in 16 32 64; do
      for c in cfg3 cfg4 cfg5; do
        run ${c}_cw${w}_$rep 300 env AC_COPIER_WGS=$w python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg
      done
      run stage_cw${w}_$rep 200 env AC_COPIER_WGS=$w $B
    done
  done ;;
wake)  # host pool woken at call entry (main) vs HEAD (prev): jobs tests, stage cfg2-cfg5 with stage traces, x2
  run tests_wake 600 $PYT -m gpu tests/test_gpu_jobs.py tests/test_gpu_bench_path.py
  for rep in 1 2; do
    for v in main prev; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run stage_${v}_$rep 200 env $L AC_STAGE_TRACE=1 $B
      for c in cfg3 cfg5 cfg4; do
        run ${c}_${v}_$rep 300 env $L AC_STAGE_TRACE=1 python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg
      done
    done
  done ;;
wake2)  # pool pre-wake: cfg2 stage x3 and cfg5 x2 interleaved, main vs prev
  for rep in 1 2 3; do
    for v in main prev; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run stage_${v}_$rep 200 env $L AC_STAGE_TRACE=1 $B
      [ $rep = 3 ] || run cfg5_${v}_$rep 300 env $L AC_STAGE_TRACE=1 python3 bench.py --config cfg5 --steps 20 --warmup 5 $BQ --no-kernel-leg
    done
  done ;;
pub)  # progress records published by a pool worker while the caller is inside the launch (main) vs HEAD (prev)
  run tests_pub 600 $PYT -m gpu tests/test_gpu_jobs.py tests/test_gpu_bench_path.py
  for rep in 1 2 3; do
    for v in main prev; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run stage_${v}_$rep 200 env $L $B
      [ $rep = 3 ] || run cfg3_${v}_$rep 300 env $L python3 bench.py --config cfg3 --steps 20 --warmup 5 $BQ --no-kernel-leg
    done
  done
  run stamps_staged 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python3 tools/stage_stamps.py --calls 40 ;;
ahead)  # LDS reads 5 / 6 bases ahead (ah5, ah6) vs 4 (main): kernel cfg2 / cfg3 / cfg5 x2
  for rep in 1 2; do
    for v in main ah5 ah6; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ksweep_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 10000 --launches 300
      run kcfg3_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 2000 --launches 30 --warmup 10
      run kcfg5_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 1000 --k 22 --sl 150 --launches 30 --warmup 10
    done
  done ;;
subq)  # waves per sub-queue 64 (main) / 16 / 32 / 128: kernel cfg2 x2, cfg3, stage cfg2 x2
  for rep in 1 2; do
    for v in main sq16 sq32 sq128; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ksweep_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 10000 --launches 300
      [ $rep = 1 ] && run kcfg3_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 2000 --launches 30 --warmup 10
      run stage_${v}_$rep 200 env $L $B
    done
  done ;;
spacing)  # the cfg2 kernel timed with events around every launch vs every 5th (back-to-back launches between), x3
  for rep in 1 2 3; do
    run every1_$rep 300 python3 tools/kernel_sweep.py --sn 10000 --launches 300 --every 1
    run every5_$rep 300 python3 tools/kernel_sweep.py --sn 10000 --launches 300 --every 5
  done ;;
legs)  # the cfg2 kernel: bench.py's kernel leg vs tools/kernel_sweep.py (every 5th launch timed), same box, x2
  for rep in 1 2; do
    run bench_$rep 300 python3 bench.py $BQ
    run sweep_$rep 300 python3 tools/kernel_sweep.py --sn 10000 --launches 100 --every 5
  done ;;
poll)  # shorter staging poll intervals (copier avail poll, gate) vs HEAD: cfg2 stage x4 interleaved
  for rep in 1 2 3 4; do
    for v in poll prev; do
      run stage_${v}_$rep 200 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so $B
    done
  done ;;
cli)  # the drop-in CLI end to end (default vs --host-exact, identical files), 10^4 and 10^5 reads, x2
  for rep in 1 2; do
    run cli_10000_$rep 300 python3 tools/cli_e2e.py --reads 10000 --lim 500
    run cli_100000_$rep 400 python3 tools/cli_e2e.py --reads 100000 --lim 2000
  done ;;
exact)  # exact count + selection on the GPU (row f1): cfg3 / cfg4 / cfg5 times and a cfg4 kernel trace
  run exact_cfg3 300 python3 tools/bench_exact.py --reads 100000 --lim 2000 --no-host
  run exact_cfg5 300 python3 tools/bench_exact.py --reads 100000 --sl 150 --k 22 --lim 1000 --no-host
  run exact_cfg4 600 python3 tools/bench_exact.py --reads 1000000 --lim 500 --no-host
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/exact_trace_cfg4" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/bench_exact.py" --reads 1000000 --lim 500 --no-host --steps 8 ) > "$OUT/exact_trace_cfg4.log" 2>&1 \
    || { echo "exact trace failed"; exit 6; }
  echo "== exact trace ok" | tee -a "$OUT/summary.log" ;;
exact2)  # keys staged in LDS for coalesced stores (main) vs HEAD (prev): exact tests, cfg3 / cfg5 / cfg4 x2, cfg4 trace
  run tests_exact 900 $PYT -m gpu tests/test_gpu_exact.py tests/test_gpu_cli.py
  for rep in 1 2; do
    for v in main prev; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ex3_${v}_$rep 300 env $L python3 tools/bench_exact.py --reads 100000 --lim 2000 --no-host
      run ex5_${v}_$rep 300 env $L python3 tools/bench_exact.py --reads 100000 --sl 150 --k 22 --lim 1000 --no-host
      run ex4_${v}_$rep 600 env $L python3 tools/bench_exact.py --reads 1000000 --lim 500 --no-host
    done
  done
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/exact_trace_cfg4" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/bench_exact.py" --reads 1000000 --lim 500 --no-host --steps 8 ) > "$OUT/exact_trace_cfg4.log" 2>&1 \
    || { echo "exact trace failed"; exit 6; }
  echo "== exact trace ok" | tee -a "$OUT/summary.log" ;;
chunk64)  # 64-KB partition chunks (ch64) vs 32 KB (prev = HEAD): exact tests on ch64, parity cfg3 / cfg5, cfg4 x2 + traces
  run tests_ch64 900 env APPROX_COUNTER_AMD_LIB=build/var/ch64/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  for v in prev ch64; do
    L="APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so"
    run par3_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --lim 2000 --steps 3 --warmup 1
    run par5_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --sl 150 --k 22 --lim 1000 --steps 3 --warmup 1
    run ex4_${v}_1 300 env $L python3 tools/bench_exact.py --reads 1000000 --lim 500 --no-host
    run ex4_${v}_2 300 env $L python3 tools/bench_exact.py --reads 1000000 --lim 500 --no-host
    ( cd /tmp && export TMPDIR=/tmp APPROX_COUNTER_AMD_LIB="$GRAFT_REPO_ROOT/build/var/$v/libapprox_counter_amd.so" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$v" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/bench_exact.py" --reads 1000000 --lim 500 --no-host --steps 8 ) > "$OUT/tr_$v.log" 2>&1 \
      || { echo "trace $v failed"; exit 6; }
  done ;;
sub_log2)  # 64 (prev = HEAD) / 128 / 256 buckets per super-bucket: parity cfg3 / cfg5, exact tests on sub8, cfg4 traces
  run tests_sub8 900 env APPROX_COUNTER_AMD_LIB=build/var/sub8/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  for v in prev sub7 sub8; do
    L="APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so"
    run par3_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --lim 2000 --steps 3 --warmup 1
    run par5_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --sl 150 --k 22 --lim 1000 --steps 3 --warmup 1
    run ex4_$v 300 env $L python3 tools/bench_exact.py --reads 1000000 --lim 500 --no-host
    ( cd /tmp && export TMPDIR=/tmp APPROX_COUNTER_AMD_LIB="$GRAFT_REPO_ROOT/build/var/$v/libapprox_counter_amd.so" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$v" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/bench_exact.py" --reads 1000000 --lim 500 --no-host --steps 8 ) > "$OUT/tr_$v.log" 2>&1 \
      || { echo "trace $v failed"; exit 6; }
  done ;;
keys_threads)  # keys kernel at 256 (prev = HEAD) / 512 / 1024 threads: parity cfg3 / cfg5, cfg4 traces
  for v in prev kt512 kt1024; do
    L="APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so"
    run par3_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --lim 2000 --steps 3 --warmup 1
    run par5_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --sl 150 --k 22 --lim 1000 --steps 3 --warmup 1
    run ex5_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --sl 150 --k 22 --lim 1000 --no-host
    ( cd /tmp && export TMPDIR=/tmp APPROX_COUNTER_AMD_LIB="$GRAFT_REPO_ROOT/build/var/$v/libapprox_counter_amd.so" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/keys_$v" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/bench_exact.py" --reads 1000000 --lim 500 --no-host --steps 8 ) > "$OUT/keys_$v.log" 2>&1 \
      || { echo "keys trace $v failed"; exit 6; }
  done ;;
keysdiag)  # keys kernel with block-private output ranges (timing diagnostic, wrong downstream) vs main: cfg4 traces
  for v in main kdiag; do
    L=$([ $v = main ] && echo "approx_counter_amd/lib/libapprox_counter_amd.so" || echo "build/var/$v/libapprox_counter_amd.so")
    ( cd /tmp && export TMPDIR=/tmp APPROX_COUNTER_AMD_LIB="$GRAFT_REPO_ROOT/$L" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/keys_$v" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/bench_exact.py" --reads 1000000 --lim 500 --no-host --steps 8 ) > "$OUT/keys_$v.log" 2>&1 \
      || { echo "keys trace $v failed"; exit 6; }
  done ;;
exact3)  # 512-thread count kernel on main: exact + CLI GPU tests, then the exact part's times and cfg4 trace
  run tests_exact 900 $PYT -m gpu tests/test_gpu_exact.py tests/test_gpu_cli.py
  ;;
count_threads)  # exact count kernel at 256 (prev = HEAD) / 512 / 1024 threads per workgroup: parity cfg3 / cfg5, times x2
  for v in prev ct512 ct1024; do
    L="APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so"
    run par3_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --lim 2000 --steps 3 --warmup 1
    run par5_$v 300 env $L python3 tools/bench_exact.py --reads 100000 --sl 150 --k 22 --lim 1000 --steps 3 --warmup 1
  done
  for rep in 1 2; do
    for v in prev ct512 ct1024; do
      L="APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so"
      run ex3_${v}_$rep 300 env $L python3 tools/bench_exact.py --reads 100000 --lim 2000 --no-host
      run ex5_${v}_$rep 300 env $L python3 tools/bench_exact.py --reads 100000 --sl 150 --k 22 --lim 1000 --no-host
      run ex4_${v}_$rep 600 env $L python3 tools/bench_exact.py --reads 1000000 --lim 500 --no-host
    done
  done ;;
ahead2)  # copy-ahead window 16 / 64 chunks vs 32 (prev = HEAD): cfg2 stage x3, cfg3 / cfg4 once
  for rep in 1 2 3; do
    for v in prev ca16 ca64; do
      run stage_${v}_$rep 200 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so $B
    done
  done
  for v in prev ca16 ca64; do
    for c in cfg3 cfg4; do
      run ${c}_${v} 300 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg
    done
  done ;;
fetch)  # split tail (main; split2: two rounds) over cur (whole-register fetch + init registers + nested-level count + no round-3 staging) over fetch (the fetch alone) over HEAD (prev)
  run tests_fetch 900 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_path.py tests/test_gpu_jobs.py
  for rep in 1 2; do
    for v in main split2 cur fetch prev; do
      L=$([ $v = main ] && echo "" || echo "APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so")
      run ksweep_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 10000 --launches 300
      run kcfg3_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 2000 --launches 30 --warmup 10
      run kcfg5_${v}_$rep 300 env $L python3 tools/kernel_sweep.py --sn 100000 --lim 1000 --k 22 --sl 150 --launches 30 --warmup 10
      run stage_${v}_$rep 200 env $L $B
    done
  done ;;
esac
done
