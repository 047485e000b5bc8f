#!/bin/bash
# Round-6 measurement batch on the GPU box (one box acquisition per call).  Every step has its
# own time limit; a test failure (rc 1) lets the next step run, anything else stops the batch.
# usage: tools/r06_measure.sh OUTDIR part...
#   stall      CPU-quota throttling vs the step-time tail: cfg2 for 10 s and
#              cfg5 for 200 steps at the default pool, at 14 participants and with a 100-us worker spin
#   stallpin   the same on pinned samples (device packing)
#   tests      the device-pack / jobs / bench-path GPU tests
#   suite      the whole -m gpu suite
#   bench      the default bench line (cfg2) and cfg3 / cfg4 / cfg5 lines
#   ab         cfg2 stage, host packing vs device packing (AC_DEVICE_PACK=0 / 1), x3 interleaved
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
  grep -h 'passed\|failed\|"ms_per_step"\|"step_ms"' "$OUT/$name.log" | cut -c1-600 | tee -a "$OUT/summary.log"
}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --no-pipelined"
B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg"
S="python3 tools/stall_check.py"
cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat > "$OUT/cgroup.txt" 2>&1
for part in "$@"; do
case $part in
stall)
  run stall_cfg2_default 120 $S --config cfg2 --seconds 10
  run stall_cfg2_t14 120 env AC_HOST_THREADS=14 $S --config cfg2 --seconds 10
  run stall_cfg2_spin100 120 env AC_HOST_SPIN_US=100 $S --config cfg2 --seconds 10
  run stall_cfg5_default 300 $S --config cfg5 --steps 200
  run stall_cfg5_t14 300 env AC_HOST_THREADS=14 $S --config cfg5 --steps 200
  run stall_cfg5_spin100 300 env AC_HOST_SPIN_US=100 $S --config cfg5 --steps 200 ;;
stallpin)
  run stallpin_cfg2 120 $S --config cfg2 --seconds 10 --pinned
  run stallpin_cfg5 300 $S --config cfg5 --steps 200 --pinned
  run stallpin_cfg4 400 $S --config cfg4 --steps 100 --pinned ;;
tests)
  run tests_dp 600 $PYT -m gpu tests/test_gpu_device_pack.py
  run tests_jobs 600 $PYT -m gpu tests/test_gpu_jobs.py tests/test_gpu_bench_path.py ;;
suite)
  run suite 1100 $PYT -m gpu tests ;;
bench)
  run bench_cfg2 300 python3 bench.py
  for c in cfg3 cfg5 cfg4; do
    run bench_$c 400 python3 bench.py --config $c --steps 20 --warmup 5 $BQ
  done ;;
ab)  # cfg2 stage: device packing (pinned sample) vs host packing of the same pinned sample vs a heap sample
  for rep in 1 2 3; do
    run ab_dev_$rep 120 $B --sample pinned
    run ab_hostpin_$rep 120 env AC_DEVICE_PACK=0 $B --sample pinned
    run ab_heap_$rep 120 $B --sample heap
  done ;;
abbig)  # cfg3 / cfg5 / cfg4 and one rank's cfg4 shard: device vs host packing
  for c in cfg3 cfg5 cfg4; do
    run abbig_dev_$c 300 python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg --sample pinned
    run abbig_heap_$c 300 python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg --sample heap
  done
  run shard_dev 300 python3 bench.py --config cfg4 --shard 0/8 --steps 50 --warmup 5 $BQ --no-kernel-leg --sample pinned
  run shard_heap_t2 300 env AC_HOST_THREADS=2 python3 bench.py --config cfg4 --shard 0/8 --steps 50 --warmup 5 $BQ --no-kernel-leg --sample heap ;;
*) echo "unknown part $part" ;;
esac
done
