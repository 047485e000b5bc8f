#!/bin/bash
# Round-3 measurement batch on the GPU box (one box acquisition): early-launch timeline and
# A/B, host pack latency, pool pinning / spin A/B, exact-count paths at cfg3-cfg5 sizes, CLI
# end to end at cfg2-cfg4 sizes.  usage: tools/r03_measure.sh OUTDIR [parts...]
set -u
OUT=$1; shift
case $OUT in /*) ;; *) OUT=${GRAFT_REPO_ROOT:-$(pwd)}/$OUT ;; esac  # absolute: the profiler steps cd to /tmp
PARTS=${*:-"early pack pool exact cli"}
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a "$OUT/summary.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/summary.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  grep -h '"ms_per_step"\|stage trace\|^job\|^both\|pin,\|"ms_per_call"\|seg [0-9]' "$OUT/$name.log" \
    | sed -e 's/.*"ms_per_step": \([0-9.]*\).*"step_ms": \({[^}]*}\).*/ms_per_step \1 \2/' | cut -c1-300 | tee -a "$OUT/summary.log"
}
B="python3 bench.py --steps 400 --warmup 10 --no-cpu-baseline --no-pipelined --no-kernel-leg"
for part in $PARTS; do
case $part in
early)
  run stamps 120 env AC_STAGE_EARLY=1 APPROX_COUNTER_AMD_LIB=build/var/stamps_noacq/libapprox_counter_amd.so python3 tools/stage_stamps.py --calls 40
  for m in 1 0 1 0; do run bench_early$m 200 env AC_STAGE_EARLY=$m AC_STAGE_TRACE=1 APPROX_COUNTER_AMD_LIB=build/var/noacq/libapprox_counter_amd.so $B; done ;;
pack)
  g++ -O3 -std=c++17 -pthread -Iapprox_counter_amd/csrc tools/pack_bench.cpp approx_counter_amd/csrc/host_pack.cpp -o "$OUT/pack_bench" || exit 2
  run pack_bench 120 "$OUT/pack_bench" 10000 3000 ;;
pool)
  for v in "AC_HOST_PIN=1" "AC_HOST_PIN=set" "AC_HOST_PIN=1 AC_HOST_SPIN_US=200" "AC_HOST_PIN=set AC_HOST_SPIN_US=200"; do
    run "pool_${v// /_}" 200 env $v python3 bench.py --steps 2000 --warmup 10 --no-cpu-baseline --no-pipelined --no-kernel-leg
  done ;;
exact)
  run exact_cfg3 300 python3 tools/bench_exact.py --reads 100000 --lim 2000
  run exact_cfg3_hash 300 env AC_EXACT_HASH=1 python3 tools/bench_exact.py --reads 100000 --lim 2000 --no-host
  run exact_cfg4 400 python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10
  run exact_cfg4_hash 400 env AC_EXACT_HASH=1 python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
  run exact_cfg5 300 python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000
  run exact_cfg5_hash 300 env AC_EXACT_HASH=1 python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --no-host ;;
exactprof)  # kernel traces of the exact count, partitioned vs hash table, at cfg4 / cfg5 sizes
  for c in "cfg4:--fast --reads 1000000 --lim 500 --steps 5" "cfg5:--fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 5"; do
    n=${c%%:*}; a=${c#*:}
    for h in 0 1; do
      d="$OUT/prof_exact_${n}_hash$h"
      ( cd /tmp && export TMPDIR=/tmp && if [ $h = 1 ]; then export AC_EXACT_HASH=1; fi
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run -- \
        python3 "$GRAFT_REPO_ROOT/tools/bench_exact.py" $a --no-host ) > "$d.log" 2>&1 || exit 3
    done
  done ;;
prof)  # PMC passes + kernel traces of the count kernel (device-resident), and a trace of the bench's stage
  ( bash tools/pmc_passes.sh cfg2 "$(basename "$OUT")_cfg2" ) > "$OUT/pmc_passes.log" 2>&1 || exit 4
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-pipelined --kernel-launches 100 ) \
    > "$OUT/prof_bench.log" 2>&1 || exit 5 ;;
cli)
  run cli_cfg2 300 python3 tools/cli_e2e.py --reads 10000 --lim 500
  run cli_cfg3 400 python3 tools/cli_e2e.py --reads 100000 --lim 2000
  run cli_cfg4 900 python3 tools/cli_e2e.py --reads 1000000 --lim 500 ;;
esac
done
