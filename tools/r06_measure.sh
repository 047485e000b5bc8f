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
BQ="--no-cpu-baseline --no-pipelined --no-exact"
B="python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-pipelined --no-kernel-leg --no-exact"
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
  run tests_dp 600 $PYT -m gpu tests/test_gpu_device_pack.py tests/test_gpu_bench_path.py
  run tests_jobs 600 $PYT -m gpu tests/test_gpu_jobs.py
  run tests_exact 600 $PYT -m gpu tests/test_gpu_exact.py ;;
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
exactpmc)  # rocprof FETCH_SIZE / WRITE_SIZE passes and a kernel trace of the exact count at cfg3 / cfg4 / cfg5
  export TMPDIR=/tmp
  for spec in "cfg3 100000 100 16 2000" "cfg4 1000000 100 16 500" "cfg5 100000 150 22 1000"; do
    set -- $spec
    EX="python3 tools/bench_exact.py --fast --reads $2 --sl $3 --k $4 --lim $5 --steps 5 --warmup 2 --no-host"
    run exact_$1_fetch 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/exact_$1_fetch" -o run -- $EX
    run exact_$1_write 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/exact_$1_write" -o run -- $EX
    run exact_$1_trace 120 rocprofv3 --kernel-trace --stats -d "$OUT/exact_$1_trace" -o run -- $EX
    run exact_$1_json 60 python3 tools/exact_pmc.py --config $1 --fetch "$OUT/exact_$1_fetch" --write "$OUT/exact_$1_write" --out "$OUT/$1_exact_pmc.json"
  done ;;
xab)  # exact-count count-kernel variants (tools/variants.sh xpack*agg*), cfg4 and cfg5, x2 interleaved
  for rep in 1 2; do for v in xpack0agg0 xpack0agg1 xpack1agg0 xpack1agg1; do
    run xab_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xab_${v}_cfg5_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10 --no-host
  done; done ;;
abdev)  # cfg2 stage: device packing (16 / 32 / 64 copier workgroups) vs host packing of a heap sample
  for rep in 1 2 3; do
    run abdev_dev16_$rep 120 $B --sample pinned
    run abdev_heap_$rep 120 $B --sample heap
    run abdev_dev32_$rep 120 env AC_COPIER_WGS=32 $B --sample pinned
    run abdev_dev64_$rep 120 env AC_COPIER_WGS=64 $B --sample pinned
  done ;;
stall2)  # the default pool (quota - 2 since r06_m3) at cfg2 for 10 s and cfg5 for 200 steps
  run stall2_cfg2 120 $S --config cfg2 --seconds 10
  run stall2_cfg5 300 $S --config cfg5 --steps 200
  run stall2_cfg3 300 $S --config cfg3 --steps 300 ;;
host8)  # 8 processes at once, each one rank's host-side work per step (submit of its 1/8 cfg4 shard), x2
  for rep in 1 2; do
    run host8_pinned_$rep 400 python3 tools/host8.py --sample pinned
    run host8_heap_$rep 400 python3 tools/host8.py --sample heap
  done ;;
shardload)  # rank 0's 1/8 cfg4 shard on the GPU with 7 host-packing load processes beside it
  run shardload_pinned 500 python3 tools/shard_load.py --sample pinned
  run shardload_heap 500 python3 tools/shard_load.py --sample heap ;;
stall3)  # cfg3 tails: device-packed (pinned), and host-packed with workers pinned to the whole CPU set
  run stall3_cfg3_pinned 300 $S --config cfg3 --steps 300 --pinned
  run stall3_cfg3_pinset 300 env AC_HOST_PIN=set $S --config cfg3 --steps 300
  run stall3_cfg3_default 300 $S --config cfg3 --steps 300 ;;
wpb)  # count kernel on resident input: 4 / 8 / 16 waves per workgroup (tools/variants.sh base wpb8 wpb16)
  export TMPDIR=/tmp
  for c in cfg2 cfg5; do
    run wpb_$c 400 bash tools/kernel_ab.sh "base wpb8 wpb16" $c
  done ;;
stamps)  # per-wave timelines of the resident cfg2 launch, 4- and 16-wave workgroups (-DAC_STAMPS builds)
  run stamps_base 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python3 tools/stamps.py
  run stamps_wpb16 120 env APPROX_COUNTER_AMD_LIB=build/var/stamps16/libapprox_counter_amd.so python3 tools/stamps.py ;;
abnodp)  # host-packed stage with and without the device packer compiled into the staged kernel
  for rep in 1 2 3; do
    run abnodp_cur_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/cur/libapprox_counter_amd.so $B --sample heap
    run abnodp_nodp_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/nodp/libapprox_counter_amd.so $B --sample heap
  done
  for c in cfg5 cfg3; do
    run abnodp_cur_$c 300 env APPROX_COUNTER_AMD_LIB=build/var/cur/libapprox_counter_amd.so python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg --sample heap
    run abnodp_nodp_$c 300 env APPROX_COUNTER_AMD_LIB=build/var/nodp/libapprox_counter_amd.so python3 bench.py --config $c --steps 20 --warmup 5 $BQ --no-kernel-leg --sample heap
  done ;;
xab2)  # count kernel: CAS as the probe, 4 / 16 keys per thread per batch, vs the current (cur)
  for rep in 1 2; do for v in cur xcas xb16 xb4; do
    run xab2_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
  done; done ;;
pin)  # host pool workers on the whole CPU set (default since r06_m6) vs one CPU each: cfg2 stage and tails
  for rep in 1 2 3; do
    run pin_set_$rep 120 $B --sample heap
    run pin_each_$rep 120 env AC_HOST_PIN=each $B --sample heap
  done
  run pinstall_cfg2_set 120 $S --config cfg2 --seconds 10
  run pinstall_cfg2_each 120 env AC_HOST_PIN=each $S --config cfg2 --seconds 10
  run pinstall_cfg3_set 300 $S --config cfg3 --steps 300
  run pinstall_cfg5_set 300 $S --config cfg5 --steps 200 ;;
final1)  # the round's end: whole GPU suite, smoke, the default bench line twice
  run suite 1200 $PYT -m gpu tests
  run smoke 300 python3 -c 'import __graft_entry__ as g; g.smoke()'
  run bench_cfg2_a 400 python3 bench.py
  run bench_cfg2_b 400 python3 bench.py --no-cpu-baseline ;;
final2)  # rocprof evidence: the bench's kernel trace, the count kernel's PMC passes, cfg3-cfg5 lines
  export TMPDIR=/tmp
  run bench_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/bench_trace" -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-pipelined --no-exact
  run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- python3 tools/kernel_run.py --config cfg2 --launches 20
  run pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- python3 tools/kernel_run.py --config cfg2 --launches 20
  run pmc_sq 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d "$OUT/pmc_sq" -o run -- python3 tools/kernel_run.py --config cfg2 --launches 20
  run pmc_json 60 python3 tools/pmc_traffic.py --fetch "$OUT/pmc_fetch" --write "$OUT/pmc_write" --valu "$OUT/pmc_sq" --workload "cfg2: k=16 sn=10000 sl=100 lim=500, start+end ends fused, 10000 reads/rank" --out "$OUT/r06_cfg2_pmc_traffic.json"
  run kern_trace 200 rocprofv3 --kernel-trace --stats -d "$OUT/kern_trace" -o run -- python3 tools/kernel_run.py --config cfg2 --launches 50 --warmup 150
  for c in cfg3 cfg5 cfg4; do
    run bench_$c 400 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined --no-exact
  done ;;
xab3)  # count kernel: claimed slots listed by a table scan (xscan) vs the per-claim append (cur)
  for rep in 1 2; do for v in cur xscan; do
    run xab3_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xab3_${v}_cfg3_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10
  done; done ;;
xtime)  # count kernel split (timing-only builds): no scoring (xt1), no inserts (xt2), full (cur)
  for rep in 1 2; do for v in cur xt1 xt2; do
    run xtime_${v}_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
  done; done ;;
rank8)  # cfg2 with one rank's share of an 8-rank node (LOCAL_WORLD_SIZE=8: a 1-participant pool): host vs device packing
  for rep in 1 2; do
    run rank8_host_$rep 120 env LOCAL_WORLD_SIZE=8 LOCAL_RANK=0 AC_DEVICE_PACK=0 $B --sample pinned
    run rank8_dev_$rep 120 env LOCAL_WORLD_SIZE=8 LOCAL_RANK=0 $B --sample pinned
  done
  run submit1 200 python3 bench.py --step-form submit --steps 200 --warmup 10 $BQ --no-kernel-leg ;;
tailab)  # count kernel: launch-tail split into one-word halves (tools/variants.sh tail1/tail2/tail4) vs cur
  # (and the packed count hand-off, hpack: AC_HAND_PACK=1)
  run tests_tail2 900 env APPROX_COUNTER_AMD_LIB=build/var/tail2/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_jobs.py tests/test_gpu_bench_path.py tests/test_gpu_device_pack.py
  run tests_hpack 900 env APPROX_COUNTER_AMD_LIB=build/var/hpack/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_jobs.py tests/test_gpu_bench_path.py
  run kab_cfg2 900 bash tools/kernel_ab.sh "cur tail1 tail2 tail4 hpack" cfg2
  run kab_cfg5 900 bash tools/kernel_ab.sh "cur tail2 hpack" cfg5
  for rep in 1 2; do for v in cur tail1 tail2 tail4 hpack; do
    run stage_${v}_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so $B
  done; done ;;
xearly)  # exact count: the next bucket's first batch requested before this bucket's inserts (xearly), buckets of
         # ~4k keys (xb4k: AC_BUCKET_KEYS=4096), both (xeb4k), vs cur
  run tests_xeb4k 600 env APPROX_COUNTER_AMD_LIB=build/var/xeb4k/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  for rep in 1 2; do for v in cur xearly xb4k xeb4k; do
    run xe_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xe_${v}_cfg3_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10
  done; done ;;
host8c2)  # 8 processes at once, each one rank's host-side work per cfg2 step: host-packed (auto) vs device-packed
  for rep in 1 2; do
    run host8c2_auto_$rep 300 python3 tools/host8.py --config cfg2 --sample pinned
    run host8c2_dev_$rep 300 env AC_DEVICE_PACK=1 python3 tools/host8.py --config cfg2 --sample pinned
  done ;;
sub7)  # exact count: 512 super-buckets of 128 buckets (sub7: AC_SUB_LOG2=7; longer level-1 runs) vs 1024 x 64 (cur)
  run tests_sub7 600 env APPROX_COUNTER_AMD_LIB=build/var/sub7/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  for rep in 1 2; do for v in cur sub7; do
    run xs_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xs_${v}_cfg3_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10
    run xs_${v}_cfg5_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10
  done; done
  export TMPDIR=/tmp
  run xs_trace_sub7 200 env APPROX_COUNTER_AMD_LIB=build/var/sub7/libapprox_counter_amd.so rocprofv3 --kernel-trace --stats -d "$OUT/xs_trace_sub7" -o run -- python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 5 --no-host ;;
xsq)  # exact count at cfg4: SQ wave-cycle split and LDS counters per kernel (where the count kernel's time goes)
  run xsq 600 bash tools/pmc_exact_sq.sh "$OUT/xsq" ;;
phab)  # exact count: phased inserts (ph8 / ph4: AC_COUNT_PHASED, batch 8 / 4) vs sub7, all with 512 x 128 buckets
  for v in ph4 ph8; do
    run tests_$v 600 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  done
  for rep in 1 2; do for v in sub7 ph8 ph4; do
    run xp_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xp_${v}_cfg3_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10
    run xp_${v}_cfg5_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10
  done; done ;;
bkab)  # exact count: 256 super-buckets of 256 (sub8), buckets of ~4k keys with a 1,024-probe reach (b4k), vs cur
  for v in sub8 b4k; do
    run tests_$v 600 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  done
  for rep in 1 2; do for v in cur sub8 b4k; do
    run xb_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xb_${v}_cfg3_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10
    run xb_${v}_cfg5_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10
  done; done
  export TMPDIR=/tmp
  run xb_trace_b4k 200 env APPROX_COUNTER_AMD_LIB=build/var/b4k/libapprox_counter_amd.so rocprofv3 --kernel-trace --stats -d "$OUT/xb_trace_b4k" -o run -- python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 5 --no-host ;;
dustab)  # exact count: DUST sums by v_dot4_u32_u8 (dust) vs the extract / multiply loop (cur)
  run tests_dust 600 env APPROX_COUNTER_AMD_LIB=build/var/dust/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  for rep in 1 2; do for v in cur dust; do
    run xd_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xd_${v}_cfg3_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10
    run xd_${v}_cfg5_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10
  done; done
  run xsq_dust 600 bash tools/pmc_exact_sq.sh "$OUT/xsq_dust" build/var/dust/libapprox_counter_amd.so ;;
xkt)  # keys kernel: static per-workgroup ranges with a non-returning count add (timing-only xkt) vs cur, kernel traces
  export TMPDIR=/tmp
  for rep in 1 2; do for v in cur xkt; do
    run xkt_${v}_$rep 200 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so rocprofv3 --kernel-trace --stats -d "$OUT/xkt_${v}_$rep" -o run -- python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 5 --no-host
    python3 tools/prof_summary.py "$OUT/xkt_${v}_$rep" | grep part_keys | tee -a "$OUT/summary.log"
  done; done ;;
aheadab)  # count kernel: ~Eq LDS reads 5 / 6 bases ahead (a5 / a6, tools/gen_tid_blocks.py --ahead) vs 4 (cur)
  run tests_a6 900 env APPROX_COUNTER_AMD_LIB=build/var/a6/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_parity.py
  run kab_cfg2 900 bash tools/kernel_ab.sh "cur a5 a6" cfg2
  run kab_cfg5 900 bash tools/kernel_ab.sh "cur a5 a6" cfg5
  run kab_cfg3 900 bash tools/kernel_ab.sh "cur a5 a6" cfg3
  for rep in 1 2; do for v in cur a5 a6; do
    run stage_${v}_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so $B
  done; done ;;
dust2ab)  # exact count: DUST with all 15 dimer places counted unconditionally (dust2) vs guarded (dust)
  run tests_dust2 600 env APPROX_COUNTER_AMD_LIB=build/var/dust2/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  for rep in 1 2; do for v in dust dust2; do
    run xd2_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xd2_${v}_cfg3_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10
  done; done ;;
dust3ab)  # exact count, k > 16: DUST by two nibble histograms + dot products (dust3) vs the guarded byte loop (dust2)
  run tests_dust3 600 env APPROX_COUNTER_AMD_LIB=build/var/dust3/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py tests/test_gpu_cli.py
  for rep in 1 2; do for v in dust2 dust3; do
    run xd3_${v}_cfg5_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10
    run xd3_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
  done; done ;;
fbfab)  # exact count with a forbidden set: LDS filter before the binary search (fbf) vs the search for every slot (dust3)
  run tests_fbf 600 env APPROX_COUNTER_AMD_LIB=build/var/fbf/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py tests/test_gpu_cli.py
  for rep in 1 2; do for v in dust3 fbf; do
    for nf in 0 1000; do
      run xf_${v}_cfg4_f${nf}_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host --forbidden $nf
    done
  done; done ;;
xhost)  # exact count's host side: HIP API + kernel + copy trace of cfg3 / cfg4 calls (where the non-kernel time goes)
  export TMPDIR=/tmp
  for c in "cfg3 100000 2000" "cfg4 1000000 500"; do
    set -- $c
    run xhost_$1 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d "/tmp/xhost_$1" -o run -- python3 tools/bench_exact.py --fast --reads $2 --lim $3 --steps 4 --warmup 2 --no-host
    python3 tools/host_gaps.py "/tmp/xhost_$1" > "$OUT/xhost_$1_timeline.txt" 2>&1; rm -rf "/tmp/xhost_$1"
  done ;;
fbb)  # exact count with a forbidden set searched per bucket (the in-tree library): tests, cfg4 / cfg5 with 0 / 1,000
  run tests_fbb 600 $PYT -m gpu tests/test_gpu_exact.py tests/test_gpu_cli.py
  for rep in 1 2; do for nf in 0 1000; do
    run xfb_cfg4_f${nf}_$rep 120 python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host --forbidden $nf
    run xfb_cfg5_f${nf}_$rep 120 python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10 --no-host --forbidden $nf
  done; done ;;
xcomp)  # exact count with pinned readbacks and device-side DUST scores for the ranking (in-tree library)
  run tests_xcomp 600 $PYT -m gpu tests/test_gpu_exact.py tests/test_gpu_cli.py
  for rep in 1 2; do
    run xc_cfg3_$rep 120 python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10
    run xc_cfg4_$rep 120 python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xc_cfg5_$rep 120 python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10
  done
  export TMPDIR=/tmp
  run xhost_cfg3 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d "/tmp/xhost_cfg3" -o run -- python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 4 --warmup 2 --no-host
  python3 tools/host_gaps.py "/tmp/xhost_cfg3" > "$OUT/xhost_cfg3_timeline.txt" 2>&1; rm -rf "/tmp/xhost_cfg3" ;;
dbab)  # exact count: histogram / list count double-buffered by bucket parity, one barrier less per bucket (db) vs cur
  run tests_db 600 env APPROX_COUNTER_AMD_LIB=build/var/db/libapprox_counter_amd.so $PYT -m gpu tests/test_gpu_exact.py
  for rep in 1 2; do for v in cur db; do
    run xdb_${v}_cfg4_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 1000000 --lim 500 --steps 10 --no-host
    run xdb_${v}_cfg3_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --lim 2000 --steps 10 --no-host
    run xdb_${v}_cfg5_$rep 120 env APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so python3 tools/bench_exact.py --fast --reads 100000 --sl 150 --k 22 --lim 1000 --steps 10 --no-host
  done; done ;;
rehearse)  # the N > 1 bench path end to end on one GPU: cfg2 weak (the driver's SCALE config), 1 / 2 / 4 gloo ranks
  run rehearse_cfg2 900 bash tools/rehearse_ranks.sh "$OUT/rehearsal" cfg2 ;;
*) echo "unknown part $part" ;;
esac
done
