#!/bin/bash
# Host-buffer stage under environment variants, interleaved on one box (stage leg only, traced):
#   bash tools/stage_env_ab.sh OUT "ENV1" "ENV2" ...   (ENV = "" or "A=1 B=2")
# BENCH_ARGS (environment): extra bench.py arguments, e.g. "--config cfg4 --steps 20"
out=$1; shift
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1)); echo "== rep $rep variant $i [$e] load $(cut -d' ' -f1-3 /proc/loadavg)"
    env $e AC_STAGE_TRACE=1 timeout -k 10 120 python3 bench.py --steps 200 --warmup 5 ${BENCH_ARGS:-} --no-cpu-baseline --no-kernel-leg --no-pipelined > $out.tmp 2>&1 || { cat $out.tmp; exit 1; }
    grep "stage trace" $out.tmp
    grep '^{' $out.tmp | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['step_ms']; print('value %.3g ms/step %.4f p50 %.4f min %.4f max %.4f' % (d['value'], d['ms_per_step'], s['p50'], s['min'], s['max']))"
  done
done
rm -f $out.tmp
