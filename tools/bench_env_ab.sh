# Same-box A/B of environment settings for bench.py (settings separated by ';', e.g. "AC_HOST_PIN=0;AC_HOST_PIN=1").
IFS=';' read -ra VARIANTS <<< "$1"
ARGS=${2:-"--steps 20 --warmup 5"}
for rep in 1 2; do for v in "${VARIANTS[@]}"; do
  env $v timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-pipelined $ARGS > gpurun_out/envab.json 2>/dev/null || exit 1
  tail -1 gpurun_out/envab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$v] value %.4g ms %.4f'%(d['value'],d['ms_per_step']), 'step_ms', {k: round(x,4) for k,x in d.get('step_ms',{}).items()}, 'kernel_ms %.4f'%d.get('kernel_ms',0))"
done; done
