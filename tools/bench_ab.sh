# Same-box A/B of bench.py variants (argument sets separated by ';').
IFS=';' read -ra VARIANTS <<< "$1"
for rep in 1 2; do for v in "${VARIANTS[@]}"; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-pipelined $v > gpurun_out/ab.json 2>/dev/null || exit 1
  tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$v] value %.4g ms %.4f'%(d['value'],d['ms_per_step']), 'step_ms', {k: round(x,4) for k,x in d.get('step_ms',{}).items()})"
done; done
