# Five default 20-step bench runs back to back (run-to-run spread of the headline).
for rep in 1 2 3 4 5; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pipelined > gpurun_out/rep_$rep.json 2>/dev/null || exit 1
  tail -1 gpurun_out/rep_$rep.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep $rep value %.4g ms %.4f'%(d['value'],d['ms_per_step']), 'step_ms', d['step_ms'], 'kernel_ms %.4f'%d['kernel_ms'])"
done
