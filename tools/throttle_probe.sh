for t in 16 12 8; do for rep in 1 2; do
  a=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
  AC_HOST_THREADS=$t timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-kernel-leg --no-cpu-baseline --no-pipelined > gpurun_out/thr_$t_$rep.json 2>/dev/null || exit 1
  b=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
  v=$(tail -1 gpurun_out/thr_$t_$rep.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4f'%d['ms_per_step'])")
  echo "threads $t rep $rep ms $v before [$a] after [$b]"
done; done
