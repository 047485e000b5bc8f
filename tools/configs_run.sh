# Bench lines of the larger BASELINE configs (1 GPU) and a 2-rank gloo rehearsal of cfg4 strong scaling.
set -e
for c in cfg3 cfg5 cfg4; do
  timeout -k 10 400 python3 bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 8 > gpurun_out/r02_bench_$c.log 2>&1
  tail -1 gpurun_out/r02_bench_$c.log | cut -c1-400
done
AC_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --config cfg4 --gpus 2 --steps 5 --warmup 2 > gpurun_out/r02_bench_cfg4_2rank_gloo.log 2>&1
tail -1 gpurun_out/r02_bench_cfg4_2rank_gloo.log | cut -c1-400
