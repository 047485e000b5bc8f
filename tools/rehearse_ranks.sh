#!/bin/bash
# Multi-rank rehearsal of the N > 1 bench path on a one-GPU box:
# cfg4 strong scaling with 1, 2 and 4 ranks sharing the GPU (gloo all-reduce on host
# copies), AC_STAGE_TRACE=1 so every rank prints its per-phase stage times, and every
# rank's host-pool plan.  usage: tools/rehearse_ranks.sh OUTDIR [config]
set -u
OUT=$1; CFG=${2:-cfg4}
mkdir -p "$OUT"
for n in 1 2 4; do
  if [ $n -eq 1 ]; then
    AC_STAGE_TRACE=1 timeout -k 10 300 python3 bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-exact \
      --no-pipelined > "$OUT/${CFG}_n$n.log" 2>&1 || exit $?
  else
    AC_STAGE_TRACE=1 AC_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --config $CFG --gpus $n \
      --steps 10 --warmup 3 --no-exact > "$OUT/${CFG}_n$n.log" 2>&1 || exit $?
  fi
  grep -E "^\[bench\] rank|stage trace" "$OUT/${CFG}_n$n.log"
  tail -1 "$OUT/${CFG}_n$n.log" | cut -c1-300
done
