#!/bin/bash
# Kernel time vs reads per end (fixed-cost fit): tools/sn_sweep.sh "2500 5000 10000 20000 40000" [bench args]
sns=$1; shift
for sn in $sns; do
  out=$(timeout -k 10 300 python bench.py --sn $sn --steps 20 --no-cpu-baseline --no-host-boundary "$@" 2>/dev/null | grep metric) || exit $?
  echo "sn $sn $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms %.4f waves %s" % (d["kernel_ms"], d["launch"]))')"
done
