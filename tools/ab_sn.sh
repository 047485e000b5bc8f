#!/bin/bash
# A/B kernel timing at a given --sn: /tmp/abs.sh SN variant...
sn=$1; shift
for v in "$@"; do
  lib=approx_counter_amd/lib/libapprox_counter_amd.so
  [ "$v" != default ] && lib=build/var/$v/libapprox_counter_amd.so
  out=$(APPROX_COUNTER_AMD_LIB=$lib timeout -k 10 200 python bench.py --sn $sn --steps 20 --no-cpu-baseline --no-host-boundary 2>/dev/null | grep metric) || exit $?
  echo "sn $sn $v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms %.4f frac %.3f" % (d["kernel_ms"], d["roofline"]["frac"]))')"
done
