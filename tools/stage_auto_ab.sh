#!/bin/bash
# Same-box A/B of library variants on the bench's stage with the library's own path choice:
#   bash tools/stage_auto_ab.sh "<variant> ..." <config> <steps>   ("default" = in-tree library)
cfg=${2:-cfg2}; steps=${3:-50}
for rep in 1 2; do for v in $1; do
  lib=approx_counter_amd/lib/libapprox_counter_amd.so
  [ "$v" != default ] && lib=build/var/$v/libapprox_counter_amd.so
  out=$(APPROX_COUNTER_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --steps $steps --warmup 3 --no-cpu-baseline --no-pipelined 2>/dev/null | grep metric) || exit 1
  echo "$cfg $v rep $rep: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("path %s step_ms p50 %.4f max %.4f value %.3e kernel_ms %.4f" % (d["stage_path_choice"]["path"], d["step_ms"]["p50"], d["step_ms"]["max"], d["value"], d["kernel_ms"]))')"
done; done
