#!/bin/bash
# Same-box A/B of library variants on the host-buffer stage (bench `value`), with the
# transfer path forced both ways:  bash tools/stage_lib_ab.sh "<variant> ..." <config> <steps>
# ("default" = the in-tree library).
cfg=${2:-cfg2}; steps=${3:-50}
for rep in 1 2; do for v in $1; do for zc in 1 0; do
  lib=approx_counter_amd/lib/libapprox_counter_amd.so
  [ "$v" != default ] && lib=build/var/$v/libapprox_counter_amd.so
  out=$(AC_STAGE_ZEROCOPY=$zc APPROX_COUNTER_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --steps $steps --warmup 3 --no-cpu-baseline --no-pipelined 2>/dev/null | grep metric) || exit 1
  echo "$cfg $v zerocopy=$zc rep $rep: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms p50 %.4f value %.3e kernel_ms %.4f" % (d["step_ms"]["p50"], d["value"], d["kernel_ms"]))')"
done; done; done
