#!/bin/bash
# A/B kernel timing of library variants (tools/variants.sh) on the GPU box:
#   tools/ab_bench.sh "cfg2 cfg3" default prio nostatic ...
# "default" is the in-tree library.  Prints the bench's kernel_ms and frac per run.
cfgs=$1; shift
for cfg in $cfgs; do
  for v in "$@"; do
    lib=approx_counter_amd/lib/libapprox_counter_amd.so
    [ "$v" != default ] && lib=build/var/$v/libapprox_counter_amd.so
    steps=50; [ "$cfg" != cfg2 ] && steps=10
    out=$(APPROX_COUNTER_AMD_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps $steps --no-cpu-baseline --no-host-boundary 2>/dev/null | grep metric) || exit $?
    echo "$cfg $v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms %.4f step_ms %.4f frac %.3f" % (d["kernel_ms"], d["ms_per_step"], d["roofline"]["frac"]))')"
  done
done
