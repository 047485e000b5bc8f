# Same-box A/B of library variants (tools/variants.sh; "main" = the in-tree library) on the
# host-buffer stage: bench.py's synchronous steps with AC_STAGE_TRACE=1, interleaved, REPS rounds.
# usage: bash tools/stage_ab.sh "<variant> <variant> ..." [reps] [extra bench.py args]
reps=${2:-2}
extra=${3:-}
cd "$GRAFT_REPO_ROOT"
for rep in $(seq 1 "$reps"); do for v in $1; do
  lib=build/var/$v/libapprox_counter_amd.so
  [ "$v" = main ] && lib=approx_counter_amd/lib/libapprox_counter_amd.so
  out=$(APPROX_COUNTER_AMD_LIB=$lib AC_STAGE_TRACE=1 timeout -k 10 200 python3 bench.py --steps 400 --warmup 10 \
        --no-cpu-baseline --no-pipelined --no-kernel-leg $extra 2>&1) || { echo "$v rep $rep failed"; echo "$out" | tail -5; exit 1; }
  echo "$v rep $rep: $(echo "$out" | grep -o '"step_ms": {[^}]*}' | head -1)"
  echo "   $(echo "$out" | grep 'stage trace' | head -1 | cut -c1-220)"
done; done
