# Kernel traces of the cfg2 stage (bench.py's synchronous steps + its kernel-only leg) under
# AC_STAGE_EARLY=1 (early launch, staged kernel waits for its inputs) and =3 (diagnostic: every
# job sent ahead, so the staged kernel runs on resident input): the staged instantiation's own
# cost against the plain kernel's, and what the staging adds.  usage: bash tools/staged_cost.sh TAG
tag=${1:-r03_staged_cost}
root=${GRAFT_REPO_ROOT:-$(pwd)}
for m in 3 1; do
  d=$root/gpurun_out/${tag}_early$m
  ( export AC_STAGE_EARLY=$m && cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$d" -o run -- \
      python3 "$root/bench.py" --steps 200 --warmup 10 --no-cpu-baseline --no-pipelined --kernel-launches 100 ) \
      > "$d.log" 2>&1 || { echo "AC_STAGE_EARLY=$m failed"; tail -5 "$d.log"; exit 1; }
  echo "== AC_STAGE_EARLY=$m"
  python3 "$root/tools/prof_summary.py" "$d" | grep wm2_count
  grep -o '"step_ms": {[^}]*}' "$d.log" | head -1
done
