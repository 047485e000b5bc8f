# Same-box A/B of library variants (tools/variants.sh) on the count kernel alone:
# rocprofv3 kernel trace of tools/kernel_run.py per variant, twice, interleaved.
# usage: bash tools/kernel_ab.sh "<variant> <variant> ..." [config]
cfg=${2:-cfg2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do for v in $1; do
  d=gpurun_out/kab_${v}_$rep
  APPROX_COUNTER_AMD_LIB=build/var/$v/libapprox_counter_amd.so timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 tools/kernel_run.py --config $cfg --launches 60 --warmup 100 > /dev/null 2>&1 || exit 1
  echo "$v rep $rep: $(python3 tools/prof_summary.py $d --skip 100 | grep wm2_count | awk -F'|' '{print "avg us", $5, "min", $6}')"
done; done
