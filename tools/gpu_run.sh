#!/bin/bash
# GPU-box driver: each step has its own time limit; a test FAILURE (rc 1) lets the
# next step run, anything else (fault, abort, segfault, timeout) stops the script.
# usage: tools/gpu_run.sh TAG  "step1 cmd" "step2 cmd" ...
set -u
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "[step $i] $cmd" | tee -a "$OUT/steps.log"
  bash -c "$cmd" > "$OUT/step$i.log" 2>&1
  rc=$?
  echo "[step $i] rc=$rc" | tee -a "$OUT/steps.log"
  tail -n 15 "$OUT/step$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
