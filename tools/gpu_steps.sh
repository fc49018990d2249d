#!/bin/bash
# Run GPU steps in sequence; stop at the first step that crashed/faulted/timed out
# (pytest rc 1 = ordinary test failures is allowed to continue).
# usage: bash tools/gpu_steps.sh "<timeout> <logname> <cmd...>" ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  read -r to log cmd <<< "$spec"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "== $log rc=$rc"; tail -12 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
