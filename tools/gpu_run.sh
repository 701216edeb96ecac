#!/bin/bash
# Runs GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
# Usage: tools/gpu_run.sh "name|seconds|command" ...
# A step that ends with 0 or 1 (test failures, assertion errors) lets the next one start; a fault, abort,
# segfault, time limit or a HIP error anywhere in the step's log stops the whole sequence.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  if grep -qiE "illegal memory access|memory access fault|HIP error|hipErrorLaunchFailure|GPU Hang" "gpurun_out/$name.log"; then
    echo "stopping after $name (GPU fault reported in its log)"
    exit 3
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
done
