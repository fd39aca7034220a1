#!/bin/bash
# Runs GPU steps in order; a step that fails "softly" (exit 1/2: test failures,
# python errors) lets the next step run, anything else (timeout 124/137, abort
# 134, segfault 139, ...) stops the session.
# usage: tools/gpu_steps.sh "<name>|<timeout_s>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; t="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${t}s): $cmd"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then
    echo "=== hard failure ($rc): stopping"
    exit $rc
  fi
done
exit 0
