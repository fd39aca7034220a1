#!/bin/bash
# Kernel-trace A/B of an environment switch on one bench.py configuration.
# usage: tools/kt_ab.sh <VAR> <valA> <valB> <bench.py args...>
# Writes gpurun_out/kt_<VAR>_<val>/kernels.md per value.
set -o pipefail
var="$1"; a="$2"; b="$3"; shift 3
export TMPDIR=/tmp
for val in "$a" "$b"; do
  out="gpurun_out/kt_${var}_${val}"
  mkdir -p "$out"
  echo "=== $var=$val"
  export "$var=$val"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/kt" -o run \
      -- python bench.py "$@" --no-npmi > "$out/kt.log" 2>&1 || exit $?
  db=$(find "$out/kt" -name "*.db" | head -n 1)
  python tools/prof_summary.py "$db" "$out/kernels.md" > /dev/null || exit $?
  head -n 8 "$out/kernels.md"
  rm -rf "$out/kt"
done
