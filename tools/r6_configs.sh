#!/bin/bash
# Round 6: 8-client (and the centralized bf16) lines of every BASELINE.json configuration on
# one MI355X, with NPMI / client-1 TSS / DSS, and a kernel table per config.
# usage: bash tools/r6_configs.sh [bench|kt]   ->  gpurun_out/r6/<name>.jsonl | kt_<name>/
mode="${1:-bench}"
out=gpurun_out/r6
mkdir -p "$out"
export TMPDIR=/tmp
run() {
  name="$1"; shift
  if [ "$mode" = bench ]; then
    echo "=== $name: $*"
    timeout -k 10 420 python bench.py "$@" > "$out/$name.jsonl" 2> "$out/$name.err"
    rc=$?
    tail -n 1 "$out/$name.jsonl" | cut -c1-220
  else
    timeout -k 10 300 bash tools/kt.sh "$name" "$@" --steps 200 --warmup 20 > "$out/kt_$name.log" 2>&1
    rc=$?
    head -n 8 "gpurun_out/kt_$name/kernels.md"
  fi
  echo "=== $name rc=$rc"
  case $rc in 0|1|2) ;; *) echo "hard failure: stop"; exit $rc ;; esac
}
run lda8 --model LDA
run ctm8_v5k --family ctm --topics 100
run ctm8_v99k --family ctm --topics 100 --vocab 100000 --docs 1500
run ctm8_v99k_bf16 --family ctm --topics 100 --vocab 100000 --docs 1500 --dtype bf16
run k200v100k8 --topics 200 --vocab 100000 --docs 1500
run bf16_8 --dtype bf16
run bf16_c1 --dtype bf16 --clients 1
exit 0
