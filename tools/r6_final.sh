#!/bin/bash
# Round-6 final bench lines on the committed kernels (gpurun_out/final/bench_<name>.jsonl).
# usage: bash tools/r6_final.sh <part 1|2>.  Every run has its own limit; a failure stops.
set -o pipefail
o=gpurun_out/final
mkdir -p "$o"
run() {  # name limit args...
  local n="$1" t="$2"; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "$o/$n.log" 2>&1 || { echo "bench $n failed"; tail -5 "$o/$n.log"; exit 1; }
  grep '^{' "$o/$n.log" > "$o/bench_$n.jsonl"
  python -c "import json; r=json.loads(open('$o/bench_$n.jsonl').read().splitlines()[-1]); print('$n', r['config']['model'], r['dtype'], r['ms_per_step'], round(r['value']), r.get('npmi'))"
}
if [ "$1" = 1 ]; then
  run driver_default 200 --steps 20 --warmup 5
  run k50 240 --steps 2000 --warmup 200
  run c1 200 --clients 1 --steps 2000 --warmup 200 --no-npmi
  run multi17 240 --clients-per-gpu 17 --steps 300 --warmup 30 --no-npmi
  run sim8 240 --sim-clients 8 --steps 500 --warmup 50 --no-npmi
  run lda1 200 --model LDA --clients 1 --steps 2000 --warmup 200 --no-npmi
  run lb256 200 --clients 1 --batch 256 --steps 1000 --warmup 100 --no-npmi
  run lb512 200 --clients 1 --batch 512 --steps 500 --warmup 50 --no-npmi
elif [ "$1" = 3 ]; then
  run lb256 200 --clients 1 --batch 256 --steps 1000 --warmup 100 --no-npmi
  run lb256k200 240 --clients 1 --batch 256 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi
  run k300b64 200 --clients 1 --topics 300 --steps 1000 --warmup 100 --no-npmi
  run multi17 240 --clients-per-gpu 17 --steps 300 --warmup 30 --no-npmi
  run k50 240 --steps 2000 --warmup 200
  run driver_default 200 --steps 20 --warmup 5
else
  run b112 200 --clients 1 --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi
  run lb256k200 240 --clients 1 --batch 256 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi
  run k300b64 200 --clients 1 --topics 300 --steps 1000 --warmup 100 --no-npmi
  run ctm99 240 --clients 1 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi
  run ctm99bf 240 --clients 1 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi --dtype bf16
  run k200v100k8 300 --topics 200 --vocab 100000 --docs 1500 --steps 200 --warmup 20
  run ctm8_v99k 360 --family ctm --topics 100 --vocab 100000 --docs 1500 --steps 100 --warmup 10
fi
exit 0
