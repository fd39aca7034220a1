#!/bin/bash
# Round-end evidence on the committed kernels: GPU tests, smoke, and one bench.py line
# per BASELINE config (gpurun_out/final/*.jsonl).  Every GPU step has its own limit; the
# first failure stops the script.
set -o pipefail
o=gpurun_out/final
mkdir -p "$o"
run() {  # name limit args...
  local n="$1" t="$2"; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "$o/$n.log" 2>&1 || { echo "bench $n failed"; exit 1; }
  grep '^{' "$o/$n.log" > "$o/bench_$n.jsonl"
  python -c "import json,sys; r=json.loads(open('$o/bench_$n.jsonl').read().splitlines()[-1]); print('$n', r['config']['model'], r['dtype'], r['ms_per_step'], r['value'])"
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
    -p no:cacheprovider > "$o/gpu_tests.log" 2>&1 || { tail -30 "$o/gpu_tests.log"; exit 1; }
tail -n 1 "$o/gpu_tests.log" | tee "$o/gpu_tests.txt"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -n 1 || exit 1
run driver_default 200 --steps 20 --warmup 5
run k50 200 --steps 2000 --warmup 200
run k50bf 200 --steps 2000 --warmup 200 --dtype bf16 --no-npmi
run lda 200 --model LDA --steps 2000 --warmup 200 --no-npmi
run ctm 200 --family ctm --topics 100 --steps 1000 --warmup 100 --no-npmi
run zs 200 --family zeroshot --topics 100 --steps 1000 --warmup 100 --no-npmi
run b74 200 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi
run b112 200 --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi
run sim8 240 --sim-clients 8 --steps 500 --warmup 50 --no-npmi
run sim8lda 240 --sim-clients 8 --model LDA --steps 500 --warmup 50 --no-npmi
run b112bf 200 --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi --dtype bf16
run ctm99 240 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi
run zs99 240 --family zeroshot --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi
run multi17 240 --clients-per-gpu 17 --steps 300 --warmup 30 --no-npmi
