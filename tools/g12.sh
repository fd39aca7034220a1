# pipelined backward with b128 operand reads: oracle tests + interleaved A/B vs bwd_pre=2
set -o pipefail
o=gpurun_out/g12; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_fused_kernels.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "precomputed or beta_split or fused_update or oracle" > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_BWD_PRE=2 r b112_pre2.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
r b112_pre3.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
done
GFEDNTM_BWD_PRE=2 r b74_pre2 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
r b74_pre3 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/b112_kernels.md > /dev/null && head -8 $o/b112_kernels.md; find $o/kt -name "*.db" -delete
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
i=0; dirs=""
for pmc in "$SQ" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc --output-format csv -d "$o/pmc$i" -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --no-npmi --steps 20 --warmup 5 > "$o/pmc$i.log" 2>&1 || exit $?
  f=$(find "$o/pmc$i" -name "*counter_collection.csv" | head -n 1); dirs="$dirs $(dirname "$f")"
done
python tools/pmc_summary.py "$o/counters.md" $dirs > /dev/null && head -5 $o/counters.md
