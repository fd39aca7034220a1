# strip forward: rolling prefetch (PF=2) vs the double-buffered 8-wave kernel (PF=1)
set -o pipefail
o=gpurun_out/g11; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_fused_kernels.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "strip or precomputed or oracle" > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_FWD_STRIP_PF=1 r b112_pf1.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
r b112_pf2.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
GFEDNTM_FWD_STRIP_PF=1 r k50_pf1.$i --steps 1000 --warmup 100 || exit $?
r k50_pf2.$i --steps 1000 --warmup 100 || exit $?
done
GFEDNTM_FWD_STRIP_PF=1 r b74_pf1 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
r b74_pf2 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
GFEDNTM_FWD_STRIP_PF=1 r ctm_pf1 --family ctm --topics 100 --steps 1000 --warmup 100 || exit $?
r ctm_pf2 --family ctm --topics 100 --steps 1000 --warmup 100 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/b112_kernels.md > /dev/null && head -8 $o/b112_kernels.md; find $o/kt -name "*.db" -delete
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
SQ2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES"
i=0; dirs=""
for pmc in "$SQ" "$SQ2" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc --output-format csv -d "$o/pmc$i" -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --no-npmi --steps 20 --warmup 5 > "$o/pmc$i.log" 2>&1 || exit $?
  f=$(find "$o/pmc$i" -name "*counter_collection.csv" | head -n 1); dirs="$dirs $(dirname "$f")"
done
python tools/pmc_summary.py "$o/counters.md" $dirs > /dev/null && head -6 $o/counters.md
python - $dirs > $o/counters_raw.md <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(lambda: collections.defaultdict(int))
for d in sys.argv[1:]:
    import glob
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:60]; c = r["Counter_Name"]
            agg[k][c] += float(r["Counter_Value"]); n[k][c] += 1
for k in agg:
    if "bwd_pipe" in k or "fwd_strip" in k or "win_sparse" in k:
        print("##", k)
        for c in sorted(agg[k]):
            print(f"  {c}: {agg[k][c] / max(1, n[k][c]):.0f}")
PY
cat $o/counters_raw.md | head -60
