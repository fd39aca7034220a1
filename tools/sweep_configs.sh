# round-3 sweep on the final kernels: every README configuration, one bench.py line each
set -o pipefail
o=gpurun_out/sweep; mkdir -p $o; export TMPDIR=/tmp
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'], r.get('npmi'))"; }
r k50 --steps 2000 --warmup 200 || exit $?
r lda --model LDA --steps 2000 --warmup 200 --no-npmi || exit $?
r k50bf --dtype bf16 --steps 2000 --warmup 200 --no-npmi || exit $?
r ctm --family ctm --topics 100 --steps 1000 --warmup 100 --no-npmi || exit $?
r zs --family zeroshot --topics 100 --steps 1000 --warmup 100 --no-npmi || exit $?
r b74 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi || exit $?
r b112 --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi || exit $?
r ctm99 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi || exit $?
r zs99 --family zeroshot --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi || exit $?
r sim8 --sim-clients 8 --steps 1000 --warmup 100 --no-npmi || exit $?
r sim16 --sim-clients 16 --steps 1000 --warmup 100 --no-npmi || exit $?
r drv --steps 20 --warmup 5 || exit $?
