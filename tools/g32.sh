# batched clients: 8-wave strip forward + 8-wave win_update tile shape when all clients' tiles
# exceed two rounds; test + interleaved A/B (env switches off each choice)
set -o pipefail
o=gpurun_out/g32; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_federation_gpu.py -q -x -k "batched" --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_BATCH_STRIP_PF=0 GFEDNTM_BATCH_WIN8=0 r sim8_off.$i --sim-clients 8 --steps 1000 --warmup 100 || exit $?
GFEDNTM_BATCH_WIN8=0 r sim8_pf.$i --sim-clients 8 --steps 1000 --warmup 100 || exit $?
r sim8_both.$i --sim-clients 8 --steps 1000 --warmup 100 || exit $?
done
GFEDNTM_BATCH_STRIP_PF=0 GFEDNTM_BATCH_WIN8=0 r sim16_off --sim-clients 16 --steps 1000 --warmup 100 || exit $?
r sim16_both --sim-clients 16 --steps 1000 --warmup 100 || exit $?
