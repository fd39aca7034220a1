# all-reduce kernel without LDS: CombinedTM V=99k 2-rank rehearsal (the ~400 MB shared
# state attach), K=50 x2, distributed GPU tests
set -o pipefail
o=gpurun_out/g24; mkdir -p $o
export GFEDNTM_REHEARSE_1GPU=1 GFEDNTM_COMM_DEBUG=1 GPU_MAX_HW_QUEUES=2
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; grep -E "xGMI state|CommError:" $o/$n.log | cut -c1-300; [ $rc -eq 0 ] || return $rc; python -c "
import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('  ', r['ms_per_step'], r.get('device_ms_per_step'), json.dumps(r.get('fedavg_attach')), r['config']['parallelism'], r.get('n_gpus'), r.get('ranks'), r.get('physical_gpus'))"; }
r ctm99x2 --gpus 2 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 30 --warmup 5 || exit $?
r k50x2 --gpus 2 --steps 300 --warmup 20 || exit $?
unset GFEDNTM_COMM_DEBUG GPU_MAX_HW_QUEUES GFEDNTM_REHEARSE_1GPU
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/dist_tests.log 2>&1; rc=$?; tail -2 $o/dist_tests.log; exit $rc
