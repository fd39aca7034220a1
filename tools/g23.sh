# multi-rank rehearsals on one GPU after the flag write-back fix (protocol evidence; timings
# are not multi-GPU numbers): K=50 x2 / x3 ranks, K=200 V=112k in-place, 2 ranks x 4 clients,
# CombinedTM V=99k x2 (the ~400 MB shared state's attach)
set -o pipefail
o=gpurun_out/g23; mkdir -p $o
export GFEDNTM_REHEARSE_1GPU=1 GFEDNTM_COMM_DEBUG=1 GPU_MAX_HW_QUEUES=2
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; grep -E "xGMI state|CommError:" $o/$n.log | cut -c1-300; [ $rc -eq 0 ] || return $rc; python -c "
import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('  ', r['ms_per_step'], r.get('device_ms_per_step'), json.dumps(r.get('fedavg_attach')), r['config']['parallelism'], r.get('n_gpus'), r.get('ranks'), r.get('physical_gpus'))"; }
r k50x2 --gpus 2 --steps 300 --warmup 20 || exit $?
r k50x3 --gpus 3 --steps 300 --warmup 20 || exit $?
r k50x2b --gpus 2 --steps 300 --warmup 20 || exit $?
r inplace112 --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 60 --warmup 10 || exit $?
r multi2x4 --gpus 2 --clients-per-gpu 4 --steps 200 --warmup 20 || exit $?
r ctm99x2 --gpus 2 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 30 --warmup 5 || exit $?
