# multi-rank rehearsals on one GPU (protocol evidence; timings are not multi-GPU numbers):
# in-place vs staged xGMI all-reduce at K=200 / V=112k, and 2 ranks x 4 clients (hierarchical)
set -o pipefail
o=gpurun_out/g9; mkdir -p $o
export GFEDNTM_REHEARSE_1GPU=1
r() { local n="$1"; shift; timeout -k 10 300 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "
import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r.get('round_split_ms'), json.dumps(r.get('fedavg_attach')), r['config']['aggregation'][-60:])"; }
GFEDNTM_XGMI_INPLACE_MB=100000 r staged112 --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 || exit $?
r inplace112 --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 || exit $?
GFEDNTM_XGMI_INPLACE_MB=100000 r staged112b --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 || exit $?
r inplace112b --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 || exit $?
r multi2x4 --gpus 2 --clients-per-gpu 4 --steps 200 --warmup 20 || exit $?
