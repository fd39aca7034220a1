# which multi-rank rehearsals time out in the xGMI wait? (each bounded; a clean CommError
# exit is recorded and the script goes on; a time limit / crash stops it)
set -o pipefail
o=gpurun_out/g16; mkdir -p $o
export GFEDNTM_REHEARSE_1GPU=1
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1; local rc=$?; echo "$n rc=$rc $(grep -o 'CommError.*' $o/$n.log | head -1 | cut -c1-120)"; python -c "
import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('  ', r['ms_per_step'], r.get('device_ms_per_step'), json.dumps(r.get('fedavg_attach')))" 2>/dev/null; [ $rc -le 1 ] || exit $rc; }
r k50x2 --gpus 2 --steps 200 --warmup 20
r k200old --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 60 --warmup 10
GFEDNTM_BWD_PRE=2 GFEDNTM_FWD_STRIP_PF=1 r k200oldk --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 60 --warmup 10
GFEDNTM_XGMI_INPLACE_MB=100000 r k200staged --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 60 --warmup 10
r k200v30 --gpus 2 --topics 200 --vocab 40000 --docs 600 --steps 60 --warmup 10
