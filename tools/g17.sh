# rehearsal wait timeouts: dump the all-reduce epochs / flags when one happens
set -o pipefail
o=gpurun_out/g17; mkdir -p $o
export GFEDNTM_REHEARSE_1GPU=1 GFEDNTM_COMM_DEBUG=1
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; grep -E "xGMI state|CommError:" $o/$n.log | cut -c1-600; [ $rc -le 1 ] || exit $rc; }
r v30a --gpus 2 --topics 200 --vocab 40000 --docs 600 --steps 60 --warmup 10
r v30b --gpus 2 --topics 200 --vocab 40000 --docs 600 --steps 60 --warmup 10
r v30c --gpus 2 --topics 200 --vocab 40000 --docs 600 --steps 60 --warmup 10
GFEDNTM_XGMI_INPLACE_MB=100000 r st112 --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 60 --warmup 10
r k50x3 --gpus 3 --steps 200 --warmup 20
