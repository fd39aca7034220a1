# which warm-up round times out, and how far apart the ranks are
set -o pipefail
o=gpurun_out/g18; mkdir -p $o
export GFEDNTM_REHEARSE_1GPU=1 GFEDNTM_COMM_DEBUG=1
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; grep -E "round [0-9]+: enq|CommError:" $o/$n.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
r v30a --gpus 2 --topics 200 --vocab 40000 --docs 600 --steps 30 --warmup 10
r v30b --gpus 2 --topics 200 --vocab 40000 --docs 600 --steps 30 --warmup 10
