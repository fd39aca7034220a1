# multi-rank rehearsals on one GPU (protocol evidence; timings are not multi-GPU numbers):
# in-place vs staged xGMI all-reduce at K=200 / V=112k, and 2 ranks x 4 clients (hierarchical)
set -o pipefail
o=gpurun_out/g9; mkdir -p $o
export GFEDNTM_REHEARSE_1GPU=1 GFEDNTM_COMM_DEBUG=1
# two processes share the one GPU here: fewer hardware queues per process (the GPU
# scheduler descheduling one rank mid-kernel leaves its peer spinning to the wait bound)
export GPU_MAX_HW_QUEUES=2
r() { local n="$1"; shift; timeout -k 10 300 python bench.py "$@" --no-npmi > $o/$n.log 2>&1; local rc=$?; grep -E "xGMI state|CommError:" $o/$n.log | cut -c1-400; [ $rc -eq 0 ] || return $rc; python -c "
import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r.get('round_split_ms'), json.dumps(r.get('fedavg_attach')), r['config']['aggregation'][-60:])"; }
GFEDNTM_XGMI_INPLACE_MB=100000 r staged112 --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 || exit $?
r inplace112 --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 || exit $?
GFEDNTM_XGMI_INPLACE_MB=100000 r staged112b --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 || exit $?
r inplace112b --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 || exit $?
r multi2x4 --gpus 2 --clients-per-gpu 4 --steps 200 --warmup 20 || exit $?
# CombinedTM K=100 V=99k over 2 ranks: the ~400 MB shared state's attach (in place)
r ctm99x2 --gpus 2 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 40 --warmup 5 || exit $?
# per-rank kernel traces (each rank its own rocprofv3 process; no launcher re-exec):
# staged vs in-place xGMI all-reduce kernels at K=200 / V=112k
export TMPDIR=/tmp
for mode in staged inplace; do
  mb=8; [ $mode = staged ] && mb=100000
  port=$((29600 + RANDOM % 300))
  pids=""
  for rk in 0 1; do
    GFEDNTM_XGMI_INPLACE_MB=$mb RANK=$rk LOCAL_RANK=$rk WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt_${mode}_r$rk -o run -- python bench.py --gpus 2 --topics 200 --vocab 150000 --docs 1500 --steps 60 --warmup 10 --no-npmi > $o/kt_${mode}_r$rk.log 2>&1 &
    pids="$pids $!"
  done
  for p in $pids; do wait $p || exit 1; done
  db=$(find $o/kt_${mode}_r0 -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/kernels_${mode}_r0.md > /dev/null && grep -E "xgmi|kernel \|" $o/kernels_${mode}_r0.md; find $o -name "*.db" -delete
done
