set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_xgmi_allreduce.py -x -q > gpurun_out/pytest_xgmi.log 2>&1 && \
GFEDNTM_REHEARSE_1GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 300 --warmup 30 > gpurun_out/bench_rehearse2.log 2>&1
echo "exit $?"
