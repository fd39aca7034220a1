cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_x|600|python -u -m pytest tests/test_xgmi_allreduce.py tests/test_federation_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "bench2|300|GFEDNTM_REHEARSE_1GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 300 --warmup 30 --no-npmi" \
  "bench4|300|GFEDNTM_REHEARSE_1GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 200 --warmup 20 --no-npmi" \
  "bench1|300|python bench.py --steps 500 --warmup 50"
