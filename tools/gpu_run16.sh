cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "bench_ctm|300|python bench.py --family ctm --topics 100 --steps 500 --warmup 50" \
  "bench_k200|400|python bench.py --topics 200 --vocab 100000 --steps 500 --warmup 50" \
  "prof_k200|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k200 -o run -- python bench.py --topics 200 --vocab 100000 --steps 200 --warmup 20 --no-npmi" \
  "prof_ctm|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ctm -o run -- python bench.py --family ctm --topics 100 --steps 200 --warmup 20 --no-npmi" \
  "rehearse2|300|GFEDNTM_REHEARSE_1GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 200 --warmup 20 --no-npmi"
