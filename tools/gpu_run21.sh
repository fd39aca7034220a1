cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_fused|600|python -u -m pytest tests/test_fused_kernels.py tests/test_federation_gpu.py tests/test_grad_aggregation.py -x -q --timeout 120 --timeout-method thread" \
  "bench|300|python bench.py" \
  "bench_k200|300|python bench.py --topics 200 --vocab 100000 --steps 500 --warmup 50" \
  "prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k50 -o run -- python bench.py --steps 500 --warmup 50 --no-npmi"
