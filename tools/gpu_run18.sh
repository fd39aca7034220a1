cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_ctm|600|python -u -m pytest tests/test_fused_kernels.py -x -q --timeout 120 --timeout-method thread -k ctm" \
  "pytest_all|600|python -u -m pytest tests/test_fused_kernels.py tests/test_federation_gpu.py tests/test_theta_infer.py -x -q --timeout 120 --timeout-method thread" \
  "bench_ctm|300|python bench.py --family ctm --topics 100" \
  "prof_ctm|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ctm -o run -- python bench.py --family ctm --topics 100 --steps 200 --warmup 20 --no-npmi"
