cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_fused|600|python -u -m pytest tests/test_fused_kernels.py tests/test_federation_gpu.py tests/test_xgmi_allreduce.py -x -q --timeout 120 --timeout-method thread" \
  "bench_lda|300|python bench.py --model LDA" \
  "prof_lda|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lda -o run -- python bench.py --model LDA --steps 500 --warmup 50 --no-npmi"
