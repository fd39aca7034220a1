cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_fused|900|python -m pytest tests/test_fused_kernels.py tests/test_federation_gpu.py -x -q" \
  "prof_lda|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lda -o run -- python bench.py --model LDA --steps 500 --warmup 50 --no-npmi" \
  "bench_lda|300|python bench.py --model LDA"
