cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_infer|400|python -u -m pytest tests/test_theta_infer.py -x -v --timeout 120 --timeout-method thread" \
  "bench_infer|300|python tools/bench_infer.py" \
  "counters_list|60|rocprofv3 -L" \
  "pmc_sq|180|rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_sq -o run -- python bench.py --steps 50 --warmup 10 --no-npmi" \
  "pmc_fetch|180|rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 50 --warmup 10 --no-npmi" \
  "pmc_write|180|rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 50 --warmup 10 --no-npmi"
