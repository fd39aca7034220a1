cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "bench_infer|300|python tools/bench_infer.py" \
  "prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python bench.py --steps 500 --warmup 50 --no-npmi" \
  "pmc_sq|180|rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc2_sq -o run -- python bench.py --steps 50 --warmup 10 --no-npmi" \
  "pmc_mfma|180|rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc2_mfma -o run -- python bench.py --steps 50 --warmup 10 --no-npmi" \
  "pmc_infer|180|rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc2_infer -o run -- python tools/bench_infer.py --docs 100000 --reps 2 --no-reference"
