cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --family ctm --topics 100 --steps 50 --warmup 10 --no-npmi"
bash tools/gpu_steps.sh \
  "pmc_sq|180|rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F32 --output-format csv -d gpurun_out/pmc_ctm2_sq -o run -- $B" \
  "pmc_mem|180|rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TA_BUSY_avr GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_ctm2_mem -o run -- $B"
