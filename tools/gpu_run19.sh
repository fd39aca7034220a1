cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --family ctm --topics 100 --steps 50 --warmup 10 --no-npmi"
bash tools/gpu_steps.sh \
  "pmc_sq|180|rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_ctm_sq -o run -- $B" \
  "pmc_fetch|180|rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d gpurun_out/pmc_ctm_fetch -o run -- $B" \
  "pmc_tcp|180|rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_ctm_tcp -o run -- $B"
