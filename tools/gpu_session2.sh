tools/gpu_steps.sh \
 "labeltests|400|python -u -m pytest tests/test_fused_kernels.py -q --timeout 120 --timeout-method thread -k 'label or bf16 or split'" \
 "gputests|700|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread"
