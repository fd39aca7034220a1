cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_ctm|600|python -u -m pytest tests/test_fused_kernels.py tests/test_theta_infer.py tests/test_models.py -x -q --timeout 120 --timeout-method thread -k 'ctm or zeroshot or theta or fit'" \
  "pytest_all|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
