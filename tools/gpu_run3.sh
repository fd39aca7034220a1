set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_xgmi_allreduce.py -x -q > gpurun_out/pytest_xgmi.log 2>&1
echo "exit $?"
