set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_fused_kernels.py -x -q -k "ctm" > gpurun_out/pytest_ctm.log 2>&1 && \
timeout -k 10 300 python bench.py --family ctm --topics 100 --steps 500 --warmup 50 > gpurun_out/bench_ctm_k100.log 2>&1 && \
timeout -k 10 300 python bench.py --family ctm --topics 50 --steps 500 --warmup 50 > gpurun_out/bench_ctm_k50.log 2>&1
echo "exit $?"
