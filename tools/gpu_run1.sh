set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 && \
timeout -k 10 300 python bench.py --model LDA > gpurun_out/bench_lda.log 2>&1 && \
timeout -k 10 400 python bench.py --topics 200 --vocab 100000 --steps 500 --warmup 50 > gpurun_out/bench_k200_v100k.log 2>&1
echo "exit $?"
