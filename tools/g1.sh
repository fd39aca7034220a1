set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g1/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/g1/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/g1/b_default.log 2>&1 || exit $?
tail -1 gpurun_out/g1/b_default.log
timeout -k 10 200 python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi > gpurun_out/g1/b112.log 2>&1 || exit $?
tail -1 gpurun_out/g1/b112.log
