#!/bin/bash
# round-4 first GPU session: new large-V fused tests, bf16 (16x16x32) decoder tests, the
# multi-client runner tests, the in-process FedAvg tests, smoke, then the CombinedTM
# V=99k profile (kernels + PMC)
tools/gpu_steps.sh \
  "largev|600|python -u -m pytest tests/test_fused_large_v.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bf16|300|python -u -m pytest tests/test_fused_kernels.py -k bf16 -x -v --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "dist|700|python -u -m pytest tests/test_distributed_gpu.py tests/test_federation_gpu.py tests/test_xgmi_allreduce.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
bash tools/profile_config.sh ctm99 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20
