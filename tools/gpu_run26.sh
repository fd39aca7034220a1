cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "ctm_r1|300|python bench.py --family ctm --topics 100 --no-npmi" \
  "ctm_r2|300|GFEDNTM_CTX_BWD_ROUNDS=2 python bench.py --family ctm --topics 100 --no-npmi" \
  "ctm_r3|300|GFEDNTM_CTX_BWD_ROUNDS=3 python bench.py --family ctm --topics 100 --no-npmi" \
  "prof_r2|300|GFEDNTM_CTX_BWD_ROUNDS=2 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ctm_r2 -o run -- python bench.py --family ctm --topics 100 --steps 200 --warmup 20 --no-npmi"
