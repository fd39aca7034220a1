cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "prof_lda|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lda -o run -- python bench.py --model LDA --steps 500 --warmup 50 --no-npmi" \
  "prof_ctm|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ctm -o run -- python bench.py --family ctm --topics 100 --steps 500 --warmup 50 --no-npmi" \
  "prof_k200|500|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k200 -o run -- python bench.py --topics 200 --vocab 100000 --steps 300 --warmup 30 --no-npmi"
