# published-quality points: TSS/DSS at eta = 1.0 (reference eta sweep) or K' = 5 frozen topics
set -o pipefail
cfg="$1"; o=gpurun_out/quality_$cfg; mkdir -p $o
timeout -k 10 1100 python -u -m gfedntm_amd.experiments.dss_tss --config config/experiments/dss_tss_$cfg.json --out $o > $o/run.log 2>&1 || { tail -5 $o/run.log; exit 1; }
tail -3 $o/run.log; cat $o/results.csv
