# Adam RMW bandwidth by access pattern and row alignment (tools/micro/adam_bw.py)
set -o pipefail
o=gpurun_out/g14; mkdir -p $o
ADAM_BW_PATTERNS=1,3 ADAM_BW_V=112000 timeout -k 10 120 python tools/micro/adam_bw.py > $o/aligned.jsonl 2>&1 || exit $?
ADAM_BW_PATTERNS=1,3 ADAM_BW_V=112027 timeout -k 10 120 python tools/micro/adam_bw.py > $o/unaligned.jsonl 2>&1 || exit $?
cat $o/aligned.jsonl $o/unaligned.jsonl | grep pattern
