set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/dbg_arena.py fp16 > $O/dbga.log 2>&1
echo EXIT $? >> $O/dbga.log
