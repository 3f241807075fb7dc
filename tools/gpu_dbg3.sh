set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/dbg_fill.py > $O/dbgf.log 2>&1
echo EXIT $? >> $O/dbgf.log
