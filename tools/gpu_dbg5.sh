set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/dbg_gn2.py > $O/dbggn2.log 2>&1
echo EXIT $? >> $O/dbggn2.log
