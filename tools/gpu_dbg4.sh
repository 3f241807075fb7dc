set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
MDX_LIB_VARIANT=gnacq GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/dbg_race.py fp16 24 same > $O/dbgacq.log 2>&1
echo EXIT $? >> $O/dbgacq.log
