set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
DBG_FILL=0x5a GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/dbg_race.py fp16 20 same > $O/dbgfill.log 2>&1 && \
DBG_FILL=0x5a GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/dbg_race.py fp32 20 same >> $O/dbgfill.log 2>&1
echo EXIT $? >> $O/dbgfill.log
