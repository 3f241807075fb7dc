set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/dbg_pipe.py fp16 2 > $O/dbgp.log 2>&1 && \
timeout -k 10 300 python tools/dbg_pipe.py fp16 1 >> $O/dbgp.log 2>&1 && \
timeout -k 10 300 python tools/dbg_pipe.py fp32 2 >> $O/dbgp.log 2>&1 && \
timeout -k 10 300 python tools/dbg_pipe.py fp16 2 >> $O/dbgp.log 2>&1
echo EXIT $? >> $O/dbgp.log
