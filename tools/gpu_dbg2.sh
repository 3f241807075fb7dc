set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/dbg_pipe.py fp16 2 nolarge > $O/dbgp2.log 2>&1 && \
timeout -k 10 300 python tools/dbg_pipe.py fp16 2 nostream >> $O/dbgp2.log 2>&1 && \
timeout -k 10 300 python tools/dbg_pipe.py fp16 2 dma128 >> $O/dbgp2.log 2>&1 && \
timeout -k 10 300 python tools/dbg_pipe.py fp16 2 "" >> $O/dbgp2.log 2>&1
echo EXIT $? >> $O/dbgp2.log
