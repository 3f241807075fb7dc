# A/B of a frame-op kernel: the current library vs a variant (MDX_LIB_VARIANT)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/kbench.py --only "$2" > $O/kb_ab.log 2>&1 && \
MDX_LIB_VARIANT=$1 timeout -k 10 300 python tools/kbench.py --only "$2" >> $O/kb_ab.log 2>&1
echo EXIT $? >> $O/kb_ab.log
