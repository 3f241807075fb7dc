# RPN proposal path: its GPU tests, then A/B timing vs a variant library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread -k "rpn or nms or proposals" > $O/trpn.log 2>&1 && \
timeout -k 10 300 python tools/rpnbench.py 32 20 > $O/rpn_ab.log 2>&1 && \
MDX_LIB_VARIANT=$1 timeout -k 10 300 python tools/rpnbench.py 32 20 >> $O/rpn_ab.log 2>&1
echo EXIT $? >> $O/trpn.log
