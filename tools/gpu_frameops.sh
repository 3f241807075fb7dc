# frame-op GPU tests, then the frame-op kernel timings (tools/kbench.py)
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_frameops_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tf$T.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --only "${2:-moments}" > $O/kb$T.log 2>&1
echo EXIT $? >> $O/tf$T.log
