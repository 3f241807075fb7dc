# GPU suite + default bench line on the current tree.  Usage: bash tools/gpu_suite.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t$T.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $O/bench$T.json 2> $O/bench$T.err
echo EXIT $? >> $O/t$T.log
