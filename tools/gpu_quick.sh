# Quick check: selected GPU tests (-k expr), then the bench line and the ROI microbenchmark.
# Usage: bash tools/gpu_quick.sh TAG 'pytest -k expression'
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
K=${2:-roi}
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread > $O/q$T.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/benchq$T.json 2> $O/benchq$T.err && \
timeout -k 10 300 python tools/roibench.py > $O/roiq$T.log 2>&1
echo EXIT $? >> $O/q$T.log
