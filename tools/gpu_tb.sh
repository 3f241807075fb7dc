# GPU tests (all, or -k expression) then the default bench line.
# Usage: bash tools/gpu_tb.sh TAG ['pytest -k expr'] [bench args]
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
K=${2:-}
O=gpurun_out
mkdir -p $O
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > $O/t$T.log 2>&1 && \
timeout -k 10 600 python bench.py ${@:3} > $O/bench$T.json 2> $O/bench$T.err
echo EXIT $? >> $O/t$T.log
