# Round measurement: GPU tests, the default bench line (with the CPU baseline
# leg), then the rocprofv3 kernel trace of the same bench command shape.
# Usage: bash tools/gpu_full.sh TAG   (outputs under gpurun_out/)
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t$T.log 2>&1 && \
timeout -k 10 500 python bench.py > $O/bench$T.json 2> $O/bench$T.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof$T.log 2>&1
echo EXIT $? >> $O/t$T.log
