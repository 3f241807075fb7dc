# Per-layer conv timings, frame-op and ROIAlign microbenchmarks.
# Usage: bash tools/gpu_probe.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --dump-convs $O/convs$T.json > $O/benchp$T.json 2> $O/benchp$T.err && \
timeout -k 10 300 python tools/kbench.py > $O/kb$T.log 2>&1 && \
timeout -k 10 300 python tools/roibench.py > $O/roi$T.log 2>&1
echo EXIT $? >> $O/kb$T.log
