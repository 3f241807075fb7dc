# fp32 probe: bench line at fp32 (per-conv dump) + kernel trace of the fp32 path.
# Usage: bash tools/gpu_fp32probe.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python bench.py --dtype fp32 --steps 4 --warmup 2 --no-cpu-baseline --dump-convs $O/convs32$T.json > $O/bench32$T.json 2> $O/bench32$T.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof32$T -o run --output-format csv -- python3 bench.py --dtype fp32 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-overlap > $O/prof32$T.log 2>&1
echo EXIT $? >> $O/bench32$T.err
