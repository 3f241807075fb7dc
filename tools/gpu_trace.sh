# Kernel trace of the default bench (steady-state overlap analysis with tools/timeline.py).
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace$T -o run --output-format csv -- python3 bench.py --steps 30 --warmup 4 --no-cpu-baseline --no-roofline > $O/trace$T.log 2>&1
echo EXIT $? >> $O/trace$T.log
