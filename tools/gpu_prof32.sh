# kernel trace + stats of the fp32 bench (serial steps), for per-kernel time
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof$T -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-roofline --no-overlap > $O/prof$T.log 2>&1
echo EXIT $? >> $O/prof$T.log
