# The round's measurement recipe on one GPU: the driver's bench command, a
# kernel trace of the default (pipelined) loop and of serial steps, and the
# HBM counters (FETCH_SIZE / WRITE_SIZE in separate passes) of serial steps,
# summarised per kernel.  Usage: bash tools/gpu_profile.sh TAG [bench args]
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
shift || true
O=gpurun_out
mkdir -p $O
B="--no-cpu-baseline --no-secondary"
timeout -k 10 600 python3 -u bench.py "$@" > $O/bench$T.json 2> $O/bench$T.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 $B --no-roofline "$@" > $O/prof$T.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profs$T -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 $B --no-roofline --no-overlap "$@" > $O/profs$T.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf$T -o f --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B --no-roofline --no-overlap "$@" > $O/pmcf$T.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw$T -o w --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B --no-roofline --no-overlap "$@" > $O/pmcw$T.log 2>&1 && \
python3 tools/pmc_summary.py $(find $O/pmcf$T -name '*counter_collection.csv' | head -1) $(find $O/pmcw$T -name '*counter_collection.csv' | head -1) 3 $O/pmc$T.json > $O/pmcsum$T.log 2>&1
echo EXIT $? >> $O/bench$T.err
