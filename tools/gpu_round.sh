# One GPU round: tests, frame-op and conv microbenchmarks, bench line, kernel
# trace, and (with PMC=1) HBM traffic counters.  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $O/t$T.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py > $O/kb$T.log 2>&1 && \
timeout -k 10 300 python tools/convbench.py > $O/cb$T.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-convs $O/convs$T.json > $O/bench$T.json 2> $O/bench$T.err && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-overlap > $O/bench${T}_serial.json 2>> $O/bench$T.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof$T -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-overlap > $O/prof$T.log 2>&1 && \
if [ "${PMC:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf$T -o f --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-overlap > $O/pmcf$T.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw$T -o w --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-overlap > $O/pmcw$T.log 2>&1
fi
echo EXIT $? >> $O/t$T.log
