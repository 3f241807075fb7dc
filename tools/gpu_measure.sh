# Round measurement: GPU tests, kernel trace (+ stats), PMC HBM traffic passes,
# then the default bench line (reads the PMC summary for roofline.traffic).
# Usage: bash tools/gpu_measure.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t$T.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof$T.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf$T -o f --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-overlap > $O/pmcf$T.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw$T -o w --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-overlap > $O/pmcw$T.log 2>&1 && \
python tools/pmc_summary.py $(echo $O/pmcf$T/*counter_collection.csv) $(echo $O/pmcw$T/*counter_collection.csv) 3 $O/pmc_kernels$T.json > $O/pmcs$T.log 2>&1 && \
cp $O/pmc_kernels$T.json profiles/r01_pmc_kernels.json && \
timeout -k 10 500 python bench.py > $O/bench$T.json 2> $O/bench$T.err
echo EXIT $? >> $O/t$T.log
