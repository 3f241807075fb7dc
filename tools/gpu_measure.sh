# Round measurement: GPU tests (optionally a -k subset), kernel trace + stats of
# the fp32 headline bench, PMC HBM traffic passes (FETCH_SIZE, WRITE_SIZE in
# separate runs), then the default bench line (reads the PMC summary for
# roofline.traffic).  Usage: bash tools/gpu_measure.sh TAG ['-k expr']
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
if [ -n "${2:-}" ]; then KA=(-k "$2"); else KA=(); fi
B=(--no-cpu-baseline --no-secondary)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > $O/t$T.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 "${B[@]}" --no-overlap > $O/prof$T.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmcf$T -o f --output-format csv -- python3 bench.py --steps 2 --warmup 1 "${B[@]}" --no-roofline --no-overlap > $O/pmcf$T.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmcw$T -o w --output-format csv -- python3 bench.py --steps 2 --warmup 1 "${B[@]}" --no-roofline --no-overlap > $O/pmcw$T.log 2>&1 && \
python tools/pmc_summary.py $(echo $O/pmcf$T/*counter_collection.csv) $(echo $O/pmcw$T/*counter_collection.csv) 3 $O/pmc_kernels$T.json > $O/pmcs$T.log 2>&1 && \
cp $O/pmc_kernels$T.json profiles/r02_pmc_kernels_fp32.json && \
timeout -k 10 600 python bench.py > $O/bench$T.json 2> $O/bench$T.err
echo EXIT $? >> $O/t$T.log
