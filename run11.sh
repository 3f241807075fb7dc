set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/convbench.py > gpurun_out/cb11.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf11 -o f --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-overlap > gpurun_out/pmcf11.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw11 -o w --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-overlap > gpurun_out/pmcw11.log 2>&1
echo EXIT $? >> gpurun_out/cb11.log
