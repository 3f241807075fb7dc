set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t10.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py > gpurun_out/kb10.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-convs gpurun_out/convs10.json > gpurun_out/bench10.json 2> gpurun_out/bench10.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof10 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/prof10.log 2>&1
echo EXIT $? >> gpurun_out/t10.log
