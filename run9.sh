set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t9.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py > gpurun_out/kb9.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-convs gpurun_out/convs9.json > gpurun_out/bench9.json 2> gpurun_out/bench9.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/prof9.log 2>&1 && \
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters9.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --kernel-trace -d gpurun_out/pmc9 -o pmc --output-format csv -- python3 tools/kbench.py --only clean --reps 2 > gpurun_out/pmc9.log 2>&1
echo EXIT $? >> gpurun_out/t9.log
