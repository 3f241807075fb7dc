set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_model_gpu.py -x -q -k "mask_nms or extractor" > gpurun_out/t3.log 2>&1 && \
timeout -k 10 500 python bench.py --steps 10 --warmup 3 > gpurun_out/bench3.json 2> gpurun_out/bench3.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/prof3.log 2>&1
echo EXIT $? >> gpurun_out/t3.log
