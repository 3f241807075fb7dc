set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s32b_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/benchS32b.json 2>gpurun_out/benchS32b.err
