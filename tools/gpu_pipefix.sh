# inpaint tests, then the pipelined fp32 loop (300 steps) that faulted before the k_inp_setup flag fix
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "inpaint or extract or pipeline or overlapped" > gpurun_out/pf_tests.log 2>&1 && \
AMD_LOG_LEVEL=1 timeout -k 10 300 python bench.py --pipeline --model-streams 1 --steps 300 --warmup 4 --no-cpu-baseline --no-secondary --no-roofline > gpurun_out/benchPF1.json 2>gpurun_out/benchPF1.err && \
AMD_LOG_LEVEL=1 timeout -k 10 300 python bench.py --pipeline --steps 300 --warmup 4 --no-cpu-baseline --no-secondary --no-roofline > gpurun_out/benchPF2.json 2>gpurun_out/benchPF2.err
