set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv2d and stream and fp32" > gpurun_out/s32_t1.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --set mdx_conv_set_stream1x1_f32=0 --dump-convs gpurun_out/convsS0.json > gpurun_out/benchS0.json 2>gpurun_out/benchS0.err && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --dump-convs gpurun_out/convsS1.json > gpurun_out/benchS1.json 2>gpurun_out/benchS1.err && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --set mdx_conv_set_stream1x1_f32=2 --dump-convs gpurun_out/convsS2.json > gpurun_out/benchS2.json 2>gpurun_out/benchS2.err
