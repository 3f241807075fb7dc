# long pipelined runs after the k_inp_setup fix (fp32 x2, fp16, split-plane), then the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 1000 --warmup 4 --no-cpu-baseline --no-secondary --no-roofline"
timeout -k 10 200 $B > gpurun_out/benchL1.json 2>gpurun_out/benchL1.err && \
timeout -k 10 200 $B > gpurun_out/benchL2.json 2>gpurun_out/benchL2.err && \
timeout -k 10 200 $B --dtype fp16 > gpurun_out/benchL3.json 2>gpurun_out/benchL3.err && \
timeout -k 10 200 $B --set mdx_conv_set_fp32_split=6 > gpurun_out/benchL4.json 2>gpurun_out/benchL4.err && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/benchDRV2.json 2>gpurun_out/benchDRV2.err
