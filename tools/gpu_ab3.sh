# per-layer A/B of fp32 dispatch knobs (bench --dump-convs)
set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary"
timeout -k 10 200 $B --dump-convs gpurun_out/convsA0.json > gpurun_out/benchA0.json 2>gpurun_out/benchA0.err && \
timeout -k 10 200 $B --winograd-min-cin 64 --dump-convs gpurun_out/convsA1.json > gpurun_out/benchA1.json 2>gpurun_out/benchA1.err && \
timeout -k 10 200 $B --set mdx_conv_set_narrow_kmax=64 --dump-convs gpurun_out/convsA2.json > gpurun_out/benchA2.json 2>gpurun_out/benchA2.err
