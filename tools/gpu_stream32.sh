# fp32 streaming 1x1 kernel: conv tests, the default full-frame parity case,
# then the fp32 bench with the kernel on and off (per-launch conv timings)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_parity_full.py -x -q --timeout 300 --timeout-method thread -k "test_conv2d or 50-32-fp32-4-0 or overlapped" > $O/ts32.log 2>&1 || { echo "EXIT tests $?" >> $O/ts32.log; exit 1; }
for v in 1 0; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary --set mdx_conv_set_stream1x1_f32=$v --dump-convs $O/convs_s32_$v.json > $O/s32_$v.json 2> $O/s32_$v.err || { echo "EXIT bench $v $?" >> $O/ts32.log; exit 1; }
done
echo "EXIT 0" >> $O/ts32.log
