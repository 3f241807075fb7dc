# fp32-as-bf16-planes kernel: GPU tests, then the fp32 bench with the native
# kernels (0) and the x6 / x9 split kernels
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -k "fp32_split or winograd or roi_align" > $O/tsplit.log 2>&1 || { echo "EXIT tests $?" >> $O/tsplit.log; exit 1; }
for v in 6 9 0; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary --set mdx_conv_set_fp32_split=$v --dump-convs $O/convs_split$v.json > $O/split$v.json 2> $O/split$v.err || { echo "EXIT bench $v $?" >> $O/tsplit.log; exit 1; }
done
echo "EXIT 0" >> $O/tsplit.log
