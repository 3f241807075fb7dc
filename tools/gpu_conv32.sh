# conv GPU tests, then fp32 bench lines (per-layer conv timings) for the fp32
# conv policies given as extra args (mdx_conv_set_dma_f32 modes).
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
shift
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread -k "conv" > $O/tc$T.log 2>&1 || { echo "EXIT $?" >> $O/tc$T.log; exit 1; }
for m in "$@"; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary --dma-f32 $m --dump-convs $O/convs$T-$m.json > $O/bench$T-$m.json 2> $O/bench$T-$m.err || { echo "EXIT $? bench $m" >> $O/tc$T.log; exit 1; }
done
echo EXIT 0 >> $O/tc$T.log
