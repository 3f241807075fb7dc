# round-4 call N: the conv kernel tests, the split-plane loop (pre-split
# weights, pointwise instance) and its serial kernel trace, split-plane
# pipelined determinism, extract loop 2 vs 3 model streams.
# Usage: bash tools/gpu_r4n.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 200 --timeout-method thread -k "test_conv2d" > $O/tconv_$T.log 2>&1; rc=$?
echo "conv tests rc=$rc"; tail -1 $O/tconv_$T.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/bx3_${T}_$i.json 2>/dev/null || { echo "bench x3 failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bx3_${T}_$i.json').read().strip().splitlines()[-1]); print('x6 loop', d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/px3_$T -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-overlap --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/px3_$T.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof ok"
bash tools/gpu_r4m.sh $T
