# round-4 call K: k_conv_x3 with the weights pre-split into planes -- the
# split-plane parity cases, then the split-plane loop and its kernel trace.
# Usage: bash tools/gpu_r4k.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_parity_full.py tests/test_model_gpu.py -m gpu -v --timeout 400 --timeout-method thread -k "fp32-4-6 or fp32-6-6 or fp32_split or winograd_planes" > $O/tx3_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/tx3_$T.log | tail -30; tail -1 $O/tx3_$T.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/bx3_${T}_$i.json 2>/dev/null || { echo "bench x3 failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bx3_${T}_$i.json').read().strip().splitlines()[-1]); print('x6 loop', d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/px3_$T -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-overlap --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/px3_$T.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof ok"
