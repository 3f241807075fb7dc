# round-4 call Y: the single-stage k_conv_x3 -- tests, A/B in the
# split-plane loop, serial trace.  Usage: bash tools/gpu_r4y.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_model_gpu.py tests/test_parity_full.py -m gpu -q --timeout 400 --timeout-method thread -k "fp32_split or preplit or winograd or fp32-4-6 or fp32-6-6" > $O/tx3_$T.log 2>&1; rc=$?
echo "x3 tests rc=$rc"; grep -E "FAILED|Error" $O/tx3_$T.log | head -5; tail -1 $O/tx3_$T.log
[ $rc -ne 0 ] && exit $rc
for sb in 1 0 1 0; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 --set mdx_conv_set_x3_single_stage=$sb > $O/bsb_${T}_$sb.json 2>/dev/null || { echo "bench sb=$sb failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bsb_${T}_$sb.json').read().strip().splitlines()[-1]); print('x6 single_stage=$sb', d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/px3_$T -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-overlap --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/px3_$T.log 2>&1 || { echo "prof failed"; exit 1; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$O/px3_$T/run_kernel_stats.csv')))
x3=sum(float(r['TotalDurationNs']) for r in rows if 'k_conv_x3' in r['Name'])/1e6/23
print('k_conv_x3 ms per serial step', round(x3,3), 'TF', round(1.2609/x3*1e3,1), 'frac of 417', round(1.2609/x3*1e3/417,3))
PY
