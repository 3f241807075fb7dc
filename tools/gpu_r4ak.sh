# round-4 call AK: Winograd GEMMs storing straight from the MFMA layout --
# bit-equality tests, then the fp32 loop A/B.  Usage: bash tools/gpu_r4ak.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 200 --timeout-method thread -k "winograd_direct or (test_conv3x3_winograd and not planes)" > $O/twd_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; grep FAILED $O/twd_$T.log | head -5; tail -1 $O/twd_$T.log
[ $rc -ne 0 ] && exit $rc
for d in 1 0 1 0; do
  timeout -k 10 300 python3 -u bench.py --steps 100 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_wino_direct=$d > $O/bwd_${T}_$d.json 2>/dev/null || { echo "bench direct=$d failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bwd_${T}_$d.json').read().strip().splitlines()[-1]); print('fp32 wino_direct=$d', d['value'])"
done
