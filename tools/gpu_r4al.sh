# round-4 call AL: the direct-store epilogue -- bit-equality tests (Winograd
# GEMMs, fp32 conv cases), then the fp32 loop A/B over modes 2 / 1 / 0.
# Usage: bash tools/gpu_r4al.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 200 --timeout-method thread -k "direct_epilogue" > $O/tde_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; grep FAILED $O/tde_$T.log | head -5; tail -1 $O/tde_$T.log
[ $rc -ne 0 ] && exit $rc
for d in 2 1 0 2 1 0; do
  timeout -k 10 300 python3 -u bench.py --steps 100 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_direct_epilogue=$d > $O/bde_${T}_$d.json 2>/dev/null || { echo "bench direct=$d failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bde_${T}_$d.json').read().strip().splitlines()[-1]); print('fp32 direct_epilogue=$d', d['value'])"
done
