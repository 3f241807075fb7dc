# round-4 call V: k_conv_x3 with the swizzled LDS layout -- its tests, the
# split-plane loop, its LDS counters and serial kernel trace.
# Usage: bash tools/gpu_r4v.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_model_gpu.py tests/test_parity_full.py -m gpu -q --timeout 400 --timeout-method thread -k "fp32_split or preplit or winograd or fp32-4-6 or fp32-6-6" > $O/tx3_$T.log 2>&1; rc=$?
echo "x3 tests rc=$rc"; grep -E "FAILED" $O/tx3_$T.log | head; tail -1 $O/tx3_$T.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/bx3_${T}_$i.json 2>/dev/null || { echo "bench x3 failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bx3_${T}_$i.json').read().strip().splitlines()[-1]); print('x6 loop', d['value'])"
done
B="--steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --no-overlap --no-extract-loop"
C1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY"
timeout -s KILL 120 rocprofv3 --pmc $C1 --kernel-trace -d $O/sq_x6_$T -o c --output-format csv -- python3 bench.py $B --set mdx_conv_set_fp32_split=6 > $O/sq_x6_$T.log 2>&1 || { echo "pmc failed"; exit 1; }
python3 tools/pmc_sq.py $(find $O/sq_x6_$T -name '*counter_collection.csv') > $O/sqsum_x6_$T.log 2>&1; head -2 $O/sqsum_x6_$T.log | cut -c1-900
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/px3_$T -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-overlap --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/px3_$T.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof ok"
