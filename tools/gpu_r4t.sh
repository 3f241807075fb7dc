# round-4 call T: LDS and issue counters of the split-plane kernel and of
# the fp32 headline's GEMM (serial steps, separate passes, no trace domains).
# Usage: bash tools/gpu_r4t.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
B="--steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --no-overlap --no-extract-loop"
C1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY"
for cfg in x6 f32; do
  if [ $cfg = x6 ]; then X="--set mdx_conv_set_fp32_split=6"; else X=""; fi
  timeout -s KILL 120 rocprofv3 --pmc $C1 --kernel-trace -d $O/sq_${cfg}_$T -o c --output-format csv -- python3 bench.py $B $X > $O/sq_${cfg}_$T.log 2>&1 || { echo "pmc $cfg failed"; tail -3 $O/sq_${cfg}_$T.log; exit 1; }
  python3 tools/pmc_sq.py $(find $O/sq_${cfg}_$T -name '*counter_collection.csv') > $O/sqsum_${cfg}_$T.log 2>&1 || { echo "summary failed"; exit 1; }
  echo "== $cfg"; head -4 $O/sqsum_${cfg}_$T.log | cut -c1-700
done
