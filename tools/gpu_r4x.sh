# round-4 call X: LDS / issue counters of the fp16 loop's kernels (serial steps).
# Usage: bash tools/gpu_r4x.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
B="--steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --no-overlap --no-extract-loop --dtype fp16"
C1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY"
timeout -s KILL 120 rocprofv3 --pmc $C1 --kernel-trace -d $O/sq_f16_$T -o c --output-format csv -- python3 bench.py $B > $O/sq_f16_$T.log 2>&1 || { echo "pmc failed"; tail -3 $O/sq_f16_$T.log; exit 1; }
python3 tools/pmc_sq.py $(find $O/sq_f16_$T -name '*counter_collection.csv') > $O/sqsum_f16_$T.log 2>&1; head -8 $O/sqsum_f16_$T.log | cut -c1-800
