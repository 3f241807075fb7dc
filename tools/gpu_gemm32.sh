# fp32 conv GEMM microbenchmarks (+ SQ counters with PMC=1).  Usage: bash tools/gpu_gemm32.sh TAG [knob=value ...]
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
shift || true
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u tools/gemm32bench.py "$@" > $O/g32$T.log 2>&1 && \
if [ "${PMC:-0}" = "1" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $O/sqa$T -o a --output-format csv -- python3 tools/gemm32bench.py "$@" > $O/sqa$T.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $O/sqb$T -o b --output-format csv -- python3 tools/gemm32bench.py "$@" > $O/sqb$T.log 2>&1 && \
  python3 tools/pmc_sq.py $(find $O/sqa$T $O/sqb$T -name '*counter_collection.csv') > $O/sq$T.txt 2>&1
fi
echo EXIT $? >> $O/g32$T.log
