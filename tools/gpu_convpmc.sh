# PMC counters of chosen convbench shapes (default: fpn output p2 + fc1), one pass per group.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
S=${1:-5,7}
T=${2:-x}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/cpa$T -o a --output-format csv -- python3 tools/convbench.py $S > $O/cpa$T.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace -d $O/cpb$T -o b --output-format csv -- python3 tools/convbench.py $S > $O/cpb$T.log 2>&1
echo EXIT $? >> $O/cpa$T.log
