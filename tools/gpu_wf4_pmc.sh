#!/bin/bash
# SQ counters of the fused Winograd kernel on one layer shape (two passes,
# each under its own kill timer), summarised by tools/sq_summary.py.
# Usage (GPU box): bash tools/gpu_wf4_pmc.sh TAG LAYER
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
T=$1; L=${2:-fpn_p2}
O=gpurun_out
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/wfa$T -o a --output-format csv -- python3 tools/winobench.py --only $L --reps 5 > $O/wfa$T.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/wfb$T -o b --output-format csv -- python3 tools/winobench.py --only $L --reps 5 > $O/wfb$T.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/wfc$T -o c --output-format csv -- python3 tools/winobench.py --only $L --reps 5 > $O/wfc$T.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/wfd$T -o d --output-format csv -- python3 tools/winobench.py --only $L --reps 5 > $O/wfd$T.log 2>&1 ; \
python3 tools/pmc_sq.py $(find $O/wf[abcd]$T -name '*counter_collection.csv') > $O/wfsum$T.log 2>&1
