# PMC counters of the ROIAlign microbenchmark (one pass per counter group).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/roipmc1 -o p --output-format csv -- python3 tools/roibench.py > $O/roipmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/roipmc2 -o p --output-format csv -- python3 tools/roibench.py > $O/roipmc2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -d $O/roipmc3 -o p --output-format csv -- python3 tools/roibench.py > $O/roipmc3.log 2>&1
echo EXIT $? >> $O/roipmc1.log
