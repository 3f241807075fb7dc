set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d $O/pmcr20a -o a --output-format csv -- python3 tools/roibench.py 0,160 > $O/pmcr20a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/pmcr20b -o b --output-format csv -- python3 tools/roibench.py 0,160 > $O/pmcr20b.log 2>&1
echo EXIT $? > $O/r20.done
