set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python tools/roistats.py > $O/roi13.log 2>&1 ; \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace -d $O/pmca13 -o a --output-format csv -- python3 tools/convbench.py 5,7 > $O/pmca13.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-trace -d $O/pmcb13 -o b --output-format csv -- python3 tools/convbench.py 5,7 > $O/pmcb13.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace -d $O/pmcc13 -o c --output-format csv -- python3 tools/convbench.py 5,7 > $O/pmcc13.log 2>&1
echo EXIT $? > $O/r13.done
