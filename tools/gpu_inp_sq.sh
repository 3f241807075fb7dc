# SQ counters of the inpaint kernels at a 1024-frame batch (one pass, its own
# kill timer).  Usage (GPU box): bash tools/gpu_inp_sq.sh TAG
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-x}
test -f moseq2-detectron-extract_amd/libmdx.so || exit 5
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $O/isq$T -o c --output-format csv -- python3 tools/kbench.py --batch 1024 --reps 2 --only prep_inpaint > $O/isq$T.log 2>&1 && \
python3 tools/pmc_sq.py $(find $O/isq$T -name '*counter_collection.csv') > $O/isqsum$T.log 2>&1
echo rc=$? >> $O/isq$T.log
