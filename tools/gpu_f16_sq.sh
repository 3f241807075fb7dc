# SQ counters of the fp16 GEMM kernels on two layer shapes (one pass, its own
# kill timer).  Usage (GPU box): bash tools/gpu_f16_sq.sh TAG
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-x}
test -f moseq2-detectron-extract_amd/libmdx.so || exit 5
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d $O/fsq$T -o c --output-format csv -- python3 tools/f16bench.py only=box_fc1,mask_conv_b64 > $O/fsq$T.log 2>&1 && \
python3 tools/pmc_sq.py $(find $O/fsq$T -name '*counter_collection.csv') > $O/fsqsum$T.log 2>&1
echo rc=$? >> $O/fsq$T.log
