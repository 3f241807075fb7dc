# SQ / TA / TCC counters of every kernel of serial bench steps (two passes,
# each with its own kill timer), summarised per kernel by tools/pmc_sq.py;
# the box pooler is k_roi_align_sep<float, false, true>.
# Usage (GPU box): bash tools/gpu_roi_sq.sh TAG
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-x}
test -f moseq2-detectron-extract_amd/libmdx.so || exit 5
B="--steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --no-overlap"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d $O/rsqa$T -o c --output-format csv -- python3 bench.py $B > $O/rsqa$T.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/rsqb$T -o c --output-format csv -- python3 bench.py $B > $O/rsqb$T.log 2>&1 && \
python3 tools/pmc_sq.py $(find $O/rsqa$T $O/rsqb$T -name '*counter_collection.csv') > $O/rsqsum$T.json 2> $O/rsqsum$T.err
echo rc=$? >> $O/rsqa$T.log
