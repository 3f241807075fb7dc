# SQ counters of the fused clean_frames kernel at a 1024-frame chunk (one
# pass, its own kill timer), summarised by tools/pmc_sq.py.
# Usage (GPU box): bash tools/gpu_clean_pmc.sh
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $O/cln -o c --output-format csv -- python3 tools/kbench.py --batch 1024 --reps 3 --only clean_stream512 > $O/cln.log 2>&1 && \
python3 tools/pmc_sq.py $(find $O/cln -name '*counter_collection.csv') > $O/clnsum.log 2>&1
