# Effective clock and MFMA busy of the conv kernels in the fp32 bench (one PMC
# pass: GRBM_GUI_ACTIVE + SQ counters; no trace domains).
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $O/clk$T -o c --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --no-overlap ${@:2} > $O/clk$T.log 2>&1
echo EXIT $? >> $O/clk$T.log
