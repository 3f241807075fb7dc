# Box fc1 alone: time + HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE,
# separate passes).  Usage: bash tools/gpu_fc1_pmc.sh TAG [knob=value ...]
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}; shift || true
O=gpurun_out; mkdir -p $O
timeout -k 10 120 python3 -u tools/fc1bench.py 5 "$@" > $O/fc1_$T.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fc1f_$T -o f --output-format csv -- python3 tools/fc1bench.py 3 "$@" > $O/fc1f_$T.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/fc1w_$T -o w --output-format csv -- python3 tools/fc1bench.py 3 "$@" > $O/fc1w_$T.log 2>&1 && \
python3 tools/pmc_dispatch.py $(find $O/fc1f_$T $O/fc1w_$T -name '*counter_collection.csv') >> $O/fc1_$T.log 2>&1
echo "EXIT $?" >> $O/fc1_$T.log
tail -3 $O/fc1_$T.log
