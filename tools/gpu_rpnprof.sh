set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rpnprof -o r --output-format csv -- python3 tools/rpnbench.py 32 20 > $O/rpnprof.log 2>&1
echo EXIT $? >> $O/rpnprof.log
