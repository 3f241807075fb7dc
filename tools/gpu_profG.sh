# kernel trace + stats of the default fp32 bench loop (pipelined), final tree
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/profG.json 2> gpurun_out/profG.err
