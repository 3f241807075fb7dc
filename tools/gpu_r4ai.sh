# round-4 call AI: the multi-rank bench path rehearsed with two gloo ranks
# sharing the one GPU (the driver's 8-GPU run uses RCCL).
# Usage: bash tools/gpu_r4ai.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
MDX_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 30 --warmup 3 --no-cpu-baseline --no-secondary > $O/bw2_$T.json 2> $O/bw2_$T.err || { echo "w2 bench failed"; tail -5 $O/bw2_$T.err; exit 1; }
tail -1 $O/bw2_$T.json | cut -c1-400
