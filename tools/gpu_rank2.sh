# Rehearse bench.py's multi-rank path on a one-GPU box: 2 ranks on the same
# GPU over gloo (barriers, per-step gather of the crops to rank 0, MAX over
# ranks); the driver's multi-GPU runs use nccl with one GPU per rank.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
MDX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline --no-secondary --no-roofline > $O/rank2.json 2> $O/rank2.err
echo EXIT $? >> $O/rank2.err
