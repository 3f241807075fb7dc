# round-4 call M: split-plane pipelined determinism, extract loop with 2 vs 3
# model streams, then the GN co-runner modes.  Usage: bash tools/gpu_r4m.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
DET_SPLIT=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u tools/determinism.py fp32 100 32 3 > $O/det_x6_$T.log 2>&1 || { echo "det x6 failed"; tail -5 $O/det_x6_$T.log; exit 1; }
tail -1 $O/det_x6_$T.log
for ms in 2 3; do
  EXTRACT_REPS=1 EXTRACT_OVERLAP_ONLY=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python3 -u tools/extract_bench.py 6000 1000 fp32 $ms > $O/xb_${T}_$ms.log 2>&1 || { echo "extract bench $ms failed"; tail -5 $O/xb_${T}_$ms.log; exit 1; }
  tail -1 $O/xb_${T}_$ms.log
done
bash tools/gpu_r4j.sh $T
