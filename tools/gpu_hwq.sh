# A/B of the HIP hardware-queue count (GPU_MAX_HW_QUEUES) for the overlapped bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 30 --warmup 4 --no-cpu-baseline --no-roofline > $O/hwq_$q.json 2>/dev/null || exit 1
  echo "q=$q $(python -c 'import json,sys; print(json.load(open(sys.argv[1]))["value"])' $O/hwq_$q.json)" >> $O/hwq.log
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --steps 30 --warmup 4 --no-cpu-baseline --no-roofline --model-streams 3 > $O/hwq_8s3.json 2>/dev/null || exit 1
echo "q=8 s3 $(python -c 'import json,sys; print(json.load(open(sys.argv[1]))["value"])' $O/hwq_8s3.json)" >> $O/hwq.log
