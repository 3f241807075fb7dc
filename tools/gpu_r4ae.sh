# round-4 call AE: four model streams -- pipelined determinism (fp32, fp16)
# and one more interleaved A/B pair.  Usage: bash tools/gpu_r4ae.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for dt in fp32 fp16; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u tools/determinism.py $dt 150 32 4 > $O/det4_${dt}_$T.log 2>&1 || { echo "det $dt failed"; tail -3 $O/det4_${dt}_$T.log; exit 1; }
  echo "$dt: $(tail -1 $O/det4_${dt}_$T.log)"
done
for ms in 4 3; do
  timeout -k 10 300 python3 -u bench.py --steps 100 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --model-streams $ms > $O/bms_${T}_$ms.json 2>/dev/null || { echo "bench ms=$ms failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bms_${T}_$ms.json').read().strip().splitlines()[-1]); print('model_streams=$ms', d['value'])"
done
