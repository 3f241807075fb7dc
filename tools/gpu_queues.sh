# fp32 bench with the HIP hardware-queue count and model-stream count varied
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
: > $O/queues.log
for q in 4 8; do for ms in 2 3; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-secondary --no-roofline --model-streams $ms > $O/q$q-$ms.json 2> $O/q$q-$ms.err || { echo "EXIT $? q$q ms$ms" >> $O/queues.log; exit 1; }
  echo "queues $q model_streams $ms -> $(python3 -c "import json; print(json.load(open('$O/q$q-$ms.json'))['value'])")" >> $O/queues.log
done; done
echo EXIT 0 >> $O/queues.log
