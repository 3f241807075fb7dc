# round-4 call AD: the hot loop with four model streams vs three (interleaved).
# Usage: bash tools/gpu_r4ad.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for ms in 4 3 4 3; do
  timeout -k 10 300 python3 -u bench.py --steps 100 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --model-streams $ms > $O/bms_${T}_$ms.json 2>/dev/null || { echo "bench ms=$ms failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bms_${T}_$ms.json').read().strip().splitlines()[-1]); print('model_streams=$ms', d['value'])"
done
