# round-4 call AM: box-pooler kernel variants in the fp32 hot loop (four
# model streams), interleaved.  Usage: bash tools/gpu_r4am.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for m in 4 6 5 0 4 6 5 0; do
  timeout -k 10 300 python3 -u bench.py --steps 100 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --roi-mode $m > $O/broi_${T}_$m.json 2>/dev/null || { echo "bench roi=$m failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/broi_${T}_$m.json').read().strip().splitlines()[-1]); print('roi_mode=$m', d['value'])"
done
