# round-4 call AJ: per-launch conv timings of the fp32 headline (serial steps).
# Usage: bash tools/gpu_r4aj.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-extract-loop --dump-convs $O/convs_$T.json > $O/bconv_$T.json 2> $O/bconv_$T.err || { echo "bench failed"; tail -3 $O/bconv_$T.err; exit 1; }
python3 - <<PY
import json
rows=json.load(open('$O/convs_$T.json'))
rows=[r for r in rows if r.get('tflops')]
rows.sort(key=lambda r: -r['us'])
tot=sum(r['us'] for r in rows)
print('launches', len(rows), 'total us', round(tot))
for r in rows[:25]: print(r)
PY
