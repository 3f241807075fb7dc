# round-4 call AF: the single-stage split-plane kernel on the 128-wide tile
# (mdx_conv_set_x3_narrow(0)) vs the 64-wide default; tests of both.
# Usage: bash tools/gpu_r4af.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for n in 0 1 0 1; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 --set mdx_conv_set_x3_narrow=$n > $O/bn128_${T}_$n.json 2>/dev/null || { echo "bench narrow=$n failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bn128_${T}_$n.json').read().strip().splitlines()[-1]); print('x6 narrow=$n', d['value'])"
done
