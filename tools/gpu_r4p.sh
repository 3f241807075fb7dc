# round-4 call P: the split-plane loop on the 128-wide k_conv_x3 tile
# (pre-split weights leave it MFMA-bound) vs the 64-wide default, and the
# split-plane roofline line.  Usage: bash tools/gpu_r4p.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for n in 1 0 1 0; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 --set mdx_conv_set_x3_narrow=$n > $O/bxn_${T}_$n.json 2>/dev/null || { echo "bench narrow=$n failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bxn_${T}_$n.json').read().strip().splitlines()[-1]); print('x6 narrow=$n', d['value'])"
done
timeout -k 10 300 python3 -u bench.py --steps 30 --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/bx6roof_$T.json 2>$O/bx6roof_$T.err || { echo "x6 roofline failed"; tail -3 $O/bx6roof_$T.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bx6roof_$T.json').read().strip().splitlines()[-1]); r=d['roofline']
print('x6', d['value'], r['kernel'][:160])
for k in r['kernels']: print('  ', k['kernel'][:60], k.get('ms_per_step'), k.get('achieved_tflops'), k.get('tflop_per_step'))
print(r['all_conv'])"
