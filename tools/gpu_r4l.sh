# round-4 call L: smoke + the whole GPU suite (the split-plane parity cases
# run the pre-split-weight k_conv_x3), then the split-plane loop and its
# serial kernel trace.  Usage: bash tools/gpu_r4l.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
bash tools/gpu_r4h.sh $T || exit $?
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/bx3_${T}_$i.json 2>/dev/null || { echo "bench x3 failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bx3_${T}_$i.json').read().strip().splitlines()[-1]); print('x6 loop', d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/px3_$T -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-overlap --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/px3_$T.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof ok"
