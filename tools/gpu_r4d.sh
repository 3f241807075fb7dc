# round-4 call D.  Usage: bash tools/gpu_r4d.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
# where the packed-FP32 GroupNorm difference starts: shadow copies of the
# level-5 GN workspace (stats | partials) and of the GN outputs
MDX_LIB_VARIANT=pk MDX_DEBUG_SHADOW=1 timeout -k 10 300 python3 -u tools/dbg_race.py fp16 30 same > $O/race_shadow_$T.log 2>&1 || { echo race failed; tail -5 $O/race_shadow_$T.log; exit 1; }
grep -c identical $O/race_shadow_$T.log; grep -v identical $O/race_shadow_$T.log | tail -12
# fc1 on the 256x256 LDS-DMA kernel (2.7 GB) vs k_conv_sb (14 GB) in the pipelined loop
for d in 0 2 0 2; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --set mdx_conv_set_dma_f32=$d > $O/bd_${T}_$d.json 2>/dev/null || { echo "bench dma $d failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bd_${T}_$d.json').read().strip().splitlines()[-1]); print('fp32 dma_f32=$d', d['value'])"
done
# split-plane loop: plane Winograd GEMMs (default) vs every layer on k_conv_x3
for m in 384 1000000000 384 1000000000; do
  MDX_WINO_X6_MIN_WGS=$m timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --set mdx_conv_set_fp32_split=6 > $O/bx6_${T}_$m.json 2>/dev/null || { echo "bench x6 $m failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bx6_${T}_$m.json').read().strip().splitlines()[-1]); print('x6 min_wgs=$m', d['value'])"
done
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py tests/test_parity_full.py -m gpu -v --timeout 800 --timeout-method thread -k "shard or mixed" > $O/tshard_$T.log 2>&1; echo "shard/mixed rc=$?"; tail -6 $O/tshard_$T.log
