# round-4 call B: seed scan for the sharded test, packed-FP32 determinism
# localisation, the re-fixed tests.  Usage: bash tools/gpu_r4b.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 -u tools/shard_seed_scan.py 192 48 96 31 9 77 5 1000 9:1 77:1 123 > $O/scan_$T.log 2>&1 || { echo scan failed; tail -5 $O/scan_$T.log; exit 1; }
cat $O/scan_$T.log | tail -12
MDX_LIB_VARIANT=pk DBG_DETAIL=1 timeout -k 10 300 python3 -u tools/dbg_race.py fp16 24 same > $O/race_pk_$T.log 2>&1 || { echo race failed; tail -5 $O/race_pk_$T.log; exit 1; }
tail -4 $O/race_pk_$T.log
GPU_MAX_HW_QUEUES=8 MDX_LIB_VARIANT=pk timeout -k 10 300 python3 -u tools/determinism.py fp16 100 32 2 > $O/det_pk_$T.log 2>&1; rc=$?
echo "det pk rc=$rc"; tail -1 $O/det_pk_$T.log
[ $rc -le 1 ] || exit $rc   # 1 = mismatches found; anything else: stop here
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -k "rpn_proposals or winograd_planes or benched_config" > $O/t$T.log 2>&1; echo "tests rc=$?"
tail -8 $O/t$T.log
# box fc1 alone: HBM bytes and time, pacing off / on
bash tools/gpu_fc1_pmc.sh B0 || exit 1
MDX_PACE=4,1 bash tools/gpu_fc1_pmc.sh B4 || exit 1
MDX_PACE=2,1 bash tools/gpu_fc1_pmc.sh B2 || exit 1
# fp16 256x128 tile: conv tests, then the fp16 loop A/B (256x256 vs 256x128)
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "test_conv2d and large" > $O/tconv_$T.log 2>&1; echo "conv tests rc=$?"; tail -2 $O/tconv_$T.log
for lt in 1 4 1 4; do
  timeout -k 10 300 python3 -u bench.py --dtype fp16 --steps 40 --no-roofline --no-cpu-baseline --no-secondary --set mdx_conv_set_large_tiles=$lt > $O/b16_${T}_lt$lt.json 2>/dev/null || { echo "bench lt$lt failed"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/b16_${T}_lt$lt.json').read().strip().splitlines()[-1]); print('fp16 large_tiles=$lt', d['value'])"
done
