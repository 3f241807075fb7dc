# round-4 call C.  Usage: bash tools/gpu_r4c.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for v in nopk pk; do
  for hw in "112 128" "14 16" "28 32"; do
    for bg in 0 3; do
      tag=${v}_bg${bg}_${hw// /x}
      timeout -k 10 120 ./tools/native/gn_repro_$v 300 $bg $hw > $O/gn_${T}_$tag.log 2>&1 || { echo "gn_repro $tag failed: $?"; exit 1; }
      echo "$tag: $(tail -1 $O/gn_${T}_$tag.log)"
    done
  done
done
timeout -k 10 400 python3 -u tools/shard_seed_scan.py 384 96 192 9 77 31 9:1 77:1 5 > $O/scan_$T.log 2>&1 || { echo scan failed; tail -5 $O/scan_$T.log; exit 1; }
grep seed $O/scan_$T.log
# persistent GEMM: correctness first (bit-equal to k_conv_sb), then A/B
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "pointwise_instances or (test_conv3x3_winograd and f32-mfma)" > $O/tsbp_$T.log 2>&1 || { echo "sbp tests failed"; tail -20 $O/tsbp_$T.log; exit 1; }
tail -1 $O/tsbp_$T.log
# persistent GEMM A/B: microbench, then the bench loop
for p in 0 1; do
  timeout -k 10 300 python3 -u tools/gemm32bench.py single_stage=$((4 + p)) > $O/g32_${T}_p$p.log 2>&1 || { echo "g32 p$p failed"; tail -3 $O/g32_${T}_p$p.log; exit 1; }
  echo "persist=$p: $(grep -i 'weighted\|total' $O/g32_${T}_p$p.log | tail -2)"
done
for p in 0 1 0 1; do
  timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --set mdx_conv_set_single_stage=$((4 + p)) > $O/b32_${T}_p$p.json 2>/dev/null || { echo "bench p$p failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b32_${T}_p$p.json').read().strip().splitlines()[-1]); print('fp32 persist=$p', d['value'])"
done
# split-plane loop with the plane Winograd GEMMs
timeout -k 10 300 python3 -u bench.py --steps 60 --no-roofline --no-cpu-baseline --no-secondary --set mdx_conv_set_fp32_split=6 > $O/bx6_$T.json 2>/dev/null || { echo "bench x6 failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bx6_$T.json').read().strip().splitlines()[-1]); print('x6 loop', d['value'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 800 --timeout-method thread -k "test_forward_full_frame and (mixed or 101-64-fp32)" > $O/tpar_$T.log 2>&1; echo "parity rc=$?"; tail -4 $O/tpar_$T.log
