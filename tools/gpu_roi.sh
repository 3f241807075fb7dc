# ROIAlign order A/B: GPU tests of the pooler + the default full-frame parity
# case, then kernel-trace stats of the serial fp32 bench with the level/band
# ROI permutation on and off, then the overlapped bench line for both
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_parity_full.py -x -q --timeout 300 --timeout-method thread -k "roi_align or 50-32-fp32-4" > $O/troi.log 2>&1 || { echo "EXIT tests $?" >> $O/troi.log; exit 1; }
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/roi$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-roofline --no-overlap --set mdx_roi_align_set_sorted=$v > $O/roiprof$v.log 2>&1 || { echo "EXIT prof $v $?" >> $O/troi.log; exit 1; }
done
for v in 1 0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-roofline --set mdx_roi_align_set_sorted=$v > $O/roib$v.json 2> $O/roib$v.err || { echo "EXIT bench $v $?" >> $O/troi.log; exit 1; }
done
echo "EXIT 0" >> $O/troi.log
