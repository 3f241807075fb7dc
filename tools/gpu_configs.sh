# BASELINE configs 3 and 5: the 10k-frame extract loop (fp32, fp16; tracking
# off/on) and the R101-FPN fp16 B=64 bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for dt in fp32 fp16; do
  EXTRACT_REPS=1 EXTRACT_OVERLAP_ONLY=1 timeout -k 10 400 python -u tools/extract_bench.py 10000 1000 $dt > $O/xl_$dt.log 2>&1 || { echo "EXIT extract $dt $?" >> $O/cfg.log; exit 1; }
done
timeout -k 10 400 python bench.py --depth 101 --dtype fp16 --batch 64 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo "EXIT bench5 $?" >> $O/cfg.log; exit 1; }
echo "EXIT 0" >> $O/cfg.log
