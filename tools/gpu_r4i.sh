# round-4 evidence, part 2: the driver's bench command, kernel traces
# (pipelined and serial) and HBM counters of the fp32 headline, then the
# fp16 and config-5 (mixed, R101 B=64) lines.  Usage: bash tools/gpu_r4i.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
bash tools/gpu_profile.sh $T || { echo "fp32 profile failed"; tail -5 $O/bench$T.err; exit 1; }
tail -1 $O/bench$T.err; tail -1 $O/bench$T.json | cut -c1-400
timeout -k 10 300 python3 -u bench.py --dtype mixed --depth 101 --batch 64 --steps 40 --no-cpu-baseline --no-secondary --no-extract-loop > $O/bench_mixed_$T.json 2> $O/bench_mixed_$T.err || { echo "mixed bench failed"; tail -5 $O/bench_mixed_$T.err; exit 1; }
tail -1 $O/bench_mixed_$T.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profm$T -o run --output-format csv -- python3 bench.py --dtype mixed --depth 101 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-roofline --no-extract-loop > $O/profm$T.log 2>&1 || { echo "mixed rocprof failed"; exit 1; }
echo "mixed rocprof ok"
