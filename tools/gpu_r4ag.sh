# round-4 call AG: the benched-config determinism test (four streams), the
# extract loop with 3 vs 4 model streams, config 5 (mixed) with four streams.
# Usage: bash tools/gpu_r4ag.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 500 --timeout-method thread -k "benched_config" > $O/tbench_$T.log 2>&1; rc=$?
echo "benched-config tests rc=$rc"; tail -1 $O/tbench_$T.log
[ $rc -ne 0 ] && exit $rc
for ms in 4 3; do
  EXTRACT_REPS=1 EXTRACT_OVERLAP_ONLY=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python3 -u tools/extract_bench.py 6000 1000 fp32 $ms > $O/xb_${T}_$ms.log 2>&1 || { echo "extract bench $ms failed"; tail -5 $O/xb_${T}_$ms.log; exit 1; }
  tail -1 $O/xb_${T}_$ms.log
done
timeout -k 10 300 python3 -u bench.py --dtype mixed --depth 101 --batch 64 --steps 40 --no-cpu-baseline --no-secondary --no-extract-loop > $O/bench_mixed_$T.json 2> $O/bench_mixed_$T.err || { echo "mixed bench failed"; tail -5 $O/bench_mixed_$T.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_mixed_$T.json').read().strip().splitlines()[-1]); print('mixed R101 B64', d['value'])"
