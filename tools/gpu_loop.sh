# All GPU tests, then the full extract loop (10k frames, chunks of 1000,
# overlapped host step, tracking off / on) in fp32 and fp16.
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/t$T.log 2>&1; echo "TESTS EXIT $?" >> $O/t$T.log
grep -q "TESTS EXIT 0" $O/t$T.log && \
EXTRACT_REPS=1 EXTRACT_OVERLAP_ONLY=1 timeout -k 10 400 python tools/extract_bench.py 10000 1000 fp32 > $O/loop32$T.json 2> $O/loop$T.err && \
EXTRACT_REPS=1 EXTRACT_OVERLAP_ONLY=1 timeout -k 10 300 python tools/extract_bench.py 10000 1000 fp16 > $O/loop16$T.json 2>> $O/loop$T.err
echo EXIT $? >> $O/t$T.log
