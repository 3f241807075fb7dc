set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
T=${1:-x}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "overlapped" --timeout 120 --timeout-method thread > $O/qs$T.log 2>&1 && \
for n in 1 2 3 4; do timeout -k 10 200 python bench.py --steps 30 --warmup 4 --no-cpu-baseline --no-roofline --model-streams $n > $O/bs${T}_$n.json 2>/dev/null || exit 1; done
echo EXIT $? >> $O/qs$T.log
