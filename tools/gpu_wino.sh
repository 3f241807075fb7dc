# Winograd: conv tests + fp32 parity, then fp32 bench lines with it on / off
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_parity_full.py -x -v --timeout 200 --timeout-method thread -k "winograd or conv2d or fp32" > $O/tw$T.log 2>&1 || { echo "EXIT $?" >> $O/tw$T.log; exit 1; }
for m in ${WMODES:-2 4 0}; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary --winograd $m --dump-convs $O/convsw$T-$m.json > $O/benchw$T-$m.json 2> $O/benchw$T-$m.err || { echo "EXIT $? bench $m" >> $O/tw$T.log; exit 1; }
done
echo EXIT 0 >> $O/tw$T.log
