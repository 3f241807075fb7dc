# GPU tests, verbose, one process.  Usage: bash tools/gpu_tests.sh TAG ['-k expr']
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
if [ -n "${2:-}" ]; then KA=(-k "$2"); else KA=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread "${KA[@]}" > $O/t$T.log 2>&1
echo EXIT $? >> $O/t$T.log
