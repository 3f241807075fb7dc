# split-plane fp32: kernel tests (both tiles), the full-frame parity case
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py tests/test_parity_full.py -x -v --timeout 300 --timeout-method thread -k "fp32_split or winograd or 50-32-fp32-4" > $O/tsplit2.log 2>&1
echo "EXIT $?" >> $O/tsplit2.log
