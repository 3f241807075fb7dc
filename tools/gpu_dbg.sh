set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/dbg_streams.py fp16 > $O/dbg16.log 2>&1
timeout -k 10 300 python tools/dbg_streams.py fp32 > $O/dbg32.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect tests/test_model_gpu.py::test_overlapped_extractor_matches_serial > $O/tc.log 2>&1
echo EXIT $? >> $O/tc.log
