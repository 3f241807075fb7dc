# clean_frames: the bit-exact GPU tests and per-op timing at batch 32 and
# 1024 (both strip widths).  Usage (GPU box): bash tools/gpu_clean.sh TAG
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
test -f moseq2-detectron-extract_amd/libmdx.so || exit 5
timeout -k 10 300 python3 -u -m pytest tests/test_frameops_gpu.py -x -q -k "clean" --timeout 120 --timeout-method thread > $O/cln_t$T.log 2>&1 && \
timeout -k 10 200 python3 -u tools/kbench.py --batch 1024 --reps 5 --only clean_stream512,clean_stream256,clean > $O/cln_k$T.log 2>&1 && \
timeout -k 10 200 python3 -u tools/kbench.py --batch 32 --only clean_stream512,clean_stream256,clean >> $O/cln_k$T.log 2>&1
echo rc=$? >> $O/cln_t$T.log
