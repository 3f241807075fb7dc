# Inpaint: the GPU parity tests, per-op timing at batch 32 and 1024, a kernel
# trace at 1024 and the HBM counters (FETCH_SIZE / WRITE_SIZE passes) at 32.
# Usage (GPU box): bash tools/gpu_inp.sh TAG
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
test -f moseq2-detectron-extract_amd/libmdx.so || exit 5
timeout -k 10 300 python3 -u -m pytest tests/test_frameops_gpu.py -x -q --timeout 120 --timeout-method thread > $O/inp_t$T.log 2>&1 && \
timeout -k 10 200 python3 -u tools/kbench.py --batch 32 --only prep_noinpaint,prep_inpaint,inpaint_only > $O/inp_k32$T.log 2>&1 && \
timeout -k 10 200 python3 -u tools/kbench.py --batch 1024 --reps 5 --only prep_noinpaint,prep_inpaint,inpaint_only > $O/inp_k1024$T.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/inp_tr$T -o t --output-format csv -- python3 tools/kbench.py --batch 1024 --reps 3 --only prep_inpaint > $O/inp_tr$T.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/inp_pf$T -o f --output-format csv -- python3 tools/kbench.py --batch 32 --reps 3 --only prep_inpaint > $O/inp_pf$T.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/inp_pw$T -o w --output-format csv -- python3 tools/kbench.py --batch 32 --reps 3 --only prep_inpaint > $O/inp_pw$T.log 2>&1
echo "rc=$?" >> $O/inp_t$T.log
