# fp32 GEMM kernel A/B (k_conv vs k_conv_m32 vs persistent k_gemm_m32p), their tests, pipeline determinism soak
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "m32 or inpaint or winograd or roi_align or pipelined or overlapped or config3 or extract_session" > $O/tE1.log 2>&1 && \
timeout -k 10 200 python3 -u tools/gemm32bench.py > $O/g32_base.log 2>&1 && \
timeout -k 10 200 python3 -u tools/gemm32bench.py f32_mfma32=1 > $O/g32_m32.log 2>&1 && \
timeout -k 10 200 python3 -u tools/gemm32bench.py f32_mfma32=2 > $O/g32_m32p.log 2>&1 && \
timeout -k 10 200 python3 -u tools/gemm32bench.py f32_mfma32=2 wino_vec=1 > $O/g32_m32pv.log 2>&1 && \
timeout -k 10 200 python3 -u tools/gemm32bench.py winograd_dma=2,0 > $O/g32_wdma.log 2>&1 && \
timeout -k 10 200 python3 -u tools/roibench.py fp32 > $O/roi32.log 2>&1 && \
timeout -k 10 300 python3 -u tools/determinism.py fp32 150 > $O/det32.log 2>&1 ; \
timeout -k 10 300 python3 -u tools/determinism.py fp16 150 > $O/det16.log 2>&1 ; echo EXIT $?
MDX_LIB_VARIANT=pk timeout -k 10 300 python3 -u tools/determinism.py fp32 150 > $O/det32pk.log 2>&1 ; \
MDX_LIB_VARIANT=pk timeout -k 10 300 python3 -u tools/determinism.py fp16 150 > $O/det16pk.log 2>&1 ; \
timeout -k 10 300 python3 -u bench.py --steps 40 --no-secondary --no-cpu-baseline --no-roofline > $O/bE1_base.json 2>/dev/null ; \
MDX_LIB_VARIANT=pk timeout -k 10 300 python3 -u bench.py --steps 40 --no-secondary --no-cpu-baseline --no-roofline > $O/bE1_pk.json 2>/dev/null ; echo EXIT2 $?
