# GEMM layer microbench of the current libmdx.so against libmdx_prev.so
# (MDX_LIB_VARIANT=prev), interleaved twice.  Usage: bash tools/gpu_ab_lib.sh TAG
O=gpurun_out
mkdir -p $O
T=${1:-x}
for r in 1 2; do
  MDX_LIB_VARIANT=prev timeout -k 10 200 python3 -u tools/gemm32bench.py > $O/ab${T}_prev_$r.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u tools/gemm32bench.py > $O/ab${T}_new_$r.log 2>&1 || exit 1
done
