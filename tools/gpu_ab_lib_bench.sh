# Bench loop (no secondaries) of the current libmdx.so against libmdx_prev.so
# (MDX_LIB_VARIANT=prev), interleaved twice.  Usage: bash tools/gpu_ab_lib_bench.sh TAG
O=gpurun_out
mkdir -p $O
T=${1:-x}
B="--no-cpu-baseline --no-secondary --no-roofline"
for r in 1 2; do
  MDX_LIB_VARIANT=prev timeout -k 10 200 python3 -u bench.py $B > $O/ab${T}b_prev_$r.json 2>&1 || exit 1
  timeout -k 10 200 python3 -u bench.py $B > $O/ab${T}b_new_$r.json 2>&1 || exit 1
done
