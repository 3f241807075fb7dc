# Bench loop (no secondaries) of the current libmdx.so against a variant
# library (MDX_LIB_VARIANT=$2, default prev: libmdx_prev.so), interleaved
# twice.  Usage: bash tools/gpu_ab_lib_bench.sh TAG [VARIANT]
O=gpurun_out
mkdir -p $O
T=${1:-x}
V=${2:-prev}
B="--no-cpu-baseline --no-secondary --no-roofline"
for r in 1 2; do
  MDX_LIB_VARIANT=$V timeout -k 10 200 python3 -u bench.py $B > $O/ab${T}b_${V}_$r.json 2>&1 || exit 1
  timeout -k 10 200 python3 -u bench.py $B > $O/ab${T}b_new_$r.json 2>&1 || exit 1
done
