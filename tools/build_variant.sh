# Build libmdx_<name>.so: the current objects with <file>.hip recompiled with
# extra flags (instrumented debugging builds; loaded with MDX_LIB_VARIANT=<name>).
# Usage: bash tools/build_variant.sh NAME FILE.hip -DFLAG ...
set -e
cd "$(dirname "$0")/../moseq2-detectron-extract_amd"
N=$1; F=$2; shift 2
mkdir -p /tmp/variant_$N
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics -I.. "$@" \
  -c csrc/$F -o /tmp/variant_$N/${F%.hip}.o
objs=$(ls csrc/build/*.o | grep -v "/${F%.hip}.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs /tmp/variant_$N/${F%.hip}.o -o libmdx_$N.so
echo built libmdx_$N.so
