# round-4 call AN: the fp16 line's kernel traces and HBM counters (bench --dtype fp16).
# Usage: bash tools/gpu_r4an.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
bash tools/gpu_profile.sh $T --dtype fp16 || { echo "fp16 profile failed"; tail -5 $O/bench$T.err; exit 1; }
tail -1 $O/bench$T.err; tail -1 $O/bench$T.json | cut -c1-300
