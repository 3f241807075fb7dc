# round-4 final evidence on the final tree: smoke, the whole GPU suite, the
# driver's bench command with kernel traces and HBM counters.
# Usage: bash tools/gpu_r4w.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
bash tools/gpu_r4h.sh $T || exit $?
bash tools/gpu_profile.sh $T || { echo "profile failed"; tail -5 $O/bench$T.err; exit 1; }
tail -1 $O/bench$T.err; tail -1 $O/bench$T.json | cut -c1-300
