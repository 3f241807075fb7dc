# round-4 call E.  Usage: bash tools/gpu_r4e.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
# the packed-FP32 GN divergence: the GN input and both workspaces of the
# first rep whose level-5 workspace differs (tools/gn_emulate.py reads it)
rm -f $O/gndump_$T.npz
MDX_LIB_VARIANT=pk MDX_DEBUG_SHADOW=1 DBG_DUMP=$O/gndump_$T.npz timeout -k 10 300 python3 -u tools/dbg_race.py fp16 30 same > $O/race_dump_$T.log 2>&1 || { echo race failed; tail -5 $O/race_dump_$T.log; exit 1; }
tail -2 $O/race_dump_$T.log
if [ -f $O/gndump_$T.npz ]; then timeout -k 10 600 python3 -u tools/gn_emulate.py $O/gndump_$T.npz > $O/gnemu_$T.log 2>&1; echo "emulate rc=$?"; cat $O/gnemu_$T.log; fi
# split-plane serial steps: where the time goes with and without the plane Winograd GEMMs
for m in 384 1000000000; do
  MDX_WINO_X6_MIN_WGS=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/px6_${T}_$m -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-overlap --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/px6_${T}_$m.log 2>&1 || { echo "prof x6 $m failed"; tail -3 $O/px6_${T}_$m.log; exit 1; }
  f=$(find $O/px6_${T}_$m -name '*kernel_stats.csv' | head -1); echo "x6 min_wgs=$m $f"; head -8 "$f" | cut -c1-200
done
