# Default bench loop (no secondaries) under single policy changes, with two
# runs of the defaults as the reference.  Usage (GPU box): bash tools/gpu_policy_sweep.sh TAG SET [SET ...]
# where SET is a comma list of FIELD=INT (or "base").
O=gpurun_out; mkdir -p $O
T=$1; shift
B="--no-cpu-baseline --no-secondary --no-roofline"
timeout -k 10 200 python3 -u bench.py $B > $O/ps${T}_base1.json 2>&1 || exit 1
for set in "$@"; do
  args=""
  for kv in ${set//,/ }; do args="$args --set $kv"; done
  timeout -k 10 200 python3 -u bench.py $B $args > $O/ps${T}_${set//[=,]/_}.json 2>&1 || exit 1
done
timeout -k 10 200 python3 -u bench.py $B > $O/ps${T}_base2.json 2>&1 || exit 1
