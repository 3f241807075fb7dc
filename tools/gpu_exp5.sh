# SQ counters of the fp32 GEMM microbench (tools/gpu_gemm32.sh PMC=1) and a
# model-stream-count A/B of the bench loop.  rc 1 does not stop the script.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp5_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp5_steps.txt; exit $rc; fi
}
run g32pmc.log env PMC=1 bash tools/gpu_gemm32.sh P5
run bE5_ms3.json timeout -k 10 300 python3 -u bench.py --steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop --model-streams 3
run bE5_ms2.json timeout -k 10 300 python3 -u bench.py --steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop
run bE5_ms1.json timeout -k 10 300 python3 -u bench.py --steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop --model-streams 1
echo done >> $O/exp5_steps.txt
