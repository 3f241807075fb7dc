# Round-6 first GPU pass: the ping-pong GEMM microbench, the reworked
# full-frame parity cases, the default bench line.  Usage: bash tools/gpu_r6a.sh TAG
export TMPDIR=/tmp
T=${1:-a}
O=gpurun_out
mkdir -p $O
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 400 python3 -u tools/ppbench.py > $O/pp$T.log 2>&1
rc=$?; echo "ppbench rc=$rc" > $O/r6$T.txt; ok $rc || exit $rc
timeout -k 10 1100 python3 -u -m pytest tests/test_parity_full.py -m gpu -v --timeout 600 --timeout-method thread > $O/par$T.log 2>&1
rc=$?; echo "parity rc=$rc" >> $O/r6$T.txt; ok $rc || exit $rc
timeout -k 10 400 python3 -u bench.py > $O/bench$T.json 2> $O/bench$T.err
echo "bench rc=$?" >> $O/r6$T.txt
