# round-4 evidence, part 1: smoke and the whole GPU suite.  Usage: bash tools/gpu_r4h.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke_$T.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/tests_$T.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR" $O/tests_$T.log | head -20; tail -1 $O/tests_$T.log
exit $rc
