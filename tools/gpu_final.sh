# Round-end evidence on the final tree: smoke, the whole GPU suite, then the
# measurement recipe (driver bench command, kernel traces, HBM counters).
# Usage: bash tools/gpu_final.sh TAG
export TMPDIR=/tmp
T=${1:-F}
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke$T.log 2>&1
rc=$?; echo "smoke rc=$rc" > $O/final$T.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/t$T.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/final$T.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_profile.sh $T
echo "profile rc=$?" >> $O/final$T.txt
