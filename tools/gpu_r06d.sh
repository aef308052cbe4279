set -u
OUT=gpurun_out/r06d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --durations=25 --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -45 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python tools/build_ablate.py --config realtime --rounds 9 --modes 0,2,4,6 > $OUT/ablate_realtime.log 2>&1 || exit $?
grep -E '"(0|2|4|6|exact)"|median' $OUT/ablate_realtime.log
timeout -k 10 300 python tools/graph_floor.py > $OUT/graph_floor.log 2>&1 || exit $?
tail -3 $OUT/graph_floor.log
