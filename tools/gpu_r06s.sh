# Round 6s: the final tree's GPU suite and smoke.
set -u
OUT=gpurun_out/r06s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --durations=15 --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 $OUT/pytest_gpu.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
tail -1 $OUT/smoke.txt
