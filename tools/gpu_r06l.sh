# Round 6l: the tree after the record layout -- full GPU suite, smoke, the
# default bench line and its rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06l; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --durations=15 --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -12 $OUT/pytest_gpu.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
tail -1 $OUT/smoke.txt
timeout -k 10 600 python bench.py > $OUT/bench.txt 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' $OUT/bench.txt | head -4
