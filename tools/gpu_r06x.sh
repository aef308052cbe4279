# Round 6x: sanity of the last product binary (rebuilt after r06v with
# dev-only additions): smoke, the record tests, the core lookup/volume tests,
# the default bench line.
set -u
OUT=gpurun_out/r06x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
tail -1 $OUT/smoke.txt
timeout -k 10 600 python -u -m pytest -q -rs --timeout 300 --timeout-method thread tests/test_records_gpu.py tests/test_corr_gpu.py tests/test_split_gpu.py tests/test_configs_gpu.py tests/test_fullsize_gpu.py > $OUT/pytest.txt 2>&1; rc=$?; tail -3 $OUT/pytest.txt; if [ $rc -gt 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > $OUT/bench.txt 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $OUT/bench.txt | head -2
