# Round 6t: the record tests incl. the config-3 full-size bit-identity.
set -u
OUT=gpurun_out/r06t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -rs --durations=5 --timeout 300 --timeout-method thread tests/test_records_gpu.py > $OUT/pytest_records.txt 2>&1 || exit $?
tail -9 $OUT/pytest_records.txt
