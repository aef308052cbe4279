# Round 6p: the cooperative record fetch as the product -- record parity
# tests, the rows-vs-records A/B and the kitti bench.
set -u
OUT=gpurun_out/r06p; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_records_gpu.py tests/test_configs_gpu.py > $OUT/pytest_records.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/records_probe.py --reps 5 > $OUT/records_probe.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config kitti --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_kitti.txt 2>&1 || exit $?
tail -2 $OUT/pytest_records.txt; tail -c 400 $OUT/records_probe.txt; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_kitti.txt
