# Round 6f: the record layout (RC_LAYOUT_RECORDS) on the GPU -- its parity
# tests, the rows-vs-records A/B at KITTI and the kitti bench both ways.
set -u
OUT=gpurun_out/r06f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_records_gpu.py > $OUT/pytest_records.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/records_probe.py --reps 5 > $OUT/records_probe.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config kitti --steps 20 --warmup 3 --no-cpu-baseline --layout records > $OUT/bench_kitti_records.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config kitti --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_kitti_rows.txt 2>&1 || exit $?
tail -c 600 $OUT/records_probe.txt
