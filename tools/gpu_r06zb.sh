# Round 6zb: layout="auto" -- the record tests and the kitti bench default.
set -u
OUT=gpurun_out/r06zb; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -rs --timeout 300 --timeout-method thread tests/test_records_gpu.py > $OUT/pytest_records.txt 2>&1 || exit $?
tail -2 $OUT/pytest_records.txt
timeout -k 10 300 python bench.py --config kitti --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_kitti.txt 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"pyramid_layout": "[a-z]*"' $OUT/bench_kitti.txt | head -3
timeout -k 10 300 python bench.py --config kitti --per-rank-of 8 --no-cpu-baseline --steps 10 --warmup 3 > $OUT/proj_kitti_8.txt 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"pyramid_layout": "[a-z]*"' $OUT/proj_kitti_8.txt | head -2
