# Round 6i: records with transposed level-2 image writes and 3-read batched gathers: parity,
# build ablation, kitti bench with records.
set -u
OUT=gpurun_out/r06i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_records_gpu.py > $OUT/pytest_records.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/records_build_ablate.py --reps 7 > $OUT/records_build_ablate.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config kitti --steps 20 --warmup 3 --no-cpu-baseline --layout records > $OUT/bench_kitti_records.txt 2>&1 || exit $?
tail -3 $OUT/pytest_records.txt; tail -c 700 $OUT/records_build_ablate.txt; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_kitti_records.txt
