# Round 6zc: the final tree after layout="auto" -- GPU suite,
# smoke, the default bench line and the kitti line.
set -u
OUT=gpurun_out/r06zc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --durations=10 --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -6 $OUT/pytest_gpu.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
tail -1 $OUT/smoke.txt
timeout -k 10 600 python bench.py > $OUT/bench.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --config kitti --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_kitti.txt 2>&1 || exit $?
for f in bench bench_kitti; do grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $OUT/$f.txt | head -2; done
