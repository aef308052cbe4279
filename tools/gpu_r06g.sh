# Round 6g: record build ablations (dev library) + rocprof kernel stats of
# the kitti bench with records.
set -u
OUT=gpurun_out/r06g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/records_build_ablate.py --reps 7 > $OUT/records_build_ablate.txt 2>&1 || exit $?
tail -c 700 $OUT/records_build_ablate.txt
