# Round 6o: record lookup variants capped at 4 waves per SIMD (dev modes 7, 8).
set -u
OUT=gpurun_out/r06o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/records_lookup_ablate.py --reps 5 --modes 0,4,7,8 > $OUT/records_lookup_ablate.txt 2>&1 || exit $?
tail -c 400 $OUT/records_lookup_ablate.txt
