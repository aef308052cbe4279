# Round 6q: record lookup with two 64-pixel groups per wave (dev mode 10).
set -u
OUT=gpurun_out/r06q; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/records_lookup_ablate.py --reps 5 --modes 0,9,10 > $OUT/records_lookup_ablate.txt 2>&1 || exit $?
tail -c 400 $OUT/records_lookup_ablate.txt
