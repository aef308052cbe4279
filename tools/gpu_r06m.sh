# Round 6n: record lookup with the cooperative whole-record fetch (dev mode 4).
set -u
OUT=gpurun_out/r06m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/records_lookup_ablate.py --reps 5 > $OUT/records_lookup_ablate.txt 2>&1 || exit $?
tail -c 400 $OUT/records_lookup_ablate.txt
