# Round 6u: record build ablation incl. non-temporal record stores (mode 6).
set -u
OUT=gpurun_out/r06u; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/records_build_ablate.py --reps 7 > $OUT/records_build_ablate.txt 2>&1 || exit $?
tail -c 900 $OUT/records_build_ablate.txt
