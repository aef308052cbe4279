# Round 6w: the split build with its MFMAs at raised wave priority (dev
# modes: phased K step 268435456, per-fragment 536870912; +3 compute only).
set -u
OUT=gpurun_out/r06w; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/build_ablate.py --config sceneflow --rounds 9 --modes 0,268435456,536870912,3,268435459 > $OUT/ablate_c2.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/build_ablate.py --config middlebury --rounds 5 --modes 0,268435456,536870912 > $OUT/ablate_c4.txt 2>&1 || exit $?
grep -E '"(exact|0|3|268435456|536870912|268435459)"|median|bit_identical' $OUT/ablate_c2.txt | head -30
grep -E 'median|bit_identical' $OUT/ablate_c4.txt | head -12
