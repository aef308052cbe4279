# Round 6k: kitti with the record layout (bench default) -- interleaved A/B
# against the rows, both bench lines on one box, rocprofv3 kernel stats and
# the three PMC passes for profiles/pmc.json.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06k; mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/records_probe.py --reps 5 > $OUT/records_probe.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config kitti --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_kitti_records.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config kitti --steps 20 --warmup 3 --no-cpu-baseline --layout rows > $OUT/bench_kitti_rows.txt 2>&1 || exit $?
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --config kitti --steps 5 --warmup 2 --no-cpu-baseline > $OUT/kt.txt 2>&1 || exit $?
B="python3 $GRAFT_REPO_ROOT/bench.py --config kitti --pmc-calibrate --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o pf -- $B > $OUT/pf.txt 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o pw -- $B > $OUT/pw.txt 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $OUT/ps -o ps -- $B > $OUT/ps.txt 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
tail -c 500 $OUT/records_probe.txt
for f in $OUT/bench_kitti_records.txt $OUT/bench_kitti_rows.txt; do grep -o '"ms_per_step": [0-9.]*' $f; done
find $OUT/kt -name "*kernel_stats.csv" | head -2
