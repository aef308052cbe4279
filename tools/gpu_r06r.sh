# Round 6r: the final tree's measurements -- the default bench line and its
# rocprofv3 kernel stats, the kitti / realtime (graph) / middlebury lines,
# the kitti kernel stats and the kitti PMC passes (profiles/pmc.json).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=$R/gpurun_out/r06r; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$n.txt 2>&1; local rc=$?; echo "[$n] rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$n.txt; exit $rc; fi; }
step bench 600 python bench.py
step bench_kitti 300 python bench.py --config kitti --no-cpu-baseline --steps 20 --warmup 3
step bench_realtime_graph 300 python bench.py --config realtime --graph --no-cpu-baseline --steps 200 --warmup 10
step bench_middlebury 300 python bench.py --config middlebury --no-cpu-baseline --steps 5 --warmup 2
cd /tmp
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-steps 0 --config4-steps 0 --no-backward
step rocprof_kitti 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profk -o trace -- python3 $R/bench.py --config kitti --steps 10 --warmup 3 --no-cpu-baseline
B="python3 $R/bench.py --config kitti --pmc-calibrate --steps 2 --warmup 1 --no-cpu-baseline"
step pf 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o pf -- $B
step pw 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o pw -- $B
step ps 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $OUT/ps -o ps -- $B
cd $R
find $OUT/prof -name "*stats*.csv" -exec sh -c 'echo "== $1"; cat "$1"' _ {} \; > $OUT/kernel_stats.txt 2>/dev/null
find $OUT/profk -name "*stats*.csv" -exec sh -c 'echo "== $1"; cat "$1"' _ {} \; > $OUT/kernel_stats_kitti.txt 2>/dev/null
for f in bench bench_kitti bench_realtime_graph bench_middlebury; do grep -o '"ms_per_step": [0-9.]*' $OUT/$f.txt | head -1; done
head -c 1500 $OUT/kernel_stats.txt
