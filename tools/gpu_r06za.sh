# Round 6z: config-3 projection inputs with the row layout (A/B of r06z) (rank 0's
# share of an N-GPU batch-sharded job on one GPU, N = 1, 2, 4, 8).
set -u
OUT=gpurun_out/r06za; mkdir -p $OUT
export TMPDIR=/tmp
for N in 1 2 4 8; do
  timeout -k 10 300 python bench.py --config kitti --per-rank-of $N --layout rows --no-cpu-baseline --steps 10 --warmup 3 > $OUT/proj_kitti_$N.txt 2>&1 || exit $?
  grep '^{' $OUT/proj_kitti_$N.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d.get('projection') or {}; k=d['kernel_ms']; print($N, round(d['ms_per_step'],3), round(k['lookup_per_launch']*1e3,1), round(k['build']*1e3,0), round(p.get('projected_value', d['value'])))"
done
