set -u
OUT=gpurun_out/r06e; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for sh in default 0,2; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-backward --e2e-steps 0 --config4-steps 0 --steps 30 --warmup 5 --shadow $sh > $OUT/bench_shadow_${sh}_$rep.log 2>&1 || exit $?
    python - "$OUT/bench_shadow_${sh}_$rep.log" "$sh" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'build', round(d['kernel_ms']['build']*1e3,1), 'lookup', round(d['kernel_ms']['lookup_per_launch']*1e3,2))
PY
  done
done
