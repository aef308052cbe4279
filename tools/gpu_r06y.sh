# Round 6y: bench.py --gpus 2 self-launch with gloo (two ranks sharing the
# one GPU) -- the N>1 path of the final tree, collectives host-side.
set -u
OUT=gpurun_out/r06y; mkdir -p $OUT
export TMPDIR=/tmp
RAFTCORR_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-backward > $OUT/launch_gloo2.txt 2>&1 || exit $?
grep '^{' $OUT/launch_gloo2.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['ms_per_step'], d.get('status'), (d.get('config4_network') or {}).get('ms_per_pair'), (d.get('config4_network') or {}).get('error'))"
