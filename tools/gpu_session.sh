#!/bin/bash
# One gpurun session: GPU tests, smoke, bench, rocprofv3 kernel trace.
# Usage (on the GPU box, via gpurun): bash tools/gpu_session.sh <tag> [stages]
#   stages: comma list of test,smoke,bench,prof (default: all)
# Every GPU step has its own time limit; a fault/abort/timeout ends the script
# (exit codes other than 0/1), a plain test failure (1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
STAGES=${2:-test,smoke,bench,prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ ",$STAGES," == *",$1,"* ]]; }
step() {  # step <name> <timeout> cmd...
    local name=$1 t=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
    tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
rocm-smi --showproductname > "$OUT/gpu.txt" 2>&1 || true
has tsplit && step pytest_split 600 python -u -m pytest tests/test_split_gpu.py tests/test_configs_gpu.py -v -rf --timeout 120 --timeout-method thread
has test  && step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
has smoke && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has bench && step bench 600 python bench.py
has e2e && step e2e_probe 900 python tools/e2e_probe.py
has probe && step line_probe 300 python tools/line_probe.py
has lprobe && step lookup_probe 300 python tools/lookup_probe.py --dev-variants ${LPROBE_VARIANTS:-201,202}
has gprobe && step gather_probe 300 python tools/gather_probe.py
has shard && step shard_probe 600 python tools/shard_probe.py
has ablate && step ablate 600 python tools/ablate.py --build-modes 0 --lookup-variants 0 --chain
has ablateb && step ablate_bwd 600 python tools/ablate.py --build-modes 0 --lookup-variants 0 --bwd
has ablatec && step ablate_conv 600 python tools/ablate.py --build-modes 0 --lookup-variants 0 --convc1
has ablatek && step ablate_kitti 600 python tools/ablate.py --config kitti --build-modes 0,2,1,3 --lookup-variants 0,1,3
has configs && step bench_realtime 300 python bench.py --config realtime --no-cpu-baseline --steps 50 --warmup 5 && step bench_realtime_graph 300 python bench.py --config realtime --graph --no-cpu-baseline --steps 200 --warmup 10
has configs && step bench_middlebury 300 python bench.py --config middlebury --no-cpu-baseline --steps 5 --warmup 2
has configs && step bench_kitti 300 python bench.py --config kitti --no-cpu-baseline --steps 10 --warmup 3
has ab16 && step ablate_b16 600 python tools/ablate.py --config kitti --build-modes ${AB16_MODES:-0,49,50,40,51} --lookup-variants 0 --rounds 5
has kitti && step bench_kitti 300 python bench.py --config kitti --no-cpu-baseline --steps 10 --warmup 3
if has profk; then
    step rocprof_kitti 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profk" -o trace \
        -- python3 bench.py --config kitti --steps 10 --warmup 3 --no-cpu-baseline --e2e-steps 0
    find "$OUT/profk" -name "*stats*.csv" -exec sh -c 'echo "== $1"; cat "$1"' _ {} \; > "$OUT/kernel_stats_kitti.txt" 2>/dev/null
    head -c 2000 "$OUT/kernel_stats_kitti.txt"
fi
if has pmck; then   # kitti build HBM bytes (profiles/traffic.json "kitti")
    step pmck_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmck_fetch" -o f \
        -- python3 tools/build_probe.py --modes 0
    step pmck_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmck_write" -o w \
        -- python3 tools/build_probe.py --modes 0
    python tools/pmc_traffic.py "$OUT/pmck_fetch" "$OUT/pmck_write" --config kitti --out "$OUT/traffic.json" > "$OUT/traffic_kitti.log" 2>&1
    cat "$OUT/traffic_kitti.log"
fi
if has prof; then
    step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
        -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-steps 0 --config4-steps 0
    find "$OUT/prof" -name "*stats*.csv" -exec sh -c 'echo "== $1"; cat "$1"' _ {} \; > "$OUT/kernel_stats.txt" 2>/dev/null
    head -c 3000 "$OUT/kernel_stats.txt"
fi
if has pmc; then
    step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o f \
        -- python3 tools/probe.py
    step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o w \
        -- python3 tools/probe.py
    step pmc_sq 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
        --output-format csv -d "$OUT/pmc_sq" -o s -- python3 tools/probe.py
    python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --out "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1
    cat "$OUT/traffic.log"
    python tools/pmc_sq.py "$OUT/pmc_sq" "$OUT/mfma.json" > "$OUT/pmc_sq.txt" 2>&1; cat "$OUT/pmc_sq.txt"
fi
if has pmcsq; then
    step pmc_sq2 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/pmc_sq2" -o s -- python3 tools/probe.py
    python tools/pmc_sq.py "$OUT/pmc_sq2" > "$OUT/pmc_sq2.txt" 2>&1; cat "$OUT/pmc_sq2.txt"
fi
if has pmcw; then   # wave-state breakdown: where each kernel's wave cycles go
    step pmc_w1 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/pmc_w1" -o s -- python3 tools/probe.py ${PROBE_ARGS:-}
    step pmc_w2 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS \
        --output-format csv -d "$OUT/pmc_w2" -o s -- python3 tools/probe.py ${PROBE_ARGS:-}
    python tools/pmc_raw.py "$OUT/pmc_w1" > "$OUT/pmc_w.txt" 2>&1; python tools/pmc_raw.py "$OUT/pmc_w2" >> "$OUT/pmc_w.txt" 2>&1; grep lookup "$OUT/pmc_w.txt"
fi
if has pmcs8; then   # split kernels (4- vs 8-wave, product vs compute-only): instruction mix and wave states
    BA8="--modes ${PMCS8_MODES:-0,3,8/0,8/3} --rounds 1 --per 3"
    step pmc_s81 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/pmc_s81" -o s -- python3 tools/build_ablate.py $BA8
    step pmc_s82 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/pmc_s82" -o s -- python3 tools/build_ablate.py $BA8
    python tools/pmc_raw.py "$OUT/pmc_s81" > "$OUT/pmc_s8.txt" 2>&1; python tools/pmc_raw.py "$OUT/pmc_s82" >> "$OUT/pmc_s8.txt" 2>&1; grep split "$OUT/pmc_s8.txt"
fi
if has pmcv; then
    step pmc_v1 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/pmc_v1" -o s -- python3 tools/probe.py ${PROBE_ARGS:-}
    step pmc_v2 120 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_TCP_TA_ADDR_STALL_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU \
        --output-format csv -d "$OUT/pmc_v2" -o s -- python3 tools/probe.py ${PROBE_ARGS:-}
    python tools/pmc_raw.py "$OUT/pmc_v1" > "$OUT/pmc_v.txt" 2>&1; python tools/pmc_raw.py "$OUT/pmc_v2" >> "$OUT/pmc_v.txt" 2>&1; cat "$OUT/pmc_v.txt"
fi
if has pmcl; then   # lookup variants: L1->L2 request count / latency, L2 hits, fabric request sizes
    step pmc_l1 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/pmc_l1" -o s -- python3 tools/probe.py ${PROBE_ARGS:-}
    step pmc_l2 120 rocprofv3 --pmc TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_HIT TCC_MISS \
        --output-format csv -d "$OUT/pmc_l2" -o s -- python3 tools/probe.py ${PROBE_ARGS:-}
    step pmc_l3 120 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ \
        --output-format csv -d "$OUT/pmc_l3" -o s -- python3 tools/probe.py ${PROBE_ARGS:-}
    { python tools/pmc_raw.py "$OUT/pmc_l1" --width 90; python tools/pmc_raw.py "$OUT/pmc_l2" --width 90;
      python tools/pmc_raw.py "$OUT/pmc_l3" --width 90; } > "$OUT/pmc_l.txt" 2>&1; grep lookup "$OUT/pmc_l.txt"
fi
if has proj; then   # per-rank shapes at N = 1/2/4/8 on one GPU (projection inputs)
    for N in 1 2 4 8; do
        step proj_kitti_$N 300 python bench.py --config kitti --per-rank-of $N --no-cpu-baseline --steps 10 --warmup 3
        step proj_middlebury_$N 300 python bench.py --config middlebury --per-rank-of $N --no-cpu-baseline --steps 5 --warmup 2
    done
fi
has shardt && step pytest_shard 600 python -u -m pytest tests/test_shard_gpu.py -v -rf --timeout 300 --timeout-method thread
# bench.py --gpus 2 without a launcher (self-launch), 2 ranks sharing cuda:0 over gloo
has launch && step launch_gloo2 600 env RAFTCORR_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-backward
has netmb && step net_middlebury_1 600 python bench.py --config middlebury --network --steps 2 --warmup 1 --no-cpu-baseline
has netmb && step net_middlebury_gloo2 900 env RAFTCORR_BENCH_BACKEND=gloo python bench.py --gpus 2 --config middlebury --network --steps 1 --warmup 1 --no-cpu-baseline
has pconv && step shard_probe_perconv 900 python tools/shard_probe.py --perconv
if has shadows; then   # config 2 / 4: level-0 shadow copy and NHWC output re-measured as whole steps
    BQ="--no-cpu-baseline --e2e-steps 0 --no-backward --config4-steps 0 --steps 20 --warmup 5"
    for rep in 1 2; do
        step shadows_sf_default_$rep 300 python bench.py $BQ
        step shadows_sf_02_$rep 300 python bench.py $BQ --shadow 0,2
        step shadows_sf_cl_$rep 300 python bench.py $BQ --channels-last
        step shadows_sf_02cl_$rep 300 python bench.py $BQ --shadow 0,2 --channels-last
        step shadows_mb_default_$rep 300 python bench.py --config middlebury $BQ
        step shadows_mb_02_$rep 300 python bench.py --config middlebury $BQ --shadow 0,2
    done
fi
if has shadowk; then   # config-3 shadow copies re-decided as whole steps
    for rep in 1 2; do
        for SH in default 2 none; do
            step shadowk_b64_${SH}_$rep 300 python bench.py --config kitti --no-cpu-baseline --steps 10 --warmup 3 --shadow $SH
        done
        for SH in default 0,2 none; do
            step shadowk_b8_${SH/,/}_$rep 300 python bench.py --config kitti --per-rank-of 8 --no-cpu-baseline --steps 20 --warmup 5 --shadow $SH
        done
    done
fi
has rtab && step realtime_ab 300 python tools/realtime_ab.py ${RTAB_VARIANTS:-RAFTCORR_LOOKUP_VARIANT=6}
has rtg && step bench_realtime_graph 300 python bench.py --config realtime --graph --no-cpu-baseline --steps 200 --warmup 10
has shard8 && step shard_probe_h8 900 python tools/shard_probe.py --halo 8
has sablr && step build_ablate_realtime 300 python tools/build_ablate.py --config realtime --modes ${SABL_MODES:-0,4096} --rounds 9
has sablm && step build_ablate_middlebury 300 python tools/build_ablate.py --config middlebury --modes ${SABL_MODES:-0,4096} --rounds 5
has sabl && step build_ablate 600 python tools/build_ablate.py --modes ${SABL_MODES:-0,8192} --rounds ${SABL_ROUNDS:-9} ${SABL_CONFIG:+--config $SABL_CONFIG}
has shear && step shear_probe 600 python tools/shear_probe.py
has tdisp && step pytest_disp 600 python -u -m pytest tests/test_disparity_gpu.py tests/test_split_gpu.py tests/test_corr_gpu.py -v -rf --timeout 120 --timeout-method thread
has pdisp && step shear_probe_product 900 python tools/shear_probe.py --product ${SHEAR_ARGS:-}
has gfloor && step graph_floor 300 python tools/graph_floor.py
has train && step train_probe 300 python tools/train_probe.py
has trainmb && step train_probe_middlebury 300 python tools/train_probe.py --config middlebury --reps 3
has lprobe2 && step lookup_probe2 600 python tools/lookup_probe.py --only-dev --dev-variants ${LPROBE_VARIANTS:-205} --dev-fields ${LPROBE_FIELDS:-bench,smooth,net} --reps ${LPROBE_REPS:-7}
if has calib; then   # FETCH_SIZE / WRITE_SIZE per byte for scattered 64-256 B rows
    step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o f \
        -- python3 tools/pmc_calib_random.py
    step calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o w \
        -- python3 tools/pmc_calib_random.py
    python tools/pmc_calib_report.py "$OUT/calib_fetch" "$OUT/calib_write" > "$OUT/calib.txt" 2>&1; cat "$OUT/calib.txt"
fi
if has pmcjson; then   # profiles/pmc.json: three counter passes of bench.py itself per config
    for C in ${PMC_CONFIGS:-sceneflow kitti middlebury realtime}; do
        BA="--config $C --pmc-calibrate --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 --config4-steps 0"
        step pmcj_${C}_f 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcj_${C}_f" -o f -- python3 bench.py $BA
        step pmcj_${C}_w 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcj_${C}_w" -o w -- python3 bench.py $BA
        step pmcj_${C}_s 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
            --output-format csv -d "$OUT/pmcj_${C}_s" -o s -- python3 bench.py $BA
        python tools/pmc_collect.py $C "$OUT/pmcj_${C}_f" "$OUT/pmcj_${C}_w" "$OUT/pmcj_${C}_s" \
            --out "$OUT/pmc.json" --tag "$TAG" > "$OUT/pmcj_${C}.txt" 2>&1; cat "$OUT/pmcj_${C}.txt"
    done
fi
exit 0
