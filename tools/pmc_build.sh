set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcb
mkdir -p $O
cd $R
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $O/a -o a -- python3 tools/build_probe.py --modes 0,32,44,47 > $O/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --output-format csv -d $O/b -o b -- python3 tools/build_probe.py --modes 0,32,44,47 > $O/b.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/c -o c -- python3 tools/build_probe.py --modes 0,32,44,47 > $O/c.log 2>&1
for x in a b c; do python3 tools/pmc_raw.py $O/$x --width 90 > $O/$x.txt; done
