#!/bin/bash
# SQ counters of the kernels matching a regex (two passes, each within the per-block counter limits) over a short
# bench.py run. usage: tools/pmc_sq.sh <tag> <kernel regex> [bench.py args]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-scan}
RX=${2:-hyk::}
shift 2 || true
export TMPDIR=/tmp
O=$R/gpurun_out/pmc_sq_$TAG
mkdir -p $O
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAVES --kernel-include-regex "$RX" -d $O/a -o run -f csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/a.json 2> $O/a.err
timeout -s KILL 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$RX" -d $O/b -o run -f csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err
python3 $R/tools/pmc_table.py $O > $R/gpurun_out/${TAG}_pmc_sq.txt
echo done
