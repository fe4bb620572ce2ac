#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 run per counter group, as gfx950 requires), restricted to the
# framework's kernels. usage: tools/pmc_probe.sh <out-dir under gpurun_out> <kernel regex> [bench args]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
RE=$2
shift 2
ARGS=${*:-"--steps 2 --warmup 1 --no-cpu-baseline"}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for c in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$RE" -d "$OUT/p$i" -o run -f csv -- \
    python3 "$R/bench.py" $ARGS > "$OUT/bench_p$i.json" 2> "$OUT/p$i.err"
done
python3 "$R/tools/pmc_table.py" "$OUT" | tee "$OUT/table.txt"
