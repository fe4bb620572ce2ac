#!/bin/bash
# round-3 GPU check U: headline span-size A/B (pass-0 spans of the unfiltered / filtered side, record-pass spans)
mkdir -p gpurun_out
for cfg in "1 1 2" "2 1 2" "1 2 2" "1 1 4" "2 2 4"; do
  set -- $cfg
  HY_PART_SUB1=$1 HY_PART_SUB2=$2 HY_PART_SUB_FILTERED=$3 timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3u_s$1_$2_$3.json 2> gpurun_out/r3u_s$1_$2_$3.err || exit 1
done
