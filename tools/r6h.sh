set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
for rep in 1 2; do
for cfg in "2 1" "2 0" "3 1" "3 0"; do
  set -- $cfg
  HY_AGG_JIT_WAVES=$1 HY_AGG_JIT_SELECT=$2 timeout -k 10 300 python bench.py --workload q1 --steps 10 --warmup 3 --no-cpu-baseline --op-kernel-stats > $O/q1_w$1_s$2_r$rep.json 2> $O/q1_w$1_s$2_r$rep.err || { echo Q1_FAILED $cfg; tail -5 $O/q1_w$1_s$2_r$rep.err; exit 1; }
done
done
echo ok
