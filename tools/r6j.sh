set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_join_gpu.py -x -q --capture=sys --timeout 300 --timeout-method thread -k "multi or large or skew or partition" > $O/tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
timeout -k 10 300 python bench.py --workload join-only --steps 10 --warmup 3 --no-cpu-baseline --op-kernel-stats > $O/joinonly_$r.json 2> $O/joinonly_$r.err || { echo JO_FAILED; tail -20 $O/joinonly_$r.err; exit 1; }
done
timeout -k 10 600 python bench.py --through-operators --steps 5 --warmup 2 > $O/ops.json 2> $O/ops.err || { echo OPS_FAILED; tail -20 $O/ops.err; exit 1; }
echo ok
