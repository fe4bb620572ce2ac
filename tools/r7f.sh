R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
: > $O/g_stress.txt
cfg=${1:-default}
for i in $(seq 1 ${2:-10}); do
  if [ "$cfg" = default ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 120 python -m pytest tests/test_operator_surface_gpu.py -x -q -k "concurrent_operators" -p no:cacheprovider > $O/g_run.txt 2>&1
  rc=$?
  echo "$cfg run $i rc=$rc $(tail -n1 $O/g_run.txt)" >> $O/g_stress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc" >> $O/g_stress.txt; exit 1; fi
  if [ $rc -eq 1 ]; then grep -m3 "^E " $O/g_run.txt >> $O/g_stress.txt; fi
done
