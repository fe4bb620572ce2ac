set -e
R=$GRAFT_REPO_ROOT
for v in "HY_ONEPASS_WIN=1" "HY_ONEPASS_WIN=4" "HY_ONEPASS_WIN=1 HY_ONEPASS_STATIC=1" "HY_ONEPASS_WIN=4 HY_ONEPASS_STATIC=1" "HY_ONEPASS=0"; do
  echo "== $v" >> $R/gpurun_out/var.txt
  env $v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/var_tmp.json 2>/dev/null
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/var_tmp.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], {k:round(v['ms_per_launch'],3) for k,v in d.get('kernels',{}).items() if 'part1' in k})" >> $R/gpurun_out/var.txt
done
