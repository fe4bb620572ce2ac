set -e
R=$GRAFT_REPO_ROOT
for v in "HY_PART_SUB_FILTERED=2" "HY_PART_SUB_FILTERED=3" "HY_PART_SUB_FILTERED=4" "HY_PART_SUB2=2" "HY_PART_SUB1=2" "HY_PART_SUB_FILTERED=4 HY_PART_SUB2=2"; do
  echo "== $v" >> $R/gpurun_out/sweep.txt
  env $v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/sw_tmp.json 2>/dev/null
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/sw_tmp.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], {k:round(v['ms_per_launch'],3) for k,v in d.get('kernels',{}).items() if 'part' in k})" >> $R/gpurun_out/sweep.txt
done
