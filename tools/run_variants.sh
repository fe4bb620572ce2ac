#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/var
cp hyrise-1_amd/_lib/libhyrise_amd.so /tmp/orig.so
for v in fma0 fma3 fma4 br0 br3 br4; do
  cp hyrise-1_amd/_lib/variants/libhyrise_amd_$v.so hyrise-1_amd/_lib/libhyrise_amd.so
  timeout -k 10 200 python -u bench.py --workload q1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err || { echo "fail $v"; break; }
  python -c "import json;d=json.load(open('gpurun_out/var/$v.json'));print('$v', d['ms_per_step'], d['roofline']['dominant_ms_per_step'], d['check']['ok'])"
done
cp /tmp/orig.so hyrise-1_amd/_lib/libhyrise_amd.so
