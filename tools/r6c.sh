# direct-path experiments: span size and the digit-byte stream (kernel traces only; NOBYTES output is invalid)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r6c
mkdir -p $O
cd /tmp
for cfg in "16 0" "8 0" "32 0" "16 1"; do
  set -- $cfg
  tag=s$1_nb$2
  if [ "$2" = 1 ]; then export HY_DIRECT_NOBYTES=1; else unset HY_DIRECT_NOBYTES; fi
  HY_DIRECT_SPAN=$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run -f csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || echo "run $tag rc=$?"
done
echo done
