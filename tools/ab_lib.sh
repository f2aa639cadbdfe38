#!/bin/bash
# A/B of two library builds (abtest/libcarbonado_hip_old.so = the baseline build,
# the in-tree library = the candidate), alternating processes: bash tools/ab_lib.sh TAG ROUNDS bench-args...
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 $R); do
  for v in old new; do
    if [ $v = old ]; then L=$PWD/abtest/libcarbonado_hip_old.so; else L=$PWD/carbonado_amd/lib/libcarbonado_hip.so; fi
    CARBONADO_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify "$@" > $O/$v.$i.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/$v.$i.log').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['roofline']['frac'])"
  done
done
