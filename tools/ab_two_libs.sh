#!/bin/bash
# A/B of two library files, alternating processes:
#   bash tools/ab_two_libs.sh TAG ROUNDS LIB_A LIB_B bench-args...
TAG=$1; R=$2; LA=$3; LB=$4; shift 4
O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 $R); do
  for v in a b; do
    if [ $v = a ]; then L=$PWD/$LA; else L=$PWD/$LB; fi
    CARBONADO_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify "$@" > $O/$v.$i.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/$v.$i.log').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['roofline']['frac'])"
  done
done
