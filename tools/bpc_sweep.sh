#!/bin/bash
# Workgroups per CU for the zfec shapes (CHIP_ZF_GRID_BPC overrides the
# library's grid), one bench process per setting.  bash tools/bpc_sweep.sh TAG
set -e -o pipefail
O=$PWD/gpurun_out/$1
mkdir -p $O
for cfg in cfg3 cfg2 cfg5; do
  for bpc in 1 2 3 4; do
    CHIP_ZF_GRID_BPC=$bpc timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --no-verify-all --no-aliased --steps 10 > $O/${cfg}_bpc$bpc.log 2>&1
  done
done
