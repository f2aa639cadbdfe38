#!/bin/bash
# Sweep the overlapped level-12 pipeline (CHIP_PIPE_PARTS x CHIP_PIPE_K1_WG) with bench.py --mode pipeline.
set -e
O=gpurun_out/${1:-pipe}; mkdir -p $O; export TMPDIR=/tmp
for cfg in ${CFGS:-"1 0" "8 2" "16 2" "32 2" "16 1" "16 3"}; do
  set -- $cfg
  CHIP_PIPE_PARTS=$1 CHIP_PIPE_K1_WG=$2 timeout -k 10 200 python3 bench.py --mode pipeline --level 12 --steps 6 --warmup 2 --no-cpu-baseline > $O/p$1_w$2.log 2>&1
  echo "parts=$1 k1wg=$2 $(grep -o '"value": [0-9.]*' $O/p$1_w$2.log) $(grep -o '"verified_object0": [a-z]*' $O/p$1_w$2.log)" >> $O/summary.txt
done
