#!/bin/bash
# The rocprofv3 part of tools/gpu_round.sh alone (kernel stats + FETCH_SIZE /
# WRITE_SIZE passes of the headline bench), with the tuning choices pinned.
#   bash tools/gpu_prof.sh TAG K4_SCHED SPLIT
set -e -o pipefail
TAG=$1; export CHIP_ZFEC_K4_SCHED=$2; export CHIP_ZF_SPLIT=$3
O=$PWD/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "CHIP_ZFEC_K4_SCHED=$CHIP_ZFEC_K4_SCHED CHIP_ZF_SPLIT=$CHIP_ZF_SPLIT" > $O/schedule.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o stats --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-aliased > $O/prof.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-aliased > $O/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-aliased > $O/pmc_write.log 2>&1
echo done > $O/done
