#!/bin/bash
# The rocprofv3 part of tools/gpu_round.sh alone: kernel stats of the
# headline bench, then FETCH_SIZE and WRITE_SIZE in passes of their own.
#   bash tools/gpu_prof.sh TAG [bench args...]
set -e -o pipefail
TAG=$1; shift
O=$PWD/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o stats --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-aliased --live-pmc off "$@" > $O/prof.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-aliased --no-box-ceiling --live-pmc off "$@" > $O/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-aliased --no-box-ceiling --live-pmc off "$@" > $O/pmc_write.log 2>&1
echo done > $O/prof_done
