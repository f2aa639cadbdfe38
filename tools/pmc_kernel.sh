#!/bin/bash
# Kernel stats + two PMC passes (instruction mix; waits, LDS conflicts) over
# one bench.py command.  bash tools/pmc_kernel.sh TAG bench-args...
set -e -o pipefail
TAG=$1; shift
O=$PWD/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o stats --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify "$@" > $O/prof.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES -d $O/i -o i --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify "$@" > $O/i.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM -d $O/j -o j --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify "$@" > $O/j.log 2>&1
echo done > $O/pmc_done
