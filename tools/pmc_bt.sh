# PMC passes over tools/bao_tune variants (usage: bash tools/pmc_bt.sh TAG SUBSET)
set -e
O=gpurun_out/${1:-pmcbt}; S=${2:-0,3,8}; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES -d $O/i -o i --output-format csv -- ./tools/bao_tune 256 32 1 $S > $O/i.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM -d $O/j -o j --output-format csv -- ./tools/bao_tune 256 32 1 $S > $O/j.log 2>&1
