set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_bao2
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/p1 -o p1 --output-format csv -- $R/tools/bao_tune 128 32 1 0,7 > $O/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR -d $O/p2 -o p2 --output-format csv -- $R/tools/bao_tune 128 32 1 0,7 > $O/p2.log 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_WRITE_WAVEFRONTS_sum -d $O/p3 -o p3 --output-format csv -- $R/tools/bao_tune 128 32 1 0,7 > $O/p3.log 2>&1 || true
echo done > $O/done
