set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_bao
mkdir -p $O
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/p1 -o p1 --output-format csv -- $R/tools/bao_tune 128 32 1 3,6 > $O/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES -d $O/p2 -o p2 --output-format csv -- $R/tools/bao_tune 128 32 1 3,6 > $O/p2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $O/p3 -o p3 --output-format csv -- $R/tools/bao_tune 128 32 1 3,6 > $O/p3.log 2>&1
timeout -k 10 120 rocprofv3 --pmc VALUBusy VALUUtilization -d $O/p4 -o p4 --output-format csv -- $R/tools/bao_tune 128 32 1 3,6 > $O/p4.log 2>&1
echo done > $O/done
