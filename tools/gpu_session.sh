#!/bin/bash
# A GPU session of named steps, each under its own time limit, stopping at
# the first failure.  bash tools/gpu_session.sh TAG step...
#   steps: tests smoke encode decode 8of16 2rank bao baodec pipe12 pdec12 pdec4 pdec8 e2e15 e2e15full
#          e2e12 e2ed15 e2edab seg1m prof1m k13fetch ecbench gcmab fileab e2edsweep stageab abilat topquadab soffab soffe2e baoab baodecab pdecab scrubbab ftsoff crcab upperab prepab scrub scrubb hasher file15 file12 prof pipe12l15 encodetorch mixprobe ftune ftunepmc valuprobe numaprobe baotune baotunepmc hasher3 valupk hasherva hashercopy hasherbind h2dprobe hashercache prof12 prof15s profbao profbaodec profpdec splitab streamab ntab ntab3 directab hostprobe slicesweep e2e3 e2eprof e2ed15full sdmaab
set -e -o pipefail
TAG=$1; shift
O=$PWD/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; }
for s in "$@"; do
  case $s in
    tests) run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    encode) run bench_encode 600 python3 bench.py ;;
    decode) run bench_decode 600 python3 bench.py --config cfg3 --no-cpu-baseline ;;
    8of16) run bench_8of16 600 python3 bench.py --config cfg5 --no-cpu-baseline ;;
    2rank) run bench_2rank_one_gpu 600 python3 bench.py --gpus 2 --objects 256 ;;
    bao) run bench_bao 600 python3 bench.py --mode bao --no-cpu-baseline ;;
    baodec) run bench_bao_decode 600 python3 bench.py --mode bao-decode --cpu-seconds 8 ;;
    pipe12) run bench_pipe12 600 python3 bench.py --mode pipeline --level 12 --verify-all ;;
    pipe12l15) run bench_pipe12_l15shape 600 python3 bench.py --mode pipeline --level 12 --object-bytes 16779371 --verify-all ;;
    pdec12) run bench_pdec12 600 python3 bench.py --mode pipeline-decode --level 12 ;;
    pdec4) run bench_pdec4 600 python3 bench.py --mode pipeline-decode --level 4 ;;
    pdec8) run bench_pdec8 600 python3 bench.py --mode pipeline-decode --level 8 ;;
    pipe12old) CHIP_FUSED=0 run bench_pipe12_twokernel 600 python3 bench.py --mode pipeline --level 12 --no-cpu-baseline ;;
    e2e15) run bench_e2e15 600 python3 bench.py --mode e2e --level 15 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 ;;
    e2e15full) run bench_e2e15_full 900 python3 bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 8 ;;
    e2e12) run bench_e2e12 600 python3 bench.py --mode e2e --level 12 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 ;;
    e2ed15) run bench_e2ed15 600 python3 bench.py --mode e2e-decode --level 15 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 ;;
    scrub) run bench_scrub 600 python3 bench.py --mode scrub --steps 2 --warmup 1 --cpu-seconds 8 ;;
    scrubb) run bench_scrub_batch 600 python3 bench.py --mode scrub-batch --steps 5 --warmup 1 --cpu-seconds 8 ;;
    hasher) run bench_hasher 600 python3 bench.py --mode hasher --steps 3 --warmup 1 --cpu-seconds 8 ;;
    hasher3) for i in 1 2 3; do run bench_hasher_numa_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; CHIP_NUMA=0 run bench_hasher_nonuma_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; done ;;
    file15) run bench_file15 600 python3 bench.py --mode file --level 15 --steps 3 --warmup 1 --cpu-seconds 8 ;;
    file12) run bench_file12 600 python3 bench.py --mode file --level 12 --steps 3 --warmup 1 --no-cpu-baseline ;;
    prof) bash tools/gpu_prof.sh $TAG ;;
    prof12) bash tools/gpu_prof.sh $TAG/p12 --mode pipeline --level 12 ;;
    prof15s) bash tools/gpu_prof.sh $TAG/p15s --mode pipeline --level 12 --object-bytes 16779371 ;;
    profbao) bash tools/gpu_prof.sh $TAG/pbao --mode bao ;;
    profbaodec) bash tools/gpu_prof.sh $TAG/pbaodec --mode bao-decode ;;
    profpdec) bash tools/gpu_prof.sh $TAG/ppdec --mode pipeline-decode --level 12 ;;
    encodetorch) run bench_encode_alloc_torch 600 python3 bench.py --alloc torch --no-cpu-baseline --live-pmc off ;;
    mixprobe) run mix_probe_bal 300 ./tools/mix_probe 1024 3 bal ;;
    ftune) run fused_tune 300 ./tools/fused_tune 256 5 ;;
    ftunepmc) run fused_tune_pmc 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU -d $O/ftpmc -o ftpmc --output-format csv -- ./tools/fused_tune 256 1 ;;
    baotune) run bao_tune 300 ./tools/bao_tune 256 32 5 ;;
    baotunepmc) run bao_tune_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $O/btpmc -o btpmc --output-format csv -- ./tools/bao_tune 256 32 1 1,3 ;;
    numaprobe) run numa_probe 120 python3 tools/numa_probe.py ;;
    hasherva) for i in 1 2 3; do run bench_hasher_va_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; CHIP_HASHER_VA=0 run bench_hasher_nova_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; done ;;
    hashercopy) for i in 1 2; do run bench_hasher_nt_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; CHIP_NT_COPY=0 run bench_hasher_memcpy_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; CHIP_COPY_THREADS=16 run bench_hasher_nt_t16_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; CHIP_HOST_COPY=direct run bench_hasher_direct_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; done ;;
    hasherbind) for i in 1 2; do run bench_hasher_bind_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; run bench_hasher_nobind_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline --no-numa-bind; done ;;
    h2dprobe) run h2d_probe 300 python3 tools/h2d_probe.py ;;
    hashercache) for i in 1 2 3; do run bench_hasher_cache_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; CHIP_HASHER_CACHE=0 run bench_hasher_nocache_$i 300 python3 bench.py --mode hasher --steps 3 --warmup 1 --no-cpu-baseline; done ;;
    splitab) CHIP_E2E_SPLIT=0 run bench_e2e15_full_nosplit 900 python3 bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline
             run bench_e2e12_split 600 python3 bench.py --mode e2e --level 12 --objects 256 --steps 3 --warmup 1 --no-cpu-baseline
             CHIP_E2E_SPLIT=0 run bench_e2e12_nosplit 600 python3 bench.py --mode e2e --level 12 --objects 256 --steps 3 --warmup 1 --no-cpu-baseline ;;
    streamab) CHIP_STREAM_ENCRYPT=0 run bench_e2e15_full_twopass 900 python3 bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline
              run bench_e2ed15 600 python3 bench.py --mode e2e-decode --level 15 --objects 256 --steps 3 --warmup 1 --no-cpu-baseline ;;
    ntab) CHIP_NT_STAGE=0 run bench_e2e15_full_ntstage0 900 python3 bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline
          run bench_e2e15_full_slice272 900 python3 bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline --slice-mib 272 ;;
    ntab3) for i in 1 2 3; do run bench_e2e15_nt_$i 300 python3 bench.py --config cfg4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify --slice-mib 272
                             CHIP_NT_STAGE=0 run bench_e2e15_plain_$i 300 python3 bench.py --config cfg4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify --slice-mib 272; done ;;
    directab) for i in 1 2 3; do run bench_e2e15_direct_$i 300 python3 bench.py --config cfg4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify --slice-mib 272
                                CHIP_E2E_DIRECT=0 run bench_e2e15_staged_$i 300 python3 bench.py --config cfg4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify --slice-mib 272; done ;;
    hostprobe) run host_encode_probe 300 ./tools/host_encode_probe 16 4 ;;
    slicesweep) for i in 1 2; do for cfg in "272 3" "544 3" "272 4" "544 2" "1088 2"; do set -- $cfg
                  run bench_e2e15_s$1_k$2_$i 300 python3 bench.py --config cfg4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify --slice-mib $1 --slots $2; done; done ;;
    e2e3) for i in 1 2 3; do run bench_e2e15_team_$i 300 python3 bench.py --config cfg4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify; done ;;
    e2eprof) run e2e15_copy_trace 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/e2eprof -o e2e --output-format csv -- python3 bench.py --config cfg4 --objects 256 --steps 3 --warmup 1 --no-cpu-baseline --no-verify ;;
    sdmaab) for i in 1 2; do HSA_ENABLE_SDMA=0 run bench_e2e15_nosdma_$i 300 python3 bench.py --config cfg4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify
                             run bench_e2e15_sdma_$i 300 python3 bench.py --config cfg4 --steps 6 --warmup 2 --no-cpu-baseline --no-verify; done ;;
    e2ed15full) run bench_e2ed15_full 600 python3 bench.py --mode e2e-decode --level 15 --steps 3 --warmup 1 --cpu-seconds 8 ;;
    e2edab) for i in 1 2; do run bench_e2ed15_full_prefix_$i 400 python3 bench.py --mode e2e-decode --level 15 --steps 4 --warmup 1 --no-cpu-baseline
                           CHIP_DECODE_PREFIX=0 run bench_e2ed15_full_whole_$i 400 python3 bench.py --mode e2e-decode --level 15 --steps 4 --warmup 1 --no-cpu-baseline; done ;;
    seg1m) run bench_e2e15_1mib 600 python3 bench.py --mode e2e --level 15 --object-bytes 1048576 --objects 16384 --steps 3 --warmup 1 --cpu-seconds 8
           run bench_e2ed15_1mib 600 python3 bench.py --mode e2e-decode --level 15 --object-bytes 1048576 --objects 16384 --steps 3 --warmup 1 --no-cpu-baseline
           run bench_pipe12_1mib_l15shape 600 python3 bench.py --mode pipeline --level 12 --object-bytes 1048811 --objects 16384 --verify-all --no-cpu-baseline
           run bench_pipe12_1mib 600 python3 bench.py --mode pipeline --level 12 --object-bytes 1048576 --objects 16384 --verify-all --no-cpu-baseline ;;
    prof1m) bash tools/gpu_prof.sh $TAG/p1m --mode pipeline --level 12 --object-bytes 1048811 --objects 16384 ;;
    k13fetch) run k13_fetch 200 ./tools/k13_fetch 256 5 ;;
    soffab) for i in 1 2; do for o in 0 56; do
              run bench_pipe12_soff${o}_$i 300 python3 bench.py --mode pipeline --level 12 --no-cpu-baseline --stream-offset $o
              run bench_pipe12_l15shape_soff${o}_$i 300 python3 bench.py --mode pipeline --level 12 --object-bytes 16779371 --no-cpu-baseline --stream-offset $o
              run bench_pipe12_1mib_l15shape_soff${o}_$i 300 python3 bench.py --mode pipeline --level 12 --object-bytes 1048811 --objects 16384 --no-cpu-baseline --stream-offset $o
            done; done ;;
    soffe2e) for i in 1 2; do run bench_e2e15_full_soff0_$i 400 python3 bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu-baseline --no-verify
                           CHIP_STREAM_OFFSET=56 run bench_e2e15_full_soff56_$i 400 python3 bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu-baseline $([ $i = 1 ] || echo --no-verify); done ;;
    baoab) for i in 1 2; do run bench_bao_soff0_$i 300 python3 bench.py --mode bao --no-cpu-baseline
                          run bench_bao_soff56_$i 300 python3 bench.py --mode bao --no-cpu-baseline --bao-stream-offset 56; done ;;
    baodecab) for i in 1 2; do run bench_bao_decode_soff0_$i 300 python3 bench.py --mode bao-decode --no-cpu-baseline --bao-stream-offset 0
                          run bench_bao_decode_soff56_$i 300 python3 bench.py --mode bao-decode --no-cpu-baseline --bao-stream-offset 56; done ;;
    pdecab) for i in 1 2; do run bench_pdec12_soff0_$i 300 python3 bench.py --mode pipeline-decode --level 12 --no-cpu-baseline --stream-offset 0
                           run bench_pdec12_soff56_$i 300 python3 bench.py --mode pipeline-decode --level 12 --no-cpu-baseline --stream-offset 56; done ;;
    scrubbab) for i in 1 2; do run bench_scrub_batch_soff0_$i 300 python3 bench.py --mode scrub-batch --steps 5 --warmup 1 --no-cpu-baseline --stream-offset 0
                           run bench_scrub_batch_soff56_$i 300 python3 bench.py --mode scrub-batch --steps 5 --warmup 1 --no-cpu-baseline --stream-offset 56; done ;;
    ftsoff) for o in 0 56 0 56; do FT_SOFF=$o run fused_tune_soff${o}_$RANDOM 300 ./tools/fused_tune 256 5 "product"; done
            for o in 0 56; do FT_SOFF=$o run fused_tune_dg_soff$o 300 ./tools/fused_tune 256 5 "K0 DG"; done ;;
    crcab) run host_encode_probe 300 ./tools/host_encode_probe 16 4
           for i in 1 2; do run bench_e2e15_full_crc3_$i 400 python3 bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu-baseline --no-verify
                           CHIP_CRC_CHAINS=1 run bench_e2e15_full_crc1_$i 400 python3 bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu-baseline --no-verify
                           run bench_e2ed15_full_crc3_$i 400 python3 bench.py --mode e2e-decode --level 15 --steps 4 --warmup 1 --no-cpu-baseline $([ $i = 1 ] || echo --no-verify)
                           CHIP_CRC_CHAINS=1 run bench_e2ed15_full_crc1_$i 400 python3 bench.py --mode e2e-decode --level 15 --steps 4 --warmup 1 --no-cpu-baseline --no-verify; done ;;
    gcmab) for g in openssl vaes; do CHIP_GCM=$g run host_encode_probe_gcm_$g 300 ./tools/host_encode_probe 16 4; done
           for i in 1 2; do for g in openssl vaes; do V=--no-verify; [ $i = 1 ] && [ $g = vaes ] && V=
             CHIP_GCM=$g run bench_e2e15_gcm_${g}_$i 400 python3 bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu-baseline $V
             CHIP_GCM=$g run bench_e2ed15_gcm_${g}_$i 400 python3 bench.py --mode e2e-decode --level 15 --steps 4 --warmup 1 --no-cpu-baseline $V
           done; done ;;
    fileab) for i in 1 2; do for sl in 64 32 16; do for io in 8 16; do
              run bench_file15_sl${sl}_io${io}_$i 300 python3 bench.py --mode file --level 15 --steps 3 --warmup 1 --no-cpu-baseline --file-slice $sl --io-threads $io
            done; done; done ;;
    e2edsweep) for i in 1 2; do for sl in 3 4; do for mib in 256 512 1024; do
                 run bench_e2ed15_s${sl}_m${mib}_$i 300 python3 bench.py --mode e2e-decode --level 15 --steps 4 --warmup 1 --no-cpu-baseline --no-verify --slots $sl --slice-mib $mib
               done; done; done ;;
    stageab) for i in 1 2 3 4; do for t in 1 8; do
               CHIP_STAGE_THREADS=$t run latency_stage${t}_$i 300 python3 tools/latency_probe.py 60 ${STAGE_LEVELS:-15,3} 1048576,4194304
             done; done ;;
    abilat) run abi_latency 300 ./tools/abi_latency 50 ;;
    abilat6) run abi_latency_patch 400 ./tools/abi_latency 40 12,4,8,15 1024,1048576,16777216 ;;
    kmtests) run pytest_km 600 python3 -u -m pytest tests/test_gpu_km.py tests/test_gpu_reroute.py tests/test_gpu_small.py tests/test_gpu_pipeline.py tests/test_gpu_bao.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    kmab) for i in 1 2; do for km in 1 0; do CHIP_KM=$km run abi_latency_km${km}_$i 300 ./tools/abi_latency 40 ${KM_LEVELS:-12,4} ${KM_SIZES:-65536,262144,1048576,4194304}; done; done ;;
    thp9) cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $O/thp_setting.txt 2>&1 || true
          for i in 1 2; do for t in 1 0; do CHIP_OUT_THP=$t run abi_latency_thp9_${t}_$i 300 ./tools/abi_latency 12 9,8 16777216; done; done ;;
    kmz) run pytest_kmz 600 python3 -u -m pytest tests/test_gpu_km.py tests/test_gpu_zfec.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    stg9) for km in 1 0; do CHIP_KM=$km ABI_LAT_STAGES=1 CHIP_SINGLE_TRACE=1 run patch_stages_km$km 120 ./tools/abi_latency 4 9,15 16777216,1048576; done ;;
    thp15) for i in 1 2; do for t in 1 0; do CHIP_OUT_THP=$t run abi_latency_thp15_${t}_$i 300 ./tools/abi_latency 8 15,9,12 16777216,1048576; done; done ;;
    zcthr) for i in 1 2; do for t in 8 1 2 4; do CHIP_ZC_THREADS=$t run abi_latency_zcthr${t}_$i 300 ./tools/abi_latency 30 12,4,8 1048576,4194304; done; done
           for t in 1 8; do CHIP_ZC_THREADS=$t CHIP_SINGLE_TRACE=1 run zcthr_trace$t 120 ./tools/abi_latency 6 12 1048576; done ;;
    kmstage) for i in 1 2; do for st in 1 0; do CHIP_KM_STAGE=$st run abi_latency_stage${st}_$i 300 ./tools/abi_latency 30 12,4 66560,262144,1048576,4194304,16777216; done; done
             for st in 1 0; do CHIP_KM_STAGE=$st run timeline_stage$st 300 rocprofv3 --kernel-trace --stats -d $O/tlst$st -o tl --output-format csv -- ./tools/abi_latency 10 12,4 1048576; done ;;
    abold) for i in 1 2; do run abi_latency_new_$i 300 ./tools/abi_latency 30 12,15,4 1048576,4194304
                             LD_LIBRARY_PATH=$PWD/tools/oldlib run abi_latency_old_$i 300 ./tools/abi_latency 30 12,15,4 1048576,4194304; done ;;
    tr15) CHIP_SINGLE_TRACE=1 run trace15_new 120 ./tools/abi_latency 8 15 1048576
          CHIP_SINGLE_TRACE=1 LD_LIBRARY_PATH=$PWD/tools/oldlib run trace15_old 120 ./tools/abi_latency 8 15 1048576 ;;
    singleprof) run single_kernels 300 rocprofv3 --kernel-trace --stats -d $O/sp -o sp --output-format csv -- ./tools/abi_latency 10 12,4,8,15 1024,1048576,4194304 ;;
    ptiles) for i in 1 2; do for t in 4 1 2 8; do CHIP_PARITY_TILES=$t run abi_latency_ptiles${t}_$i 300 ./tools/abi_latency 30 12,8 262144,1048576,4194304; done; done
            for t in 4 1; do CHIP_PARITY_TILES=$t run ptiles_kernels$t 300 rocprofv3 --kernel-trace --stats -d $O/pt$t -o pt --output-format csv -- ./tools/abi_latency 10 12,8 1048576; done ;;
    pdma) for i in 1 2; do for d in 1 0; do CHIP_KM_PARITY_DMA=$d run abi_latency_pdma${d}_$i 300 ./tools/abi_latency 30 12,14 262144,1048576,4194304,16777216; done; done
          CHIP_SINGLE_TRACE=1 run pdma_trace 120 ./tools/abi_latency 6 12 1048576 ;;
    ksmax) for i in 1 2; do for m in 64 128 256; do CHIP_KS_SINGLE_MAX=$m run abi_latency_ksmax${m}_$i 300 ./tools/abi_latency 30 12,4 49152,65536,131072,262144; done; done ;;
    pearly) for i in 1 2; do for e in 262144 0 99999999; do CHIP_KM_PARITY_EARLY=$e run abi_latency_pearly${e}_$i 300 ./tools/abi_latency 30 12,14 66560,131072,262144,524288,1048576,4194304; done; done ;;
    peertab) for i in 1 2; do for t in 1 0; do CHIP_PEER_TABLES=$t run abi_latency_peertab${t}_$i 300 ./tools/abi_latency 30 15,13,9 1024,16384,1048576; done; done ;;
    zdtl) CHIP_SINGLE_TRACE=1 run zfec_decode_trace 120 ./tools/abi_latency 10 8 1048576 ;;
    kmtl) CHIP_SINGLE_TRACE=1 run km_single_trace 120 ./tools/abi_latency 10 12,4 1048576
          run timeline_km_1m 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/tlkm -o tl --output-format csv -- ./tools/abi_latency 10 12,4 1048576 ;;
    kmsg) for sg in 16 32; do CHIP_KM_SG=$sg run pytest_km_sg$sg 300 python3 -u -m pytest tests/test_gpu_km.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread; done ;;
    sgab) for i in 1 2; do for sg in 64 32 16; do CHIP_KM_SG=$sg run abi_latency_sg${sg}_$i 300 ./tools/abi_latency 40 12,4 262144,1048576,4194304; done; done
          CHIP_SINGLE_TRACE=1 run km_single_trace 120 ./tools/abi_latency 10 12 1048576 ;;
    zctests) run pytest_zc 600 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_written.py tests/test_gpu_zfec.py tests/test_gpu_km.py tests/test_gpu_reroute.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    thpout) cat /sys/kernel/mm/transparent_hugepage/enabled > $O/thp_setting.txt 2>&1 || true
            for i in 1 2; do for t in 1 0; do CHIP_OUT_THP=$t run abi_latency_outthp${t}_$i 300 ./tools/abi_latency 12 12,4,8 4194304,16777216; done; done ;;
    latency) run bench_latency 900 python3 bench.py --mode latency ;;
    latencyq) run bench_latency_quick 300 python3 bench.py --mode latency --latency-levels 12,4 --latency-sizes 1048576 --latency-reps 20 ;;
    r6tests) run pytest_r6 600 python3 -u -m pytest tests/test_gpu_reroute.py tests/test_gpu_rccl.py tests/test_gpu_small.py tests/test_gpu_scrub.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    timeline1m) run timeline_1m 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/tl -o tl --output-format csv -- ./tools/abi_latency 20 12 1048576 ;;
    topquadab) for i in 1 2; do for tq in 0 1; do CHIP_TOP_QUAD=$tq run abi_latency_tq${tq}_$i 300 ./tools/abi_latency 50; done; done ;;
    upperab) for i in 1 2; do for u in 1 0; do
               CHIP_UPPER_PASS=$u run bench_pipe12_1mib_up${u}_$i 300 python3 bench.py --mode pipeline --level 12 --object-bytes 1048576 --objects 16384 --no-cpu-baseline
               CHIP_UPPER_PASS=$u run bench_pipe12_1mib_l15shape_up${u}_$i 300 python3 bench.py --mode pipeline --level 12 --object-bytes 1048811 --objects 16384 --no-cpu-baseline
             done; done ;;
    ecbench) run ec_bench 120 bash -c 'echo T 20 | ./tools/secp_field_check' && run ecies_rate 120 ./tools/ecies_rate 16 2000 ;;
    prepab) for i in 1 2; do V=--no-verify; [ $i = 1 ] && V=
            CHIP_E2E_TRACE=1 run bench_e2e15_1mib_prep_$i 400 python3 bench.py --mode e2e --level 15 --object-bytes 1048576 --objects 16384 --steps 4 --warmup 1 --no-cpu-baseline $V
            CHIP_E2E_TRACE=1 CHIP_ECIES_PREP=0 run bench_e2e15_1mib_noprep_$i 400 python3 bench.py --mode e2e --level 15 --object-bytes 1048576 --objects 16384 --steps 4 --warmup 1 --no-cpu-baseline --no-verify
            CHIP_E2E_TRACE=1 run bench_e2e15_full_$i 400 python3 bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu-baseline $V; done ;;
    e2e14) run bench_e2e14 300 python3 bench.py --mode e2e --level 14 --objects 512 --steps 4 --warmup 1 --no-cpu-baseline
           CHIP_E2E_DIRECT=0 run bench_e2e14_staged 300 python3 bench.py --mode e2e --level 14 --objects 512 --steps 4 --warmup 1 --no-cpu-baseline --no-verify ;;
    valupk) run valu_probe_pk 300 ./tools/valu_probe 40000 pk ;;
    valuprobe) run valu_probe_b3x2 300 ./tools/valu_probe 40000 b3x2 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done > $O/done
