#!/bin/bash
# One GPU session: parity tests, bench lines for every mode, rocprofv3 kernel
# stats and the FETCH_SIZE / WRITE_SIZE passes for the headline kernel.
# Usage (from the repo root, on the GPU box): bash tools/gpu_round.sh TAG
set -e -o pipefail
TAG=${1:-r1}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python3 bench.py --verify-all > $O/bench_encode.log 2>&1
timeout -k 10 600 python3 bench.py --mode decode --no-cpu-baseline > $O/bench_decode.log 2>&1
timeout -k 10 600 python3 bench.py --k 8 --m 16 --no-cpu-baseline > $O/bench_8of16.log 2>&1
timeout -k 10 600 python3 bench.py --mode bao --no-cpu-baseline > $O/bench_bao.log 2>&1
timeout -k 10 600 python3 bench.py --mode bao-decode --cpu-seconds 8 > $O/bench_bao_decode.log 2>&1
timeout -k 10 600 python3 bench.py --mode pipeline --level 12 --verify-all > $O/bench_pipe12.log 2>&1
timeout -k 10 600 python3 bench.py --mode e2e --level 15 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_e2e15.log 2>&1
timeout -k 10 600 python3 bench.py --mode e2e --level 12 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_e2e12.log 2>&1
timeout -k 10 600 python3 bench.py --mode e2e-decode --level 15 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_e2ed15.log 2>&1
timeout -k 10 600 python3 bench.py --mode scrub --steps 2 --warmup 1 --cpu-seconds 8 > $O/bench_scrub.log 2>&1
timeout -k 10 600 python3 bench.py --mode hasher --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_hasher.log 2>&1
# the profiles run the 4-of-8 schedule and the one-launch/two-halves choice
# the encode line picked on this box, so that every profiled launch is a
# whole-batch launch of that kernel (the first large batches of a process
# otherwise tune on slices of themselves)
export CHIP_ZFEC_K4_SCHED=$(python3 -c "import json,sys; ls=[l for l in open(sys.argv[1]) if l.startswith('{')]; print(json.loads(ls[-1])['roofline']['schedule']['k4'])" $O/bench_encode.log)
export CHIP_ZF_SPLIT=$(python3 -c "import json,sys; ls=[l for l in open(sys.argv[1]) if l.startswith('{')]; print(max(0, json.loads(ls[-1])['roofline']['schedule']['split']))" $O/bench_encode.log)
echo "CHIP_ZFEC_K4_SCHED=$CHIP_ZFEC_K4_SCHED CHIP_ZF_SPLIT=$CHIP_ZF_SPLIT" > $O/schedule.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o stats --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-aliased > $O/prof.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-aliased > $O/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-aliased > $O/pmc_write.log 2>&1
echo done > $O/done
