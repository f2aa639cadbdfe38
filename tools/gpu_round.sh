#!/bin/bash
# One GPU session: parity tests, smoke, bench lines for every mode, rocprofv3
# kernel stats and the FETCH_SIZE / WRITE_SIZE passes for the headline kernel.
# Usage (from the repo root, on the GPU box): bash tools/gpu_round.sh TAG [quick]
set -e -o pipefail
TAG=${1:-r2}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > $O/bench_encode.log 2>&1
timeout -k 10 600 python3 bench.py --config cfg3 --no-cpu-baseline > $O/bench_decode.log 2>&1
timeout -k 10 600 python3 bench.py --config cfg5 --no-cpu-baseline > $O/bench_8of16.log 2>&1
timeout -k 10 600 python3 bench.py --gpus 2 --objects 256 --no-cpu-baseline > $O/bench_2rank_one_gpu.log 2>&1
if [ "$2" != quick ]; then
timeout -k 10 600 python3 bench.py --mode bao --no-cpu-baseline > $O/bench_bao.log 2>&1
timeout -k 10 600 python3 bench.py --mode bao-decode --cpu-seconds 8 > $O/bench_bao_decode.log 2>&1
timeout -k 10 600 python3 bench.py --mode pipeline --level 12 --verify-all > $O/bench_pipe12.log 2>&1
timeout -k 10 600 python3 bench.py --mode e2e --level 15 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_e2e15.log 2>&1
timeout -k 10 600 python3 bench.py --mode e2e --level 12 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_e2e12.log 2>&1
timeout -k 10 600 python3 bench.py --mode e2e-decode --level 15 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_e2ed15.log 2>&1
timeout -k 10 600 python3 bench.py --mode scrub --steps 2 --warmup 1 --cpu-seconds 8 > $O/bench_scrub.log 2>&1
timeout -k 10 600 python3 bench.py --mode hasher --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_hasher.log 2>&1
fi
bash tools/gpu_prof.sh $TAG
echo done > $O/done
