#!/bin/bash
# GPU session for the encode() pipeline: parity tests, device-resident level-12
# bench, host-batch E2E level 12 and 15, rocprofv3 kernel stats of the device bench.
set -e -o pipefail
O=gpurun_out/${1:-pipe}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py --mode pipeline --level 12 > $O/bench_pipe12.log 2>&1
timeout -k 10 300 python3 bench.py --mode e2e --level 12 --objects 256 --steps 3 --warmup 1 --cpu-seconds 8 > $O/bench_e2e12.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o stats --output-format csv -- python3 bench.py --mode pipeline --level 12 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
