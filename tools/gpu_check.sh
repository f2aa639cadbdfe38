#!/bin/bash
# Quick GPU check: parity tests, smoke, a 2-rank bench rehearsal on one GPU.
# Usage (on the GPU box, from the repo root): bash tools/gpu_check.sh TAG
set -e -o pipefail
O=gpurun_out/${1:-check}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --objects 256 --steps 3 --warmup 1 > $O/bench_2rank.log 2>&1
