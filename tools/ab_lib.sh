#!/bin/bash
# A/B of two builds of the library on one box, interleaved: the in-tree build
# vs carbonado_amd/lib/libcarbonado_hip_ab.so (a copy of the previous build).
#   bash tools/ab_lib.sh OUTDIR ROUNDS bench-args...
set -e -o pipefail
O=$1; shift
N=$1; shift
mkdir -p $O
for i in $(seq 1 $N); do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $O/new_$i.json 2> $O/new_$i.err
  CARBONADO_HIP_LIB=$PWD/carbonado_amd/lib/libcarbonado_hip_ab.so timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $O/old_$i.json 2> $O/old_$i.err
done
for f in $O/new_*.json $O/old_*.json; do
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['roofline']['avg_launch_ms'], d['verified_object0'])" $f
done
