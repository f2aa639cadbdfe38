#!/bin/bash
# A/B of one library build under two environments, interleaved on one box:
#   bash tools/ab_env.sh OUTDIR ROUNDS "ENV_A" "ENV_B" bench-args...
# e.g. bash tools/ab_env.sh gpurun_out/split 3 "CHIP_ZF_SPLIT=0" "CHIP_ZF_SPLIT=1" --mode decode
set -e -o pipefail
O=$1; N=$2; A=$3; B=$4; shift 4
mkdir -p $O
for i in $(seq 1 $N); do
  env $A timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $O/a_$i.json 2> $O/a_$i.err
  env $B timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $O/b_$i.json 2> $O/b_$i.err
done
echo "A: $A   B: $B   args: $*"
for f in $O/a_*.json $O/b_*.json; do
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[1], d['value'], r['frac'], r['avg_launch_ms'], d['verified_object0'], (d.get('aliased_data_shards') or {}).get('value'))" $f
done
