#!/bin/bash
# E2E encode() level 12 from pinned host memory: slots x slice size sweep.
#   bash tools/e2e_sweep.sh OUTDIR
set -e -o pipefail
O=$1
mkdir -p $O
for cfg in "3 256" "2 256" "4 256" "3 128" "3 512" "4 128" "6 128"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --mode e2e --level 12 --objects 256 --steps 3 --warmup 1 --no-cpu-baseline \
    --slots $1 --slice-mib $2 > $O/s$1_m$2.json 2> $O/s$1_m$2.err
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['roofline']['achieved'], d['verified_object0'])" $O/s$1_m$2.json
done
