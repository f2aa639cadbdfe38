set -e -o pipefail
O=gpurun_out/ab
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-verify --steps 10 > $O/new_enc_$i.log 2>&1
  CHIP_ZFEC_K4_U1=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-verify --steps 10 > $O/old_enc_$i.log 2>&1
  timeout -k 10 200 python3 bench.py --mode decode --no-cpu-baseline --no-verify --steps 10 > $O/new_dec_$i.log 2>&1
  CHIP_ZFEC_K4_U1=1 timeout -k 10 200 python3 bench.py --mode decode --no-cpu-baseline --no-verify --steps 10 > $O/old_dec_$i.log 2>&1
done
