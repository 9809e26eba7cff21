#!/bin/bash
# Reference-chain ensemble for the at-scale PSNR bar (TEST INFRASTRUCTURE, CPU, this container):
# the CPU chain of scripts/psnr_at_scale.py from initialisations perturbed by 1e-6 with seeds
# 6..12 (seed 5 is the fixture's own perturbed run), 2DGS at 0.3x and 3DGS at 0.1x the fine-stage
# learning rates; two runs at a time, 4 threads each (the fixture's own thread count).
# Outputs tests/golden/psnr_ensemble/{2d,3d}_seed<N>.json; scripts/psnr_ensemble.py merges them.
cd "$(dirname "$0")/.."
jobs=""
for s in 6 7 8 9 10 11 12; do jobs="$jobs 2d:0.3:$s 3d:0.1:$s"; done
echo $jobs | tr ' ' '\n' | xargs -P 2 -I{} bash -c '
  IFS=: read gs lr s <<< "{}"
  out=tests/golden/psnr_ensemble/${gs}_seed${s}.json
  [ -s "$out" ] && exit 0
  OMP_NUM_THREADS=4 nice -n 19 python scripts/psnr_at_scale.py --gs $gs --lr-scale $lr --perturb-seed $s --out $out \
     > /tmp/psnr_ens_${gs}_${s}.log 2>&1'
