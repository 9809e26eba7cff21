#!/bin/bash
# Reference-chain ensemble at the unscaled fine-stage rates (3DGS, lr_scale 1; TEST
# INFRASTRUCTURE, CPU, this container): the CPU chain of scripts/psnr_at_scale.py from
# initialisations perturbed by 1e-6 with seeds 6..11 (seed 5 is the fixture's own perturbed
# run), two at a time, 4 threads each.  Outputs tests/golden/psnr_ensemble/3d_lr1_seed<N>.json;
# scripts/psnr_ensemble.py --gs 3d --fixture psnr_scale_3d_lr1 --prefix 3d_lr1 merges them.
cd "$(dirname "$0")/.."
for s in 6 7 8 9 10 11; do echo $s; done | xargs -P ${P:-2} -I{} bash -c '
  out=tests/golden/psnr_ensemble/3d_lr1_seed{}.json
  [ -s "$out" ] && exit 0
  OMP_NUM_THREADS=4 nice -n 19 python scripts/psnr_at_scale.py --gs 3d --lr-scale 1.0 --perturb-seed {} --out $out \
     > /tmp/psnr_ens_3d_lr1_{}.log 2>&1'
