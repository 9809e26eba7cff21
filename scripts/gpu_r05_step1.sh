# Round 5, step 1: this round's baseline on a fresh box (default bench line incl. secondaries)
# and the HIP chain's at-scale PSNR ensemble (scripts/psnr_hip_ensemble.py).
set -o pipefail
O=gpurun_out/r05s1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json; echo
timeout -k 10 400 python -u scripts/psnr_hip_ensemble.py --gs 2d --lr-scale 0.3 > $O/ens2d.log 2>&1 || { tail -20 $O/ens2d.log; exit 1; }
tail -3 $O/ens2d.log
timeout -k 10 400 python -u scripts/psnr_hip_ensemble.py --gs 3d --lr-scale 0.1 > $O/ens3d.log 2>&1 || { tail -20 $O/ens3d.log; exit 1; }
tail -3 $O/ens3d.log
cp gpurun_out/psnr_hip_ensemble_*.json $O/
