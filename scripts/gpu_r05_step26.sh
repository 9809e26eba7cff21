# Round 5, step 26: the 3DGS forward's waves per SIMD (106 VGPRs at D=4 = 4 waves; 5 / 6 forced),
# interleaved c2 A/Bs on one box.
set -o pipefail
TAG=r05s26/f5 LIB_B=horizongs_amd/_lib_f5/libhgsr.so CONFIGS="c2" REPS=2 bash scripts/gpu_r04_ab.sh &&
TAG=r05s26/f6 LIB_B=horizongs_amd/_lib_f6/libhgsr.so CONFIGS="c2" REPS=2 bash scripts/gpu_r04_ab.sh
