# unit thresholds re-swept on the class-marking build
set -o pipefail
mkdir -p gpurun_out/r5thr
OUT=gpurun_out/r5thr N=1e11 ROUNDS=3 TMO=300 bash tools/gpu/ab.sh prod k16 tb2048 tb1_256 tb1_512 ta79 || exit 1
OUT=gpurun_out/r5thr N=1e12 ROUNDS=1 TMO=300 bash tools/gpu/ab.sh prod k16 tb2048 tb1_256 tb1_512 ta79 || exit 1
