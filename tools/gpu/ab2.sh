# Interleaved A/B of variants at 1e11 (ROUNDS) and 1e12 (1 round): ab2.sh name ...
set -o pipefail
OUT=gpurun_out/ab2 N=1e11 ROUNDS=${ROUNDS:-2} bash tools/gpu/ab.sh "$@" || exit 1
OUT=gpurun_out/ab2 N=1e12 ROUNDS=1 TMO=900 bash tools/gpu/ab.sh "$@" || exit 1
