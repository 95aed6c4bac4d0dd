# nontemporal mask stores: A/B at 1e11 and 1e12
set -o pipefail
mkdir -p gpurun_out/r5nt
OUT=gpurun_out/r5nt N=1e11 ROUNDS=3 TMO=300 bash tools/gpu/ab.sh prod ntst || exit 1
OUT=gpurun_out/r5nt N=1e12 ROUNDS=2 TMO=300 bash tools/gpu/ab.sh prod ntst || exit 1
