# primes per block counted from the raw image words (rc) instead of the 15 output words (prod)
set -o pipefail
O=gpurun_out/r5rc
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod rc > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod rc > /dev/null || exit 1
cat $O/ab_*.txt
bash tools/gpu/window_ab3.sh rc 2>&1 | grep -v amdgpu.ids
