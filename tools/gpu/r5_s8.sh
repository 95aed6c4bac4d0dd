# 8-mark run steps (s8), MODE-1 first mark unconditional (m1u), both; parity of both on the GPU suite subset
set -o pipefail
O=gpurun_out/r5s8
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod s8 m1u s8m1u > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod s8 m1u s8m1u > /dev/null || exit 1
cat $O/ab_*.txt
