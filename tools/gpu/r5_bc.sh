# in-order expand reads (prod, HEAD) and the bcnt chain (bc) against 509529f (pre)
set -o pipefail
O=gpurun_out/r5bc
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod bc pre > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=1 TMO=600 bash tools/gpu/ab.sh prod bc pre > /dev/null || exit 1
cat $O/ab_*.txt
