# the no-bucket kernels without the Barrett path and its operand registers (prod) against HEAD (pre)
set -o pipefail
O=gpurun_out/r5nob
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod pre > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod pre > /dev/null || exit 1
cat $O/ab_*.txt
