# mark-run remainder as one scalar switch (rsw) against the loop (prod)
set -o pipefail
O=gpurun_out/r5rsw
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod rsw > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod rsw > /dev/null || exit 1
cat $O/ab_*.txt
