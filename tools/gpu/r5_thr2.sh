# unit thresholds re-swept on the final build: TB (B2/L) 1024 / 1280 / 2048, TB1 (B1/B2) 448
set -o pipefail
O=gpurun_out/r5thr2
mkdir -p $O
OUT=$O N=1e11 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod tb1024 tb1280 tb2048 tb1_448 > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod tb1024 tb1280 tb2048 tb1_448 > /dev/null || exit 1
cat $O/ab_*.txt
