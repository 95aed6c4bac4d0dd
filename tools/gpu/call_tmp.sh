set -o pipefail
O=gpurun_out/c8
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh head mul24 st4 st16 > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=1 TMO=400 bash tools/gpu/ab.sh head mul24 st4 st16 > /dev/null || exit 1
cat $O/ab_*.txt
OUT=$O/window bash tools/gpu/window_evidence.sh || exit 1
