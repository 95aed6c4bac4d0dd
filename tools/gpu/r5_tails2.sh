# unrolled short tails: L sets with 3-4 tail steps (t34), B2 units with <= 4 (b2t), both (t34b2)
set -o pipefail
O=gpurun_out/r5tails2
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod t34 b2t t34b2 > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod t34 b2t t34b2 > /dev/null || exit 1
cat $O/ab_*.txt
