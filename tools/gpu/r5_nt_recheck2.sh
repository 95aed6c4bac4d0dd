# store policy after the live-prime bounds, wide ranges
set -o pipefail
O=gpurun_out/r5ntr
mkdir -p $O
for n in 4e11 1e12; do
  OUT=$O N=$n ROUNDS=2 TMO=500 bash tools/gpu/ab.sh prod nt0 ntinf > /dev/null || exit 1
done
cat $O/ab_4e11.txt $O/ab_1e12.txt
