set -o pipefail
O=gpurun_out/c9
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh head st64 pilp pmax > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=1 TMO=400 bash tools/gpu/ab.sh head st64 pilp pmax > /dev/null || exit 1
cat $O/ab_*.txt
OUT=$O/ko N=1e11 bash tools/gpu/knockout_pmc.sh 0 1 2 4 8 16 32 || exit 1
OUT=$O/ko N=1e11 ROUNDS=2 TMO=500 bash tools/gpu/ab.sh ko0 ko1 ko2 ko4 ko8 ko16 ko32 > /dev/null || exit 1
cat $O/ko/ab_1e11.txt
