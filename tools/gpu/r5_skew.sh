# expand/init chunks handed from the youngest waves to the oldest (sk1: 2,1,1,0 chunks per age group; sk2: 2,2,0,0)
set -o pipefail
O=gpurun_out/r5skew
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod sk1 sk2 > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod sk1 sk2 > /dev/null || exit 1
cat $O/ab_*.txt
bash tools/gpu/window_ab3.sh sk1 sk2 2>&1 | grep -v amdgpu.ids
