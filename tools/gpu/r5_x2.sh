# expand: LUT index v ^ ((v >> 2) & 63) (x2), no hi-first block reads (nhf), both (x2nhf)
set -o pipefail
O=gpurun_out/r5x2
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod x2 nhf x2nhf > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=1 TMO=600 bash tools/gpu/ab.sh prod x2 nhf x2nhf > /dev/null || exit 1
cat $O/ab_*.txt
bash tools/gpu/window_ab3.sh x2 2>&1 | grep -v amdgpu.ids
