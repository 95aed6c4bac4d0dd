# loop headers aligned to 32 / 64 / 128 bytes (instruction fetch) against the unaligned build
set -o pipefail
O=gpurun_out/r5align
mkdir -p $O
OUT=$O N=1e11 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod al32 al64 al128 > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod al32 al64 al128 > /dev/null || exit 1
cat $O/ab_*.txt
bash tools/gpu/window_ab3.sh al32 al64 al128 2>&1 | grep -v amdgpu.ids
