# MODE-2 plane chains two at a time (m2p) against one at a time (prod): 1e12, chunk 8, 1e11, GPU parity subset
set -o pipefail
O=gpurun_out/r5m2p
mkdir -p $O
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod m2p > /dev/null || exit 1
OUT=$O N=1e11 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod m2p > /dev/null || exit 1
cat $O/ab_*.txt
for v in prod m2p; do
  if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
  echo "== $v" >> $O/rank_steps.txt
  DSE_LIB=$L timeout -k 10 240 python tools/rank_steps.py 1e12 8 >> $O/rank_steps.txt 2>&1 || { tail -20 $O/rank_steps.txt; exit 1; }
done
grep -E "^==|chunk 8|critical" $O/rank_steps.txt
bash tools/gpu/window_ab3.sh m2p 2>&1 | grep -v amdgpu.ids
