# -e of each plane step by one v_bfe_i32 where used (nef) instead of 8 registers (prod)
set -o pipefail
O=gpurun_out/r5nef
mkdir -p $O
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod nef > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod nef > /dev/null || exit 1
cat $O/ab_*.txt
for v in prod nef; do
  if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
  echo "== $v" >> $O/rank_steps.txt
  DSE_LIB=$L timeout -k 10 240 python tools/rank_steps.py 1e12 8 >> $O/rank_steps.txt 2>&1 || { tail -20 $O/rank_steps.txt; exit 1; }
done
grep -E "^==|chunk 8|critical" $O/rank_steps.txt
