# Kb mod p for 2^32 <= Kb < 2^38: q p by v_mul_u32_u24 for sets of primes >= 2^15 (qp) against v_mul_lo_u32 (prod)
set -o pipefail
O=gpurun_out/r5qp
mkdir -p $O
OUT=$O N=1e12 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod qp > /dev/null || exit 1
OUT=$O N=1e11 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod qp > /dev/null || exit 1
cat $O/ab_*.txt
for v in prod qp; do
  if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
  echo "== $v" >> $O/rank_steps.txt
  DSE_LIB=$L timeout -k 10 240 python tools/rank_steps.py 1e12 8 >> $O/rank_steps.txt 2>&1 || { tail -20 $O/rank_steps.txt; exit 1; }
done
grep -E "^==|chunk 8|critical" $O/rank_steps.txt
