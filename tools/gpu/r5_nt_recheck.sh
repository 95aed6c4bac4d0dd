# store policy re-checked after the live-prime bounds: prod (policy) / nt0 (always) / ntinf (never)
set -o pipefail
O=gpurun_out/r5ntr
mkdir -p $O
for n in 1e11 2e11; do
  OUT=$O N=$n ROUNDS=2 TMO=400 bash tools/gpu/ab.sh prod nt0 ntinf > /dev/null || exit 1
done
cat $O/ab_*.txt
for v in prod nt0 ntinf; do
  if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
  echo "== $v" >> $O/rank_steps.txt
  DSE_LIB=$L timeout -k 10 240 python tools/rank_steps.py 1e12 8 >> $O/rank_steps.txt 2>&1 || { tail -20 $O/rank_steps.txt; exit 1; }
done
grep -E "^==|chunk|critical" $O/rank_steps.txt
