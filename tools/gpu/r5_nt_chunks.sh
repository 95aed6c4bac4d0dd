# per-chunk costs of N=1e12 P=8 with the store policy (prod), never-nt and always-nt, interleaved
set -o pipefail
O=gpurun_out/r5ntc
mkdir -p $O
for r in 1 2; do
  for v in prod ntinf nt0; do
    if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
    echo "== $r $v" >> $O/rank_steps_nt.txt
    DSE_LIB=$L timeout -k 10 240 python tools/rank_steps.py 1e12 8 >> $O/rank_steps_nt.txt 2>&1 || { tail -20 $O/rank_steps_nt.txt; exit 1; }
  done
done
grep -E "^==|chunk|critical" $O/rank_steps_nt.txt
