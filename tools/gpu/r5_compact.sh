# one-launch base-table compaction (prod) against HEAD (pre): GPU suite, step time, base table time
set -o pipefail
O=gpurun_out/r5compact
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
OUT=$O N=1e11 ROUNDS=3 TMO=600 bash tools/gpu/ab.sh prod pre > /dev/null || exit 1
cat $O/ab_1e11.txt
for v in prod pre; do
  if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
  for np in "1e11 8" "1e12 8"; do
    echo "== $v $np" >> $O/rank_steps.txt
    DSE_LIB=$L timeout -k 10 240 python tools/rank_steps.py $np >> $O/rank_steps.txt 2>&1 || { tail -20 $O/rank_steps.txt; exit 1; }
  done
done
grep -E "^==|base table|critical" $O/rank_steps.txt
