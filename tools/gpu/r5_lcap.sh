# per-piece large-prime bounds (prod) against the store-policy commit (nt1): parity, A/B, chunk costs, window
set -o pipefail
O=gpurun_out/r5lcap
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for n in 1e11 1e12; do
  OUT=$O N=$n ROUNDS=2 TMO=500 bash tools/gpu/ab.sh prod nt1 > /dev/null || exit 1
done
cat $O/ab_*.txt
for v in prod nt1; do
  if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
  echo "== $v" >> $O/rank_steps.txt
  DSE_LIB=$L timeout -k 10 240 python tools/rank_steps.py 1e12 8 >> $O/rank_steps.txt 2>&1 || { tail -20 $O/rank_steps.txt; exit 1; }
done
grep -E "^==|chunk|critical" $O/rank_steps.txt
bash tools/gpu/window_ab3.sh nt1 2>&1 | grep -v amdgpu.ids
