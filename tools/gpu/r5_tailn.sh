# MODE-0 tails of at most 1-2 steps as unrolled predicated marks (prod) against HEAD (hd)
set -o pipefail
O=gpurun_out/r5tailn
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
OUT=$O N=1e11 ROUNDS=3 TMO=500 bash tools/gpu/ab.sh prod hd > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=2 TMO=500 bash tools/gpu/ab.sh prod hd > /dev/null || exit 1
cat $O/ab_*.txt
