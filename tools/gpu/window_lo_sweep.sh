set -o pipefail
for r in 1 2; do
  for k in 20 19 18 17; do
    echo -n "lo=2^$k: "; timeout -k 10 120 python tools/window_bench.py bucket_lo_log2=$k || exit 1
  done
done
