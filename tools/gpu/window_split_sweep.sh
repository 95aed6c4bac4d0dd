# window time by band split (bucket_split_log2; production 2^28)
set -o pipefail
for r in 1 2; do
  for k in 26 27 28 29 30; do
    echo -n "split=2^$k: "; timeout -k 10 120 python tools/window_bench.py bucket_split_log2=$k || exit 1
  done
done
