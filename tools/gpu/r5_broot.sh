# bucketed pass for ranges with sqrt(max) in (2^18 / 2^19, 2^20] (test option bucket_root_log2)
set -o pipefail
O=gpurun_out/r5broot
mkdir -p $O
for o in "" "bucket_root_log2=19" "bucket_root_log2=19,bucket_lo_log2=18" "bucket_root_log2=18,bucket_lo_log2=18"; do
  for np in "1e12 8" "1e12 1" "4e11 1"; do
    echo "== [$o] $np" >> $O/rs.txt
    DSE_OPTS=$o timeout -k 10 240 python tools/rank_steps.py $np >> $O/rs.txt 2>&1 || { tail -20 $O/rs.txt; exit 1; }
  done
done
grep -E "^==|chunk|critical" $O/rs.txt
