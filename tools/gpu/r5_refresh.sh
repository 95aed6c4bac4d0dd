# Refresh the round-5 evidence after the store-policy merge: bench line, config sweep,
# rank steps, rocprofv3 trace + PMC of the bench, A/B against the round-start build.
set -o pipefail
O=gpurun_out/ev5b
mkdir -p $O
OUT=$O bash tools/gpu/rank_steps_all.sh || exit 1
timeout -k 10 600 bash tools/profile.sh r05 || exit 1
for n in 1e11 1e12; do
  OUT=$O N=$n ROUNDS=2 TMO=500 bash tools/gpu/ab.sh prod r04 > /dev/null || exit 1
done
cat $O/ab_*.txt
