# machine schedulers for the no-bucket translation unit on the final code: iterative-ilp, max-ilp, max-memory-clause
set -o pipefail
O=gpurun_out/r5sched
mkdir -p $O
OUT=$O N=1e11 ROUNDS=2 TMO=600 bash tools/gpu/ab.sh prod sIlp sMilp sMmc > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=1 TMO=600 bash tools/gpu/ab.sh prod sIlp sMilp sMmc > /dev/null || exit 1
cat $O/ab_*.txt
