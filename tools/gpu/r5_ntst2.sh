# non-temporal mask stores against N: always (nt0), never (ntinf), by the table size (prod)
set -o pipefail
mkdir -p gpurun_out/r5nt2
for n in 1e11 2e11 4e11 1e12; do
  OUT=gpurun_out/r5nt2 N=$n ROUNDS=2 TMO=400 bash tools/gpu/ab.sh prod nt0 ntinf || exit 1
done
