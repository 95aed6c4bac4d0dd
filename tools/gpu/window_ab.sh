#!/bin/bash
# Window [1e18, 1e18+1e10] timing (tools/window_bench.py) for library variants, interleaved:
#   OUT=gpurun_out/<dir> ROUNDS=2 bash tools/gpu/window_ab.sh prod bu ...
set -o pipefail
OUT=${OUT:-gpurun_out/wab}; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    L=$([ "$v" = prod ] && echo distributed-sieve-e_amd/mail_sieve_e/libdse.so || echo variants/libdse_$v.so)
    echo -n "$r $v: " | tee -a $OUT/window_ab.txt
    DSE_LIB=$L timeout -k 10 120 python tools/window_bench.py 2>&1 | tail -1 | tee -a $OUT/window_ab.txt || exit 1
  done
done
