#!/bin/bash
# A/B of variant libraries (tools/ab_libs.py): OUT=gpurun_out/<dir> N=<n> ROUNDS=<r> ab.sh name ...
set -o pipefail
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
AB_N=${N:-1e11} AB_ROUNDS=${ROUNDS:-2} timeout -k 10 ${TMO:-600} python tools/ab_libs.py "$@" 2>&1 | tee -a $OUT/ab_${N:-1e11}.txt
