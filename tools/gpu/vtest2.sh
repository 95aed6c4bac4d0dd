# Parity subset against each variant in VS (DSE_TEST_LIB), then an interleaved A/B at 1e11 and 1e12:
#   VS="a b" vtest2.sh name ...
set -o pipefail
mkdir -p gpurun_out/vt
for V in ${VS:-}; do
  DSE_TEST_LIB=variants/libdse_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_logical.py -x -q --timeout 200 --timeout-method thread -k "kb_float or ragged or random_ranges or golden_sweep or 1e10 or geometries or pooled" > gpurun_out/vt/tests_$V.log 2>&1 || { tail -30 gpurun_out/vt/tests_$V.log; exit 1; }
  echo "$V: $(tail -n 1 gpurun_out/vt/tests_$V.log)"
done
OUT=gpurun_out/vt N=1e11 ROUNDS=${ROUNDS:-2} bash tools/gpu/ab.sh "$@" || exit 1
OUT=gpurun_out/vt N=1e12 ROUNDS=1 TMO=900 bash tools/gpu/ab.sh "$@" || exit 1
