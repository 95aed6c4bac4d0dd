# no-copy large-unit operands: A/B at 1e11, 1e12, the window, and the parity suite on the variant
set -o pipefail
mkdir -p gpurun_out/r5noc
OUT=gpurun_out/r5noc N=1e11 ROUNDS=3 TMO=300 bash tools/gpu/ab.sh prod noc || exit 1
OUT=gpurun_out/r5noc N=1e12 ROUNDS=2 TMO=300 bash tools/gpu/ab.sh prod noc || exit 1
bash tools/gpu/window_ab.sh noc > gpurun_out/r5noc/window_ab.txt 2>&1 || exit 1
DSE_TEST_LIB=$PWD/variants/libdse_noc.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_logical.py > gpurun_out/r5noc/parity.log 2>&1
