# round-5 batch: window bucket-threshold sweep, operand/expand/L-setup variants at 1e11 and 1e12,
# then the bucket/window/pooled GPU tests on the production build
set -o pipefail
mkdir -p gpurun_out/r5win2 gpurun_out/r5pf
bash tools/gpu/window_lo_sweep.sh > gpurun_out/r5win2/sweep.txt 2>&1 || exit 1
OUT=gpurun_out/r5pf N=1e11 ROUNDS=2 TMO=300 bash tools/gpu/ab.sh prod pf3 xpf pfx lsc atail combo m2x4 q61 q79 || exit 1
OUT=gpurun_out/r5pf N=1e12 ROUNDS=2 TMO=400 bash tools/gpu/ab.sh prod pf3 xpf lsc atail m2x4 q79 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_logical.py tests/test_gpu_rccl.py -k "window or bucket or spill or overflow or pooled" \
  > gpurun_out/r5win2/tests.log 2>&1
