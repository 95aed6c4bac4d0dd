# window/bucket GPU tests, then rocprofv3 kernel stats (prod and the variant $1)
set -o pipefail
mkdir -p gpurun_out/w
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "window or bucket" > gpurun_out/w/test.log 2>&1 || { tail -30 gpurun_out/w/test.log; exit 1; }
tail -1 gpurun_out/w/test.log
bash tools/gpu/window_prof.sh "$@"
