# round-5 batch 2: the merged build against the round-start build (b8901d9) at 1e11, 1e12 and the
# window, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/r5b2
OUT=gpurun_out/r5b2 N=1e11 ROUNDS=3 TMO=300 bash tools/gpu/ab.sh prod r04 || exit 1
OUT=gpurun_out/r5b2 N=1e12 ROUNDS=2 TMO=300 bash tools/gpu/ab.sh prod r04 || exit 1
bash tools/gpu/window_ab.sh r04 > gpurun_out/r5b2/window_ab.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5b2/gputest.log 2>&1
