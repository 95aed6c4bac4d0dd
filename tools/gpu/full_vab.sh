# Full GPU suite on the in-tree library, parity subset on variant V, A/B at 1e11 and 1e12:
# V=<name> full_vab.sh name ...
set -o pipefail
mkdir -p gpurun_out/fv
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fv/gputest.log 2>&1 || { tail -40 gpurun_out/fv/gputest.log; exit 1; }
tail -1 gpurun_out/fv/gputest.log
V=${V:-} bash tools/gpu/vtest_ab.sh "$@"
