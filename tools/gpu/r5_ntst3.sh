# run-time store policy: GPU suite on the in-tree build, window timing against never-nt
set -o pipefail
O=gpurun_out/r5nt3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
bash tools/gpu/window_ab3.sh ntinf nt0 > $O/window.txt 2>&1 || { cat $O/window.txt; exit 1; }
cat $O/window.txt
