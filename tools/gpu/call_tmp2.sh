set -o pipefail
mkdir -p gpurun_out/c25
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c25/tests.log 2>&1 || { tail -30 gpurun_out/c25/tests.log; exit 1; }
tail -2 gpurun_out/c25/tests.log
OUT=gpurun_out/c25 N=1e11 ROUNDS=3 TMO=500 bash tools/gpu/ab.sh head prod > /dev/null || exit 1
cat gpurun_out/c25/ab_1e11.txt
timeout -k 10 240 python tools/rank_steps.py 1e11 8 > gpurun_out/c25/rs_prod.txt 2>&1 || exit 1
DSE_LIB=variants/libdse_head.so timeout -k 10 240 python tools/rank_steps.py 1e11 8 > gpurun_out/c25/rs_head.txt 2>&1 || exit 1
grep -h "base table\|critical" gpurun_out/c25/rs_prod.txt gpurun_out/c25/rs_head.txt
