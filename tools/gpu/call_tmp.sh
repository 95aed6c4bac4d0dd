set -o pipefail
O=gpurun_out/c3
mkdir -p $O
for v in oor oor2; do
DSE_TEST_LIB=variants/libdse_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
tail -1 $O/tests_$v.log
done
OUT=$O N=1e11 ROUNDS=3 TMO=500 bash tools/gpu/ab.sh base pp1 oor oor2 oor2t8 > /dev/null || exit 1
OUT=$O N=1e12 ROUNDS=1 TMO=400 bash tools/gpu/ab.sh base pp1 oor oor2 oor2t8 > /dev/null || exit 1
cat $O/ab_*.txt
