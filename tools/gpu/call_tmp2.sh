set -o pipefail
mkdir -p gpurun_out/c19
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_logical.py tests/test_gpu_rccl.py -m gpu -x -q -k "bucket or window or table" --timeout 300 --timeout-method thread > gpurun_out/c19/tests.log 2>&1 || { tail -30 gpurun_out/c19/tests.log; exit 1; }
tail -2 gpurun_out/c19/tests.log
for i in 1 2 3; do for v in prod head sg128 sg64t16k g1k2 g1k8; do if [ $v = prod ]; then unset DSE_LIB; else export DSE_LIB=variants/libdse_$v.so; fi; echo -n "$v: "; timeout -k 10 120 python tools/window_bench.py || exit 1; done; done
unset DSE_LIB
bash tools/gpu/window_kstats.sh head sg128 sg64t16k g1k2 g1k8 > gpurun_out/c19/kstats.txt 2>&1 || { tail -30 gpurun_out/c19/kstats.txt; exit 1; }
grep "==\|window \[\|fill_stage\|bucket_sort" gpurun_out/c19/kstats.txt
