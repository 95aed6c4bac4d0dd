set -o pipefail
mkdir -p gpurun_out/c12
bash tools/gpu/window_kstats.sh c16g1 c16g2 c16g1r8 c16g1r24 c16g1g2k c12g1 nk3 nk1 > gpurun_out/c12/kstats.txt 2>&1 || { tail -30 gpurun_out/c12/kstats.txt; exit 1; }
grep "==\|window \[\|fill_stage\|wheel_segments_kernel<true>" gpurun_out/c12/kstats.txt
for i in 1 2; do for v in prod c16g1 c16g1g2k; do if [ $v = prod ]; then unset DSE_LIB; else export DSE_LIB=variants/libdse_$v.so; fi; echo -n "$v: "; timeout -k 10 120 python tools/window_bench.py || exit 1; done; done
