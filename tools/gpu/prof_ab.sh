# PMC + trace of the in-tree library's bench at 1e11 (tools/gpu/pmc_deep.sh), the two GPU test
# files that cover a change's risk, then an interleaved A/B of variants at 1e11 and 1e12:
# prof_ab.sh name ...
set -o pipefail
OUT=gpurun_out/pmc_prod N=1e11 bash tools/gpu/pmc_deep.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "kb_float or ragged or random_ranges or golden_sweep or 1e10" > gpurun_out/pab_tests.log 2>&1 || { tail -30 gpurun_out/pab_tests.log; exit 1; }
tail -1 gpurun_out/pab_tests.log
OUT=gpurun_out/pab N=1e11 ROUNDS=2 bash tools/gpu/ab.sh "$@" || exit 1
OUT=gpurun_out/pab N=1e12 ROUNDS=1 TMO=900 bash tools/gpu/ab.sh "$@" || exit 1
