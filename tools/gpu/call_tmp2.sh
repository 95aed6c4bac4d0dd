set -o pipefail
mkdir -p gpurun_out/c26
OUT=gpurun_out/c26 N=1e11 ROUNDS=3 TMO=500 bash tools/gpu/ab.sh head fcfI fcfL fcfIL > /dev/null || exit 1
OUT=gpurun_out/c26 N=1e12 ROUNDS=1 TMO=400 bash tools/gpu/ab.sh head fcfI fcfL fcfIL > /dev/null || exit 1
cat gpurun_out/c26/ab_*.txt
