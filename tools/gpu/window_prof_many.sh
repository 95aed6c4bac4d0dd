# rocprofv3 kernel stats of the window for several variants (no count check): bash tools/gpu/window_prof_many.sh name...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w
for v in "$@"; do
  if [ "$v" = prod ]; then unset DSE_LIB; else export DSE_LIB=variants/libdse_$v.so; fi
  DSE_NOCHECK=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w/prof_$v -o run -- python tools/window_bench.py > gpurun_out/w/prof_$v.log 2>&1 || exit 1
  echo "== $v"; grep "window \[" gpurun_out/w/prof_$v.log
done
