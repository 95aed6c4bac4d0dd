# rocprofv3 kernel stats of the window for the production library and a variant (DSE_LIB)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w
for v in prod ${1:-}; do
  [ -z "$v" ] && continue
  if [ "$v" = prod ]; then unset DSE_LIB; else export DSE_LIB=variants/libdse_$v.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w/prof_$v -o run -- python tools/window_bench.py > gpurun_out/w/prof_$v.log 2>&1 || exit 1
  echo "== $v"; find gpurun_out/w/prof_$v -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-5 | head -12
done
