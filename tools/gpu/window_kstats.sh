# rocprofv3 kernel stats of the window bench for prod and variants (DSE_NOCHECK: variants may be wrong)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wk
for v in prod "$@"; do
  if [ "$v" = prod ]; then unset DSE_LIB; else export DSE_LIB=variants/libdse_$v.so; fi
  DSE_NOCHECK=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wk/prof_$v -o run -- python tools/window_bench.py > gpurun_out/wk/prof_$v.log 2>&1 || exit 1
  echo "== $v"; grep window gpurun_out/wk/prof_$v.log; find gpurun_out/wk/prof_$v -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 tools/kstats.py {} 10
done
