set -o pipefail
mkdir -p gpurun_out/c27
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c27/rs -o rs -- python3 tools/rank_steps.py window 8 > gpurun_out/c27/rs.log 2>&1 || { tail -20 gpurun_out/c27/rs.log; exit 1; }
cp "$(find gpurun_out/c27/rs -name '*kernel_stats.csv' | head -1)" gpurun_out/c27/kstats.csv
python3 tools/kstats.py gpurun_out/c27/kstats.csv 14
grep -E "slice|critical" gpurun_out/c27/rs.log
