# Round-end evidence: all GPU tests, the default bench line (CPU baseline included), every BASELINE
# config on one GPU, rocprofv3 kernel stats + PMC passes of the bench (tools/profile.sh), window kernel stats
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; j=json.load(open('$O/bench.json')); print('bench', j['ms_per_step'], j['value'], j['verified'], j['roofline']['kernel_ms'], j['cpu_baseline']['value'])"
timeout -k 10 300 python tools/config_sweep.py $O/configs_1gpu.json > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
tail -8 $O/configs.log
timeout -k 10 600 bash tools/profile.sh r03final || exit 1
bash tools/gpu/window_kstats.sh
timeout -k 10 420 python -u tools/parity_sweep.py 300 24301 > $O/parity_sweep.txt 2>&1 || { tail -5 $O/parity_sweep.txt; exit 1; }
tail -1 $O/parity_sweep.txt
