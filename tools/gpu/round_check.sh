# Full GPU check of the tree: GPU tests, default bench, config sweep, window kernel profile
set -o pipefail
mkdir -p gpurun_out/rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rc/gputest.log 2>&1 || { tail -40 gpurun_out/rc/gputest.log; exit 1; }
tail -1 gpurun_out/rc/gputest.log
timeout -k 10 180 python bench.py > gpurun_out/rc/bench.json 2> gpurun_out/rc/bench.err || { tail -20 gpurun_out/rc/bench.err; exit 1; }
python3 -c "import json; j=json.load(open('gpurun_out/rc/bench.json')); print('bench', j['ms_per_step'], j['value'], j['verified'], j['roofline']['kernel_ms'])"
timeout -k 10 300 python tools/config_sweep.py gpurun_out/rc/configs_1gpu.json > gpurun_out/rc/configs.log 2>&1 || { tail -20 gpurun_out/rc/configs.log; exit 1; }
cat gpurun_out/rc/configs.log | tail -12
bash tools/gpu/window_prof.sh
