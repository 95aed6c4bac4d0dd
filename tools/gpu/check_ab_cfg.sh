# GPU tests + default bench + interleaved A/B of variants at 1e11 and 1e12 + the config sweep of
# each variant: check_ab_cfg.sh name ... (prod = the in-tree library)
set -o pipefail
O=gpurun_out/cabc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 180 python bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; j=json.load(open('$O/bench.json')); print('bench', j['ms_per_step'], j['value'], j['verified'], j['roofline']['kernel_ms'])"
OUT=$O N=1e11 ROUNDS=3 bash tools/gpu/ab.sh "$@" || exit 1
OUT=$O N=1e12 ROUNDS=1 TMO=900 bash tools/gpu/ab.sh "$@" || exit 1
for v in "$@"; do
  lib=variants/libdse_$v.so; [ $v = prod ] && lib=distributed-sieve-e_amd/mail_sieve_e/libdse.so
  DSE_LIB=$lib timeout -k 10 300 python tools/config_sweep.py $O/configs_$v.json > $O/configs_$v.log 2>&1 || { tail -20 $O/configs_$v.log; exit 1; }
  echo "== configs $v"; python3 -c "
import json
for r in json.load(open('$O/configs_$v.json'))['rows']: print(r['config'], round(r['ms_median'], 3), r['verified'])"
done
