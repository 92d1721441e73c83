# per-config bench lines on the final code (CPU baseline from the default run)
set -o pipefail
O=gpurun_out/r02cfg; mkdir -p $O
for c in c1 c3 c4; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --config $c > $O/$c.json 2> $O/$c.err || { echo "FAIL $c"; tail -5 $O/$c.err; exit 1; }
python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], d['values_ok'], d['oracle_sample_ok'], d['decoded_ok'], d['commit_only']['GBps'], d['receive_only']['GBps'], d['config']['pipeline'])"
done
timeout -k 10 600 python bench.py --no-cpu-baseline --no-pcie --config c3 --total-instances 8192 --steps 5 --warmup 1 > $O/c3s.json 2> $O/c3s.err || { echo "FAIL c3s"; tail -5 $O/c3s.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3s.json')); print('c3 8192', d['value'], d['ms_per_step'], d['values_ok'], d['oracle_sample_ok'], d['decoded_ok'], d['config']['pipeline'])"
