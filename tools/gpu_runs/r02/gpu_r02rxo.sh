# bench with the receive_step-only pass (receive_only.receive_step) at every config
set -o pipefail
O=gpurun_out/r02rxo; mkdir -p $O
for c in c2 c1 c4 c3; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 30 --config $c > $O/$c.json 2> $O/$c.err || { echo "FAIL $c"; tail -5 $O/$c.err; exit 1; }
python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['values_ok'], d['receive_only'], d['commit_only']['GBps'])"
done
