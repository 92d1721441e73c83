# experiment: verify / receive-step SHA kernels at occupancy 4 (<= 128 VGPRs, 36 B/lane scratch)
set -o pipefail
O=gpurun_out/r02occ; mkdir -p $O
for r in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 30 > $O/d$r.json 2> $O/d$r.err || { echo "FAIL"; tail -5 $O/d$r.err; exit 1; }
python -c "import json; d=json.load(open('$O/d$r.json')); r=d['roofline']; print('default', d['value'], d['values_ok'], d['stage_ms'], 'iso leaf', r['isolated']['avg_ms'], 'recv', d['receive_only']['ms_per_batch'], 'rxstep', d['receive_only']['receive_step']['ms_per_batch'])"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 30 --pipeline 7 > $O/p7$r.json 2> $O/p7$r.err || { echo "FAIL"; tail -5 $O/p7$r.err; exit 1; }
python -c "import json; d=json.load(open('$O/p7$r.json')); print('p7', d['value'], d['values_ok'], d['stage_ms'])"
done
