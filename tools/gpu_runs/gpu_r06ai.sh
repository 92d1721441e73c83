# Round 6: the driver's N=8 bench rehearsed on one GPU at the default per-rank
# workload (1,024 C2 instances per rank, host-fed leg on every rank).
set -o pipefail
O=gpurun_out/${RUN:-r06ai}; mkdir -p $O
t0=$(date +%s)
timeout -k 10 1000 python bench.py --gpus 8 --rehearse-on-one-gpu --no-cpu-baseline > $O/rehearse8_full.json 2> $O/rehearse8_full.err || { echo BENCHFAIL; tail -30 $O/rehearse8_full.err; exit 1; }
echo wall $(( $(date +%s) - t0 )) s
python -c "import json; d=json.load(open('$O/rehearse8_full.json')); p=d['pcie_inclusive']; print(d['value'], d['n_gpus'], d['config'].get('hbm_plan',{}).get('schedule'), d['decoded_ok'], d['values_ok'], 'host', p['aggregate_GBps'], 'kept', p['kept']['aggregate_GBps'], 'fused', p['fused']['aggregate_GBps'], p['ok'], [r['host_fed']['GBps'] for r in d['ranks']])"
echo ok
