# Round 6: the driver's 8-rank launch rehearsed on one GPU WITH the host-fed
# leg on every rank (2,048 instances, 256 per rank), all eight ranks' pinned
# epochs at once.
set -o pipefail
O=gpurun_out/${RUN:-r06t}; mkdir -p $O
timeout -k 10 500 python bench.py --gpus 8 --rehearse-on-one-gpu --total-instances 2048 --steps 3 --warmup 3 --no-isolated --no-joined-leg --no-cpu-baseline > $O/rehearse8_hostfed.json 2> $O/rehearse8_hostfed.err || { echo BENCHFAIL; tail -30 $O/rehearse8_hostfed.err; exit 1; }
python -c "import json; d=json.load(open('$O/rehearse8_hostfed.json')); p=d['pcie_inclusive']; print(d['value'], d['n_gpus'], p['aggregate_GBps'], p['per_rank_GBps'], p['fused']['aggregate_GBps'], p['fused']['per_rank_GBps'], p['ok'])"
echo ok
