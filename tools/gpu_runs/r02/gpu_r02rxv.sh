# repeat A/B: receive-step hashing at priority 0 (RBC_RXV_PRIO=0) vs the default 2, interleaved
set -o pipefail
O=gpurun_out/r02rxv; mkdir -p $O
for r in 1 2 3 4 5 6; do
for v in 2 0; do
RBC_RXV_PRIO=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 100 > $O/v${v}_$r.json 2> $O/v${v}_$r.err || { echo "FAIL"; exit 1; }
python -c "import json; d=json.load(open('$O/v${v}_$r.json')); print('rxv$v', d['value'], d['values_ok'])"
done; done
