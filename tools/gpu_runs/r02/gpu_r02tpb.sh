# experiment: block size of the combined receive-step SHA launch (placement)
set -o pipefail
O=gpurun_out/r02tpb; mkdir -p $O
for tpb in 256 64 128 64; do
RBC_RX_TPB=$tpb timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 30 > $O/t$tpb.json 2> $O/t$tpb.err || { echo "FAIL $tpb"; tail -5 $O/t$tpb.err; exit 1; }
python -c "import json; d=json.load(open('$O/t$tpb.json')); print('$tpb', d['value'], d['values_ok'], d['receive_only']['GBps'], d['receive_only']['receive_step']['ms_per_batch'])"
done
RBC_RX_TPB=64 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 30 --pipeline 7 > $O/p7.json 2> $O/p7.err && python -c "import json; d=json.load(open('$O/p7.json')); print('p7 tpb64', d['value'], d['values_ok'])"
