# experiment: block size of sha_rows_kernel (leaves / verify / regen)
set -o pipefail
O=gpurun_out/r02shatpb; mkdir -p $O
for tpb in 256 64 256 64 128; do
RBC_SHA_TPB=$tpb timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 30 > $O/t$tpb.json 2> $O/t$tpb.err || { echo "FAIL $tpb"; tail -5 $O/t$tpb.err; exit 1; }
python -c "import json; d=json.load(open('$O/t$tpb.json')); r=d['roofline']; print('$tpb', d['value'], d['values_ok'], d['stage_ms'], 'iso leaf', r['isolated']['avg_ms'], 'recv', d['receive_only']['ms_per_batch'], 'commit', d['commit_only']['ms_per_batch'])"
done
for c in c1 c4; do for tpb in 256 64; do
RBC_SHA_TPB=$tpb timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 30 --config $c > $O/$c$tpb.json 2> $O/$c$tpb.err || { echo "FAIL $c $tpb"; exit 1; }
python -c "import json; d=json.load(open('$O/$c$tpb.json')); print('$c $tpb', d['value'], d['values_ok'])"
done; done
