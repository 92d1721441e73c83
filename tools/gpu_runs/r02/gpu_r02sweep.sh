# final code: instances-per-GPU sweep at C2 (--pipeline 7 default)
set -o pipefail
O=gpurun_out/r02sweep; mkdir -p $O
for i in 512 1024 2048 4096; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 60 --instances $i > $O/i$i.json 2> $O/i$i.err || { echo "FAIL $i"; tail -5 $O/i$i.err; exit 1; }
python -c "import json; d=json.load(open('$O/i$i.json')); print('$i', d['value'], d['ms_per_step'], d['values_ok'], d['decoded_ok'])"
done
