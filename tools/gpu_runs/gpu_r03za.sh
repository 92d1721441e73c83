# Round 3, final code: repeatability of the default line (6 runs), instances
# per GPU at C2, and C3 as BASELINE configs[3] states it on one GPU.
set -o pipefail
O=gpurun_out/r03za; mkdir -p $O
B="--no-cpu-baseline --no-pcie"
for rep in 1 2 3 4 5 6; do
  timeout -k 10 300 python bench.py $B > $O/d.json 2>> $O/err || { echo "DFAIL"; tail -20 $O/err; exit 1; }
  python -c "import json; d=json.load(open('$O/d.json')); print('default', d['value'], d['ms_per_step'])"
done
for I in 512 2048 4096; do
  timeout -k 10 300 python bench.py $B --instances $I --steps 60 > $O/i.json 2>> $O/err || { echo "IFAIL $I"; tail -20 $O/err; exit 1; }
  python -c "import json; d=json.load(open('$O/i.json')); print('instances $I', d['value'], d['ms_per_step'], d['config']['hbm_plan']['schedule'])"
done
timeout -k 10 600 python bench.py $B --config c3 --total-instances 8192 --steps 5 --warmup 2 > $O/c3s.json 2>> $O/err || { echo "C3FAIL"; tail -20 $O/err; exit 1; }
python -c "import json; d=json.load(open('$O/c3s.json')); print('c3 8192', d['value'], d['ms_per_step'], d['config']['hbm_plan']['schedule'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'])"
echo ok
