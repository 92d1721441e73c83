# Round 3, final code: BASELINE configs[3] as stated on one GPU (all 8,192 x
# 4 MiB instances; the serial schedule, since three shard sets do not fit).
set -o pipefail
O=gpurun_out/r03zt; mkdir -p $O
timeout -k 10 600 python bench.py --config c3 --total-instances 8192 --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > $O/c3_8192.json 2> $O/c3_8192.err || { echo C3FAIL; tail -20 $O/c3_8192.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3_8192.json')); print(d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['config']['hbm_plan']['schedule'])"
echo ok
