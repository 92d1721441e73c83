# Round 5: the C3 lines again, now that profiles/pmc_traffic_r05l_c3*.json
# give their rooflines measured traffic (1,024 x 4 MiB pipelined; all 8,192 on
# one GPU, serial).
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
Q="--no-cpu-baseline --no-pcie --no-batcher --no-joined-leg"
timeout -k 10 300 python bench.py --config c3 --steps 60 $Q > $O/c3.json 2> $O/c3.err || { echo BENCHFAIL c3; tail -20 $O/c3.err; exit 1; }
timeout -k 10 600 python bench.py --config c3 --total-instances 8192 --steps 4 --warmup 1 $Q > $O/c3_8192.json 2> $O/c3_8192.err || { echo BENCHFAIL c3_8192; tail -20 $O/c3_8192.err; exit 1; }
python -c "import json; [print(f, (lambda d: (d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], {k: (d[k] or {}).get('traffic') for k in ('roofline','roofline_encode','roofline_verify','roofline_decode') if k in d}))(json.load(open('$O/'+f+'.json')))) for f in ('c3','c3_8192')]"
echo ok
