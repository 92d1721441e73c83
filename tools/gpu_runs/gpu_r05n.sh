# Round 5: rbc_validate_packed's own GPU test (layout checks + oracle parity at
# N = 37, 128, 256), then C3 at 8,192 on one GPU again (the serial line now
# carries roofline_verify with its PMC traffic).
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batcher.py -x -v --timeout 240 --timeout-method thread > $O/batcher_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/batcher_tests.log; exit 1; }
tail -1 $O/batcher_tests.log
timeout -k 10 600 python bench.py --config c3 --total-instances 8192 --steps 4 --warmup 1 --no-cpu-baseline --no-pcie --no-batcher --no-joined-leg > $O/c3_8192.json 2> $O/c3_8192.err || { echo BENCHFAIL; tail -20 $O/c3_8192.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3_8192.json')); print(d['value'], d['decoded_ok'], d['values_ok'], {k: (d[k] or {}).get('traffic') for k in ('roofline','roofline_encode','roofline_verify')})"
echo ok
