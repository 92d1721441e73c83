set -o pipefail
O=gpurun_out/r02cfg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py -x -q --timeout 280 --timeout-method thread -k "falls_back or schedules" > $O/test.log 2>&1 || { echo TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-pcie --config c3 --total-instances 8192 --steps 5 --warmup 1 > $O/c3s.json 2> $O/c3s.err || { echo "FAIL c3s"; tail -5 $O/c3s.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3s.json')); print('c3 8192', d['value'], d['ms_per_step'], d['values_ok'], d['oracle_sample_ok'], d['decoded_ok'], d['config']['pipeline'])"
