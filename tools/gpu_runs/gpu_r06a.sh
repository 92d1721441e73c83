# Round 6, first call: the ABI-6 paths (validate leaves, verified interpolate,
# sparse validate gather, batcher epoch) and the host-fed leg on 1 and 2 ranks,
# then a default bench line (joined value + host-fed epoch).
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_verified.py tests/test_gpu_batcher.py tests/test_gpu_parity.py -k "verified or batcher or epoch or fused_join or validate_packed" > $O/t_verified.log 2>&1 || { echo TESTFAIL1; tail -40 $O/t_verified.log; exit 1; }
timeout -k 10 600 $T tests/test_gpu_bench.py -k "host_fed or schedules" > $O/t_bench.log 2>&1 || { echo TESTFAIL2; tail -40 $O/t_bench.log; exit 1; }
timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 > $O/epoch.jsonl 2> $O/epoch.err || { echo EPOCHFAIL; tail -20 $O/epoch.err; exit 1; }
cat $O/epoch.jsonl
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -30 $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); p=d['pcie_inclusive']; print('value', d['value'], d['ms_per_step'], d['config']['value_form'][:12], 'row', (d.get('value_row_view') or {}).get('value'), 'host', p['aggregate_GBps'], p['rank0'].get('alone_GBps'), p['rank0']['pcie_GBps'], p['ok'])"
tail -3 $O/t_verified.log $O/t_bench.log
echo ok
