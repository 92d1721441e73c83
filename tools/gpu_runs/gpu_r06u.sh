# Round 6, ABI 7: validated ECHO rows kept on the device for interpolate.
# The new parity tests (capi keep / kept interpolate, ragged, the batcher's
# keep ring at two sizes), the batcher epoch with its kept pass, the host-fed
# leg's kept run (1 and 2 ranks), then the 8-rank rehearsal with the host-fed
# leg on every rank.
set -o pipefail
O=gpurun_out/${RUN:-r06u}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_verified.py tests/test_gpu_batcher.py -k "keep or kept or epoch" > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 $T tests/test_gpu_bench.py::test_bench_host_fed_leg_on_every_rank > $O/tests_bench.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests_bench.log; exit 1; }
tail -3 $O/tests_bench.log
timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 > $O/epoch.jsonl 2> $O/epoch.err || { echo EPOCHFAIL; tail -20 $O/epoch.err; cat $O/epoch.jsonl; exit 1; }
cat $O/epoch.jsonl
timeout -k 10 300 python tools/host_bench.py --epoch 1024 > $O/host_c2.json 2> $O/host_c2.err || { echo HOSTFAIL; tail -20 $O/host_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/host_c2.json')); print('host', d['GBps'], 'fused', d['fused']['GBps'], 'kept', d['kept']['GBps'], d['kept']['ok'], d['alone_GBps'])"
RUN=${RUN:-r06u} bash tools/gpu_runs/gpu_r06t.sh
