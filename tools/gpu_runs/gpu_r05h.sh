# Round 5: deferred D2H enqueued only after its kernels (Slot::kdone) -- the
# validate lane's test + sweep, its kernel / copy trace, and the host batch
# API (PCIe-inclusive) as a regression check.
set -o pipefail
bash tools/gpu_runs/gpu_r05c.sh || exit 1
bash tools/gpu_runs/gpu_r05g.sh || exit 1
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_abi.py -x -q --timeout 200 --timeout-method thread -k "host or batcher or abi or golden" > $O/hosttests.log 2>&1 || { echo TESTFAIL; tail -30 $O/hosttests.log; exit 1; }
tail -1 $O/hosttests.log
timeout -k 10 200 python tools/host_bench.py > $O/host_bench.jsonl 2> $O/host_bench.err || { echo HOSTFAIL; tail -10 $O/host_bench.err; exit 1; }
cat $O/host_bench.jsonl | head -12
