# Round 6: one wave per row in the zero-copy gathers (C4's 384-B rows) and one
# flat D2H of a pinned 64-B-pitch shard_commit output: GPU parity of the host
# API, then the host-fed epoch at every config.
set -o pipefail
O=gpurun_out/${RUN:-r06k}; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_verified.py tests/test_gpu_batcher.py tests/test_gpu_parity.py tests/test_gpu_wire.py tests/test_cpp_abi.py tests/test_gpu_encoder.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in c2 c4 c1 c3; do
  inst=1024; [ $cfg = c4 ] && inst=16384; [ $cfg = c3 ] && inst=512
  timeout -k 10 300 python tools/host_bench.py --config $cfg --epoch $inst --inflight 2 > $O/host_$cfg.json 2> $O/host_$cfg.err || { echo HOSTFAIL; tail -20 $O/host_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$O/host_$cfg.json')); print('$cfg', d['GBps'], d['fused']['GBps'], d['alone_GBps'], d['pcie_GBps'], d['ok'])"
done
echo ok
