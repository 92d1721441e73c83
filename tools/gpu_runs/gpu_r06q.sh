# Round 6: each host-API slot's D2H on a copy stream of its own, gated on its
# kernels by an event (ab/d2hs, RBC_D2H_STREAM=1), against the deferred D2H on
# the slot's one stream (product), at the default 4 and at 8 hardware queues.
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O
R=$(pwd)
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
RBC_GPU_LIB=$R/ab/d2hs/librbc_gpu.so LD_LIBRARY_PATH=$R/ab/d2hs timeout -k 10 600 $T tests/test_gpu_verified.py tests/test_gpu_batcher.py > $O/tests_d2hs.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_d2hs.log; exit 1; }
tail -1 $O/tests_d2hs.log
for rep in 1 2; do
for lib in base d2hs; do
for q in 4 8; do
  ( export GPU_MAX_HW_QUEUES=$q
    if [ $lib = d2hs ]; then export RBC_GPU_LIB=$R/ab/d2hs/librbc_gpu.so LD_LIBRARY_PATH=$R/ab/d2hs; fi
    timeout -k 10 300 python tools/host_bench.py --config c2 --epoch 1024 --inflight 2 > $O/host_${lib}_q${q}_$rep.json 2> $O/host_${lib}_q${q}_$rep.err || { echo HOSTFAIL; tail -20 $O/host_${lib}_q${q}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/host_${lib}_q${q}_$rep.json')); print('$lib', 'q$q', d['GBps'], d['fused']['GBps'], d['alone_GBps'], d['pcie_GBps'], d['fused']['pcie_GBps'], d['ok'])"
    timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 - svi > $O/epoch_${lib}_q${q}_$rep.jsonl 2> $O/epoch_${lib}_q${q}_$rep.err || { echo EPOCHFAIL; tail -20 $O/epoch_${lib}_q${q}_$rep.err; exit 1; }
    grep -v '"phase": "check"' $O/epoch_${lib}_q${q}_$rep.jsonl | python -c "import sys, json; [print(' ', (d:=json.loads(l))['interpolate'], d['seconds'], d['GBps']) for l in sys.stdin]"
    timeout -k 10 300 tools/batcher_bench validate-sweep 256 16 200 1024 88064 > $O/vsweep_${lib}_q${q}_$rep.jsonl 2> $O/vsweep_${lib}_q${q}_$rep.err || { echo SWEEPFAIL; exit 1; }
    grep '"validate"' $O/vsweep_${lib}_q${q}_$rep.jsonl | python -c "import sys, json; [print('  validate', (d:=json.loads(l))['outstanding'], d['GBps']) for l in sys.stdin]" ) || exit 1
done
done
done
echo ok
