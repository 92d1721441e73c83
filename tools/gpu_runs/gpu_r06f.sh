# Round 6: the host API's deferred D2H (product) against enqueueing each
# submission's D2H at once (ab/nodefer, RBC_DEFER_D2H=0) under the host-fed
# epoch and the batcher's drop-in epoch; trace overlap of the nodefer epoch.
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
R=$(pwd)
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
RBC_GPU_LIB=$R/ab/nodefer/librbc_gpu.so LD_LIBRARY_PATH=$R/ab/nodefer timeout -k 10 600 $T tests/test_gpu_verified.py tests/test_gpu_batcher.py > $O/tests_nodefer.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_nodefer.log; exit 1; }
tail -1 $O/tests_nodefer.log
for rep in 1 2; do
for lib in base nodefer; do
  ( if [ $lib = nodefer ]; then export RBC_GPU_LIB=$R/ab/nodefer/librbc_gpu.so LD_LIBRARY_PATH=$R/ab/nodefer; fi
    for infl in 2 3; do
      timeout -k 10 300 python tools/host_bench.py --epoch 1024 --inflight $infl > $O/host_${lib}_i${infl}_$rep.json 2> $O/host_${lib}_i${infl}_$rep.err || { echo HOSTFAIL; tail -20 $O/host_${lib}_i${infl}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/host_${lib}_i${infl}_$rep.json')); print('$lib', 'i$infl', d['GBps'], d['fused']['GBps'], d['alone_GBps'], d['ok'])"
    done
    timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 - svi > $O/epoch_${lib}_$rep.jsonl 2> $O/epoch_${lib}_$rep.err || { echo EPOCHFAIL; tail -20 $O/epoch_${lib}_$rep.err; exit 1; }
    grep -v '"phase": "check"' $O/epoch_${lib}_$rep.jsonl | python -c "import sys, json; [print(' ', (d:=json.loads(l))['interpolate'], d['seconds'], d['GBps'], d['launches']) for l in sys.stdin]"
    timeout -k 10 300 tools/batcher_bench validate-sweep 256 16 200 1024 88064 > $O/vsweep_${lib}_$rep.jsonl 2> $O/vsweep_${lib}_$rep.err || { echo SWEEPFAIL; exit 1; }
    grep '"validate"' $O/vsweep_${lib}_$rep.jsonl | python -c "import sys, json; [print('  validate', (d:=json.loads(l))['outstanding'], d['GBps']) for l in sys.stdin]" ) || exit 1
done
done
( cd /tmp && export TMPDIR=/tmp && export RBC_GPU_LIB=$R/ab/nodefer/librbc_gpu.so && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$O/trace -o run --output-format csv -- python3 $R/tools/host_bench.py --epoch 1024 --inflight 2 > $R/$O/host_trace.json 2> $R/$O/host_trace.err ) || { echo PROFFAIL; tail -20 $O/host_trace.err; exit 1; }
python -c "import json; d=json.load(open('$O/host_trace.json')); [print(w[0], w[1], w[2]) for w in d['timed_windows_ns']]" | while read k a b; do python tools/copy_overlap.py $O/trace $a $b | tee $O/overlap_$k.json; done
echo ok
