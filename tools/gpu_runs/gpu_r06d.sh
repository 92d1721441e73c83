# Round 6: receive-side H2D by SDMA (every row, one flat copy; ab/dense =
# RBC_ZERO_COPY_READS=0) against the zero-copy gather kernels (product), under
# the host-fed epoch: the duplex probe showed kernel reads || SDMA D2H carry
# ~60 GB/s in total, SDMA both ways ~97.
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
RBC_GPU_LIB=$(pwd)/ab/dense/librbc_gpu.so LD_LIBRARY_PATH=$(pwd)/ab/dense timeout -k 10 600 $T tests/test_gpu_verified.py tests/test_gpu_batcher.py > $O/tests_dense.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_dense.log; exit 1; }
timeout -k 10 600 $T tests/test_gpu_verified.py > $O/tests_base.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_base.log; exit 1; }
tail -1 $O/tests_dense.log $O/tests_base.log
for rep in 1 2; do
for lib in base dense; do
  ( if [ $lib = dense ]; then export RBC_GPU_LIB=$(pwd)/ab/dense/librbc_gpu.so LD_LIBRARY_PATH=$(pwd)/ab/dense; fi
    timeout -k 10 300 python tools/host_bench.py --epoch 1024 --inflight 2 > $O/host_${lib}_$rep.json 2> $O/host_${lib}_$rep.err || { echo HOSTFAIL; tail -20 $O/host_${lib}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/host_${lib}_$rep.json')); print('$lib', d['library'][-25:], d['GBps'], d['fused']['GBps'], d['alone_GBps'], d['pcie_GBps'], d['fused']['pcie_GBps'], d['ok'])"
    timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 - svi > $O/epoch_${lib}_$rep.jsonl 2> $O/epoch_${lib}_$rep.err || { echo EPOCHFAIL; tail -20 $O/epoch_${lib}_$rep.err; exit 1; }
    grep -v '"phase": "check"' $O/epoch_${lib}_$rep.jsonl | python -c "import sys, json; [print(' ', (d:=json.loads(l))['interpolate'], d['seconds'], d['GBps'], d['launches']) for l in sys.stdin]" ) || exit 1
done
done
echo ok
