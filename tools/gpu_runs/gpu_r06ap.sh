# Round 6: the short-value gather (shard_commit of many pinned values < 256 KiB,
# C4) with 1,024 waves instead of 256 (ab/librbc_gpu_gv256.so); the
# short-values GPU test on it, then C4 host-fed epochs twice each.
set -o pipefail
O=gpurun_out/${RUN:-r06ap}; mkdir -p $O
R=$(pwd)
RBC_GPU_LIB=$R/ab/librbc_gpu_gv256.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verified.py -k "short_pinned" > $O/tests_gv256.txt 2>&1 || { echo TESTFAIL; tail -30 $O/tests_gv256.txt; exit 1; }
tail -1 $O/tests_gv256.txt
for rep in 1 2; do
  for lib in base gv256; do
    if [ $lib = base ]; then unset RBC_GPU_LIB; else export RBC_GPU_LIB=$R/ab/librbc_gpu_$lib.so; fi
    timeout -k 10 300 python tools/host_bench.py --config c4 --epoch 16384 > $O/host_c4_${lib}_$rep.json 2> $O/host_c4_${lib}_$rep.err || { echo HOSTFAIL; tail -20 $O/host_c4_${lib}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/host_c4_${lib}_$rep.json')); print('c4 $lib $rep', 'drop-in', d['GBps'], 'kept', d['kept']['GBps'], 'fused', d['fused']['GBps'], d['ok'], d['alone_GBps'])"
  done
done
echo ok
