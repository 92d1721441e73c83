# Round 6: A/B of the zero-copy gathers with four reads in flight per lane
# (ab/librbc_gpu_gunroll.so, RBC_GATHER_UNROLL=1): the verified/kept GPU tests
# on it, then host-fed epochs at C4, C2, C3, twice each, both libraries.
set -o pipefail
O=gpurun_out/${RUN:-r06ag}; mkdir -p $O
R=$(pwd)
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
RBC_GPU_LIB=$R/ab/librbc_gpu_gunroll.so timeout -k 10 600 $T tests/test_gpu_verified.py > $O/tests_gunroll.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_gunroll.log; exit 1; }
tail -1 $O/tests_gunroll.log
for rep in 1 2; do
  for lib in base gunroll; do
    if [ $lib = base ]; then unset RBC_GPU_LIB; else export RBC_GPU_LIB=$R/ab/librbc_gpu_$lib.so; fi
    for cfg in c4 c2 c3; do
      ni=$([ $cfg = c4 ] && echo 16384 || echo 1024); [ $cfg = c3 ] && ni=256
      timeout -k 10 300 python tools/host_bench.py --config $cfg --epoch $ni > $O/host_${cfg}_${lib}_$rep.json 2> $O/host_${cfg}_${lib}_$rep.err || { echo HOSTFAIL; tail -20 $O/host_${cfg}_${lib}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/host_${cfg}_${lib}_$rep.json')); print('$cfg $lib $rep', 'drop-in', d['GBps'], 'kept', d['kept']['GBps'], 'fused', d['fused']['GBps'], d['ok'], d['alone_GBps'])"
    done
  done
done
echo ok
