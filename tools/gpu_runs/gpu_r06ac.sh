# Round 6: where the C4 host-fed epoch's time goes -- kernel + copy trace of
# tools/host_bench.py --config c4 --epoch 16384 -- and an A/B of the
# zero-copy gathers with more waves for short rows (ab/librbc_gpu_gshort.so,
# RBC_GATHER_SHORT_ROWS=1): C4 and C2 host-fed epochs, twice each.
set -o pipefail
O=gpurun_out/${RUN:-r06ac}; mkdir -p $O
R=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/tools/host_bench.py --config c4 --epoch 16384 > $R/$O/host_c4_prof.json 2> $R/$O/host_c4_prof.err ) || { echo PROFFAIL; tail -20 $O/host_c4_prof.err; exit 1; }
head -14 $O/prof/run_kernel_stats.csv
head -6 $O/prof/run_memory_copy_stats.csv
for rep in 1 2; do
  for lib in base gshort; do
    if [ $lib = base ]; then unset RBC_GPU_LIB; else export RBC_GPU_LIB=$R/ab/librbc_gpu_$lib.so; fi
    for cfg in c4 c2; do
      ni=$([ $cfg = c4 ] && echo 16384 || echo 1024)
      timeout -k 10 300 python tools/host_bench.py --config $cfg --epoch $ni > $O/host_${cfg}_${lib}_$rep.json 2> $O/host_${cfg}_${lib}_$rep.err || { echo HOSTFAIL; tail -20 $O/host_${cfg}_${lib}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/host_${cfg}_${lib}_$rep.json')); print('$cfg $lib $rep', 'drop-in', d['GBps'], 'kept', d['kept']['GBps'], 'fused', d['fused']['GBps'], d['ok'], d['alone_GBps'])"
    done
  done
done
echo ok
