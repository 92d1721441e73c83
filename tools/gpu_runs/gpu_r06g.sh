# Round 6: latency of the synchronous single-call drop-ins with
# blocking-sync slot events (product) against spin-waited events (ab/spin),
# and the validate lane at 1 k / 88 k outstanding under each.
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
R=$(pwd)
for rep in 1 2; do
for lib in base spin; do
  ( if [ $lib = spin ]; then export RBC_GPU_LIB=$R/ab/spin/librbc_gpu.so LD_LIBRARY_PATH=$R/ab/spin; fi
    timeout -k 10 300 python tools/latency_probe.py 300 > $O/lat_${lib}_$rep.json 2> $O/lat_${lib}_$rep.err || { echo LATFAIL; tail -20 $O/lat_${lib}_$rep.err; exit 1; }
    echo $lib; cat $O/lat_${lib}_$rep.json
    timeout -k 10 300 tools/batcher_bench validate-sweep 256 16 200 1024 88064 > $O/vsweep_${lib}_$rep.jsonl 2> $O/vsweep_${lib}_$rep.err || { echo SWEEPFAIL; exit 1; }
    grep '"validate"' $O/vsweep_${lib}_$rep.jsonl | python -c "import sys, json; [print('  validate', (d:=json.loads(l))['outstanding'], d['GBps']) for l in sys.stdin]" ) || exit 1
done
done
echo ok
