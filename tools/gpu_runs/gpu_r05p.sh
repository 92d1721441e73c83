# Round 5: the default bench twice with the longer validate-lane passes (six
# windows per level) and the host SHA-NI baseline as the median of three passes.
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 600 python bench.py > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err || { echo BENCHFAIL; tail -20 $O/bench_default_$rep.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['batcher']; print(d['value'], [(s['outstanding'], s['GBps'], s['seconds']) for s in b['sweep']], b['host_sha_ni']['runs_GBps'], b['gpu_over_host_at_epoch'])" $O/bench_default_$rep.json
done
echo ok
