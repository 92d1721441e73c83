set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a_gputest.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02a_gputest.log; exit 1; }
tail -3 gpurun_out/r02a_gputest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err || { echo BENCHFAIL; tail -30 gpurun_out/r02a_bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --force-gather --no-cpu-baseline > gpurun_out/r02a_bench_gather.json 2> gpurun_out/r02a_bench_gather.err || { echo GATHERFAIL; tail -30 gpurun_out/r02a_bench_gather.err; exit 1; }
echo ok
