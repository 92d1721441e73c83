set -o pipefail
mkdir -p gpurun_out/r02ak
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ak/gputest.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02ak/gputest.log; exit 1; }
tail -3 gpurun_out/r02ak/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/r02ak/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 gpurun_out/r02ak/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r02ak/bench_default.json 2> gpurun_out/r02ak/bench_default.err || { echo BENCHFAIL; tail -30 gpurun_out/r02ak/bench_default.err; exit 1; }
cat gpurun_out/r02ak/bench_default.json
timeout -k 10 900 bash tools/profile.sh r02c > gpurun_out/r02ak/profile.log 2>&1 || { echo PROFFAIL; tail -30 gpurun_out/r02ak/profile.log; exit 1; }
echo ok
