set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02c_gputest.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02c_gputest.log; exit 1; }
tail -3 gpurun_out/r02c_gputest.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' || exit 1
