# Round 6, final tree (1/2): the whole GPU suite and smoke().
set -o pipefail
O=gpurun_out/${RUN:-r06i}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
echo ok
