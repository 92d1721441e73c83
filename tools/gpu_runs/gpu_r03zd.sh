# Round 3, last call: the full GPU suite and smoke on the final tree.
set -o pipefail
O=gpurun_out/r03zd; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo ok
