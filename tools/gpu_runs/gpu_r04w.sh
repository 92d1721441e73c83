#!/bin/bash
# Round 4: the committed tree at the end of the session -- GPU suite and smoke.
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo ok
