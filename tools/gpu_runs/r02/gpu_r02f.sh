set -o pipefail
mkdir -p gpurun_out/r02f
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02f/gputest.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02f/gputest.log; exit 1; }
tail -2 gpurun_out/r02f/gputest.log
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
for i in 1 2; do
  $B > gpurun_out/r02f/serial_$i.json 2>/dev/null || exit 1
  $B --pipeline 1 > gpurun_out/r02f/pipe_$i.json 2>/dev/null || exit 1
  RBC_VERIFY_COMPACT=0 $B > gpurun_out/r02f/serial_nocompact_$i.json 2>/dev/null || exit 1
  RBC_VERIFY_COMPACT=0 $B --pipeline 1 > gpurun_out/r02f/pipe_nocompact_$i.json 2>/dev/null || exit 1
done
$B --config c4 > gpurun_out/r02f/c4.json 2>/dev/null || exit 1
$B --config c4 --pipeline 1 > gpurun_out/r02f/c4_pipe.json 2>/dev/null || exit 1
$B --config c1 > gpurun_out/r02f/c1.json 2>/dev/null || exit 1
$B --config c1 --pipeline 1 > gpurun_out/r02f/c1_pipe.json 2>/dev/null || exit 1
echo ok
