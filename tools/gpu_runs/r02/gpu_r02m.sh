set -o pipefail
mkdir -p gpurun_out/r02m
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02m/gputest.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02m/gputest.log; exit 1; }
tail -2 gpurun_out/r02m/gputest.log
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
for i in 1 2; do
  $B > gpurun_out/r02m/c2_$i.json 2>/dev/null || exit 1
  RBC_VERIFY_PATH=2 $B > gpurun_out/r02m/c2_path_$i.json 2>/dev/null || exit 1
done
$B --config c4 > gpurun_out/r02m/c4.json 2>/dev/null || exit 1
$B --config c1 > gpurun_out/r02m/c1.json 2>/dev/null || exit 1
RBC_VERIFY_PATH=2 $B --config c1 > gpurun_out/r02m/c1_path.json 2>/dev/null || exit 1
echo ok
