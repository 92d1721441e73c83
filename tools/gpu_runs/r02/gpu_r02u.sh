set -o pipefail
mkdir -p gpurun_out/r02u
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02u/test.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02u/test.log; exit 1; }
tail -2 gpurun_out/r02u/test.log
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
$B > gpurun_out/r02u/c2_1.json 2>gpurun_out/r02u/err || { echo FAIL; tail -30 gpurun_out/r02u/err; exit 1; }
$B --pipeline 0 > gpurun_out/r02u/c2_serial.json 2>/dev/null || exit 1
$B > gpurun_out/r02u/c2_2.json 2>/dev/null || exit 1
for c in c1 c4; do $B --config $c > gpurun_out/r02u/${c}.json 2>/dev/null || exit 1; done
echo ok
