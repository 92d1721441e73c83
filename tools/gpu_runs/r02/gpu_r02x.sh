set -o pipefail
mkdir -p gpurun_out/r02x
timeout -k 10 300 python bench.py --no-pcie --no-cpu-baseline > gpurun_out/r02x/c2.json 2>gpurun_out/r02x/err || { echo FAIL; tail -30 gpurun_out/r02x/err; exit 1; }
timeout -k 10 300 python bench.py --no-pcie --no-cpu-baseline --config c4 > gpurun_out/r02x/c4.json 2>>gpurun_out/r02x/err || { echo FAIL; tail -30 gpurun_out/r02x/err; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02x/test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02x/test.log; exit 1; }
tail -2 gpurun_out/r02x/test.log
