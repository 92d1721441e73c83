set -o pipefail
mkdir -p gpurun_out/r02w
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "every_instance or full_size" --durations 10 > gpurun_out/r02w/test.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02w/test.log; exit 1; }
tail -25 gpurun_out/r02w/test.log
