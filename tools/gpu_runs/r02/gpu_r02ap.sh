set -o pipefail
mkdir -p gpurun_out/r02ap
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02ap/test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02ap/test.log; exit 1; }
tail -1 gpurun_out/r02ap/test.log
timeout -k 10 120 ./tests/cpp/rbc_test > gpurun_out/r02ap/cpp.log 2>&1 || { echo CPPFAIL; tail gpurun_out/r02ap/cpp.log; exit 1; }
tail -1 gpurun_out/r02ap/cpp.log
export RBC_BATCHER_DEPTH=4 RBC_HOST_SLOTS=4
timeout -k 10 200 ./tools/batcher_bench 1024 16 64 64 2048 200 > gpurun_out/r02ap/d4.jsonl 2>&1 || { echo FAIL; cat gpurun_out/r02ap/d4.jsonl; exit 1; }
timeout -k 10 200 ./tools/batcher_bench 256 16 512 64 8192 1000 > gpurun_out/r02ap/d4_big.jsonl 2>&1 || { echo FAIL; exit 1; }
cat gpurun_out/r02ap/d4.jsonl gpurun_out/r02ap/d4_big.jsonl | cut -c1-330
