set -o pipefail
mkdir -p gpurun_out/r02av
timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_protocol_lockstep.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02av/test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02av/test.log; exit 1; }
tail -1 gpurun_out/r02av/test.log
rm -f gpurun_out/r02av/proto.jsonl
for a in "32 10 262144 1000" "64 21 65536 1000" "128 42 65536 3000"; do
  timeout -k 10 300 ./tools/protocol_bench $a >> gpurun_out/r02av/proto.jsonl 2>&1 || { echo FAIL $a; tail -5 gpurun_out/r02av/proto.jsonl; exit 1; }
done
cut -c1-300 gpurun_out/r02av/proto.jsonl
