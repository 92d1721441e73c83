set -o pipefail
mkdir -p gpurun_out/r02an
A="1024 16 64 64 2048 200"
timeout -k 10 200 ./tools/batcher_bench_old $A > gpurun_out/r02an/old.jsonl 2>&1 || { echo OLDFAIL; cat gpurun_out/r02an/old.jsonl; exit 1; }
timeout -k 10 200 ./tools/batcher_bench $A > gpurun_out/r02an/new.jsonl 2>&1 || { echo NEWFAIL; cat gpurun_out/r02an/new.jsonl; exit 1; }
RBC_BATCHER_DEPTH=4 RBC_HOST_SLOTS=4 timeout -k 10 200 ./tools/batcher_bench $A > gpurun_out/r02an/new_d4.jsonl 2>&1 || { echo D4FAIL; cat gpurun_out/r02an/new_d4.jsonl; exit 1; }
timeout -k 10 200 ./tools/batcher_bench 1024 32 256 64 4096 200 > gpurun_out/r02an/new_w256.jsonl 2>&1 || { echo WFAIL; exit 1; }
for f in old new new_d4 new_w256; do echo $f; cat gpurun_out/r02an/$f.jsonl | cut -c1-330; done
