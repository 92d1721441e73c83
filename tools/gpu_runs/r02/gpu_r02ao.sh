set -o pipefail
mkdir -p gpurun_out/r02ao
export RBC_BATCHER_DEPTH=4 RBC_HOST_SLOTS=4
for args in "256 1 4096 64 4096 200" "256 4 2048 64 8192 1000" "256 16 512 64 8192 1000" "256 64 128 64 8192 2000"; do
  timeout -k 10 200 ./tools/batcher_bench $args > gpurun_out/r02ao/tmp.jsonl 2>&1 || { echo FAIL; cat gpurun_out/r02ao/tmp.jsonl; exit 1; }
  grep validate gpurun_out/r02ao/tmp.jsonl | cut -c1-330
done
