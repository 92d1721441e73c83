set -o pipefail
mkdir -p gpurun_out/r02ba
rm -f gpurun_out/r02ba/proto.jsonl
for a in "32 10 262144 1000 1" "32 10 262144 1000 8" "128 42 65536 3000 1" "128 42 65536 3000 4" "128 42 65536 3000 16"; do
  timeout -k 10 300 ./tools/protocol_bench $a >> gpurun_out/r02ba/proto.jsonl 2>&1 || { echo FAIL $a; tail -5 gpurun_out/r02ba/proto.jsonl; exit 1; }
done
cut -c1-260 gpurun_out/r02ba/proto.jsonl
