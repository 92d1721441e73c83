set -o pipefail
mkdir -p gpurun_out/r02as
for a in "4 1 1024" "16 5 65536" "16 5 262144" "32 10 262144" "64 21 65536"; do
  timeout -k 10 300 ./tools/protocol_bench $a >> gpurun_out/r02as/proto.jsonl 2>&1 || { echo FAIL $a; tail -5 gpurun_out/r02as/proto.jsonl; exit 1; }
done
cat gpurun_out/r02as/proto.jsonl
