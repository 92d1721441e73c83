set -o pipefail
mkdir -p gpurun_out/r02at
rm -f gpurun_out/r02at/proto.jsonl
for a in "32 10 262144 200" "32 10 262144 1000" "32 10 262144 3000" "64 21 65536 1000" "64 21 65536 3000" "128 42 65536 3000"; do
  timeout -k 10 300 ./tools/protocol_bench $a >> gpurun_out/r02at/proto.jsonl 2>&1 || { echo FAIL $a; tail -5 gpurun_out/r02at/proto.jsonl; exit 1; }
done
cut -c1-330 gpurun_out/r02at/proto.jsonl
