set -o pipefail
for a in "128 42 65536 3000 1" "128 42 65536 3000 8"; do
  timeout -k 10 300 ./tools/protocol_bench $a > gpurun_out/r02bb.json 2>&1 || { echo FAIL; cat gpurun_out/r02bb.json; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r02bb.json')); print(d['threads'], d['seconds'], d['gpu_launches'], d['thread_seconds'])"
done
