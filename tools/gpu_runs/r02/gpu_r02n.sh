set -o pipefail
mkdir -p gpurun_out/r02n
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
for i in 1 2; do
  for ns in 2 3 4; do
    $B --sets $ns > gpurun_out/r02n/c2_sets${ns}_$i.json 2>/dev/null || { echo FAIL $ns; exit 1; }
  done
done
$B --config c1 > gpurun_out/r02n/c1_sets3.json 2>/dev/null || exit 1
$B --config c4 > gpurun_out/r02n/c4_sets3.json 2>/dev/null || exit 1
$B --config c3 > gpurun_out/r02n/c3_sets3.json 2>/dev/null || exit 1
echo ok
