set -o pipefail
mkdir -p gpurun_out/r02j
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
for I in 1024 2048 4096 8192; do
  $B --instances $I > gpurun_out/r02j/c2_$I.json 2>/dev/null || { echo FAIL $I; exit 1; }
done
$B --instances 4096 --pipeline 0 > gpurun_out/r02j/c2_4096_serial.json 2>/dev/null || exit 1
$B --config c4 --instances 65536 > gpurun_out/r02j/c4_65536.json 2>/dev/null || exit 1
echo ok
