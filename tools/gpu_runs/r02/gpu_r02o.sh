set -o pipefail
mkdir -p gpurun_out/r02o
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
for i in 1 2; do
  $B > gpurun_out/r02o/c2_p1_$i.json 2>/dev/null || { echo FAIL1; exit 1; }
  $B --pipeline 2 > gpurun_out/r02o/c2_p2_$i.json 2>gpurun_out/r02o/p2.err || { echo FAIL2; tail gpurun_out/r02o/p2.err; exit 1; }
done
$B --pipeline 2 --sets 4 > gpurun_out/r02o/c2_p2_s4.json 2>/dev/null || exit 1
for c in c1 c3 c4; do
  $B --config $c --pipeline 2 > gpurun_out/r02o/${c}_p2.json 2>/dev/null || exit 1
done
echo ok
