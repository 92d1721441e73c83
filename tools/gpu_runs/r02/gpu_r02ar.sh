set -o pipefail
mkdir -p gpurun_out/r02ar
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie --no-isolated"
$B --pipeline 5 > gpurun_out/r02ar/p5_1.json 2>gpurun_out/r02ar/err || { echo FAIL; tail -30 gpurun_out/r02ar/err; exit 1; }
$B > gpurun_out/r02ar/p1_1.json 2>/dev/null || exit 1
$B --pipeline 5 > gpurun_out/r02ar/p5_2.json 2>/dev/null || exit 1
$B > gpurun_out/r02ar/p1_2.json 2>/dev/null || exit 1
for c in c1 c4; do $B --config $c --pipeline 5 > gpurun_out/r02ar/${c}_p5.json 2>/dev/null || exit 1; $B --config $c > gpurun_out/r02ar/${c}_p1.json 2>/dev/null || exit 1; done
echo ok
