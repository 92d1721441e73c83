set -o pipefail
mkdir -p gpurun_out/r02r
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
$B --pipeline 3 > gpurun_out/r02r/c2_p3_1.json 2>gpurun_out/r02r/err || { echo FAIL3; tail -30 gpurun_out/r02r/err; exit 1; }
$B > gpurun_out/r02r/c2_p1_1.json 2>/dev/null || exit 1
$B --pipeline 3 > gpurun_out/r02r/c2_p3_2.json 2>/dev/null || exit 1
$B > gpurun_out/r02r/c2_p1_2.json 2>/dev/null || exit 1
for c in c1 c3 c4; do $B --config $c --pipeline 3 > gpurun_out/r02r/${c}_p3.json 2>/dev/null || exit 1; done
echo ok
