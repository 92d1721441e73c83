set -o pipefail
mkdir -p gpurun_out/r02p
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
$B > gpurun_out/r02p/base.json 2>/dev/null || exit 1
for sp in 2/8 3/8 4/8 5/16 7/16; do
  RBC_BENCH_CU_SPLIT=$sp $B > gpurun_out/r02p/split_${sp/\//_}.json 2>gpurun_out/r02p/err || { echo FAIL $sp; tail gpurun_out/r02p/err; exit 1; }
done
echo ok
