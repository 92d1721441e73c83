set -o pipefail
mkdir -p gpurun_out/r02q
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
for i in 1 2; do
$B > gpurun_out/r02q/base_$i.json 2>/dev/null || exit 1
RBC_BENCH_PWAIT=verify $B --sets 3 > gpurun_out/r02q/pwait3_$i.json 2>gpurun_out/r02q/err || { tail gpurun_out/r02q/err; exit 1; }
RBC_BENCH_PWAIT=verify $B --sets 4 > gpurun_out/r02q/pwait4_$i.json 2>/dev/null || exit 1
done
echo ok
