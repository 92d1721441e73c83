set -o pipefail
mkdir -p gpurun_out/r02g
B="timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
for i in 1 2; do
  $B > gpurun_out/r02g/pipe_$i.json 2>/dev/null || exit 1
  RBC_BENCH_PRIO=R $B > gpurun_out/r02g/pipe_prioR_$i.json 2>/dev/null || exit 1
  RBC_BENCH_PRIO=P $B > gpurun_out/r02g/pipe_prioP_$i.json 2>/dev/null || exit 1
done
$B --pipeline 0 > gpurun_out/r02g/serial.json 2>/dev/null || exit 1
echo ok
