set -o pipefail
mkdir -p gpurun_out/r02b
B="timeout -k 10 300 python bench.py"
$B --config c3 --total-instances 8192 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02b/c3_8192.json 2> gpurun_out/r02b/c3_8192.err || { echo C3FAIL; tail -20 gpurun_out/r02b/c3_8192.err; exit 1; }
echo c3 done
for i in 1 2 3; do
  $B --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02b/c2_serial_$i.json 2>/dev/null || exit 1
  $B --steps 20 --warmup 3 --no-cpu-baseline --pipeline 1 > gpurun_out/r02b/c2_pipe_$i.json 2>/dev/null || exit 1
done
echo ab done
$B --config c1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02b/c1.json 2>/dev/null || exit 1
$B --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02b/c4.json 2>/dev/null || exit 1
echo ok
