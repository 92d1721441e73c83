set -o pipefail
mkdir -p gpurun_out/r02i
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02i/bench.json 2> gpurun_out/r02i/bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r02i/bench.err; exit 1; }
timeout -k 10 400 python bench.py --config c3 --total-instances 8192 --steps 3 --warmup 1 --no-pcie --cpu-configs c3 > gpurun_out/r02i/c3_8192.json 2> gpurun_out/r02i/c3_8192.err || { echo C3FAIL; tail -20 gpurun_out/r02i/c3_8192.err; exit 1; }
for c in c1 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-pcie --cpu-configs $c > gpurun_out/r02i/$c.json 2> gpurun_out/r02i/$c.err || { echo FAIL $c; tail -20 gpurun_out/r02i/$c.err; exit 1; }
done
echo ok
