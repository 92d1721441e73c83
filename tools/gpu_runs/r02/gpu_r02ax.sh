set -o pipefail
mkdir -p gpurun_out/r02ax
timeout -k 10 400 python bench.py > gpurun_out/r02ax/c2.json 2> gpurun_out/r02ax/c2.err || { echo FAIL; tail -20 gpurun_out/r02ax/c2.err; exit 1; }
for c in c1 c3 c4; do timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --no-pcie > gpurun_out/r02ax/$c.json 2>/dev/null || { echo FAIL $c; exit 1; }; done
timeout -k 10 600 python bench.py --config c3 --total-instances 8192 --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/r02ax/c3_strong.json 2>/dev/null || { echo FAIL c3s; exit 1; }
echo ok
