set -o pipefail
NO_PMC=1 timeout -k 10 400 bash tools/profile.sh r02v_ser --steps 20 --warmup 3 --no-cpu-baseline --no-pcie --pipeline 0 > gpurun_out/r02v_ser.log 2>&1 || { echo FAIL; tail -20 gpurun_out/r02v_ser.log; exit 1; }
NO_PMC=1 timeout -k 10 400 bash tools/profile.sh r02v_c1 --steps 20 --warmup 3 --no-cpu-baseline --no-pcie --pipeline 0 --config c1 > gpurun_out/r02v_c1.log 2>&1 || { echo FAIL; tail -20 gpurun_out/r02v_c1.log; exit 1; }
echo ok
