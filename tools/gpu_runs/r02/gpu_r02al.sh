set -o pipefail
NO_PMC=1 timeout -k 10 400 bash tools/profile.sh r02al_c4 --steps 10 --warmup 3 --no-cpu-baseline --no-pcie --no-isolated --config c4 > gpurun_out/r02al_c4.log 2>&1 || { echo FAIL; tail -20 gpurun_out/r02al_c4.log; exit 1; }
NO_PMC=1 timeout -k 10 400 bash tools/profile.sh r02al_c4s --steps 10 --warmup 3 --no-cpu-baseline --no-pcie --no-isolated --config c4 --pipeline 0 > gpurun_out/r02al_c4s.log 2>&1 || { echo FAIL; tail -20 gpurun_out/r02al_c4s.log; exit 1; }
echo ok
