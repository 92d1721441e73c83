set -o pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02e/gputest.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02e/gputest.log; exit 1; }
tail -2 gpurun_out/r02e/gputest.log
timeout -k 10 300 python bench.py > gpurun_out/r02e/bench.json 2> gpurun_out/r02e/bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r02e/bench.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-pcie --force-gather > gpurun_out/r02e/torchrun.json 2> gpurun_out/r02e/torchrun.err || { echo TRFAIL; tail -20 gpurun_out/r02e/torchrun.err; exit 1; }
wc -l gpurun_out/r02e/torchrun.json
