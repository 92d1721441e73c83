set -o pipefail
mkdir -p gpurun_out/r02l
timeout -k 10 300 python bench.py --gpus 2 --rehearse-on-one-gpu --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/r02l/spawn2.json 2> gpurun_out/r02l/spawn2.err || { echo S2FAIL; tail -30 gpurun_out/r02l/spawn2.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 3 --rehearse-on-one-gpu --total-instances 1000 --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/r02l/spawn3_strong.json 2> gpurun_out/r02l/spawn3.err || { echo S3FAIL; tail -30 gpurun_out/r02l/spawn3.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --rehearse-on-one-gpu --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/r02l/torchrun2.json 2> gpurun_out/r02l/torchrun2.err || { echo TRFAIL; tail -30 gpurun_out/r02l/torchrun2.err; exit 1; }
wc -l gpurun_out/r02l/*.json
