# Round 3, final code: the driver's launch form (torch.distributed.run) --
# one rank with the RCCL gather forced, and two ranks rehearsed on this one
# GPU (no RCCL: one device) -- to check the round-3 rendezvous (secret file,
# deadlines) and watchdog under torchrun's environment.
set -o pipefail
O=gpurun_out/r03zm; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-pcie --force-gather > $O/torchrun1.json 2> $O/torchrun1.err || { echo TR1FAIL; tail -20 $O/torchrun1.err; exit 1; }
python -c "import json; d=json.load(open('$O/torchrun1.json')); print('n1', d['value'], d['n_gpus'], d['gather_ok'], d['rccl']['nranks'], d['rccl']['version_str'], d['ranks'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --rehearse-on-one-gpu --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > $O/torchrun2.json 2> $O/torchrun2.err || { echo TR2FAIL; tail -30 $O/torchrun2.err; exit 1; }
python -c "import json; d=json.load(open('$O/torchrun2.json')); print('n2', d['value'], d['n_gpus'], d['decoded_ok'], d['values_ok'], d['gather_ok'], d['config']['instances_total'], d['ranks'])"
echo ok
