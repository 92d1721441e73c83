# A/B of wave issue priorities (RBC_TX_PRIO / RBC_RX_PRIO) on the pipelined C2 bench
set -o pipefail
O=gpurun_out/r02prio; mkdir -p $O
run() {  # run <tag> <tx> <rx> [bench args]
    local tag=$1 tx=$2 rx=$3; shift 3
    RBC_TX_PRIO=$tx RBC_RX_PRIO=$rx timeout -k 10 120 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['values_ok'], d['stage_ms'])"
}
run base0 0 0
run rx3 0 3
run rx2 0 2
run tx3 3 0
run rx1 0 1
run base1 0 0
run rx3b 0 3
run rx3_c1 0 3 --config c1
run base_c1 0 0 --config c1
run rx3_c4 0 3 --config c4
run base_c4 0 0 --config c4
