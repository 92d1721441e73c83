# priorities under --pipeline 7 (occupancy-4 build): encode / leaves / receive
set -o pipefail
O=gpurun_out/r02prio3; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['values_ok'], d['stage_ms'])"
}
for r in 1 2; do
run base_$r X=1 --
run enc3_$r RBC_ENC_PRIO=3 --
run enc3_tx1_rx2_$r RBC_ENC_PRIO=3 RBC_TX_PRIO=1 --
run enc2_rx1_$r RBC_ENC_PRIO=2 RBC_RX_PRIO=1 --
run rx1_$r RBC_RX_PRIO=1 --
run enc1_$r RBC_ENC_PRIO=1 --
done
