# receive-step hashing priority vs the receiver's decode priority under --pipeline 7
set -o pipefail
O=gpurun_out/r02prio4; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 60 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['values_ok'], d['stage_ms'])"
}
for r in 1 2; do
run base_$r X=1 --
run rxv0_$r RBC_RXV_PRIO=0 --
run rxv1_$r RBC_RXV_PRIO=1 --
run rxv3_$r RBC_RXV_PRIO=3 RBC_RX_PRIO=2 --
run rx3v2_$r RBC_RXV_PRIO=2 RBC_RX_PRIO=3 --
done
