# leaf-hashing priority (proposer, phase 2) vs the receiver's decode under --pipeline 7
set -o pipefail
O=gpurun_out/r02prio5; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 60 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['values_ok'], d['stage_ms'])"
}
for r in 1 2; do
run base_$r X=1 --
run lv3_$r RBC_TX_PRIO=3 RBC_ENC_PRIO=0 --
run lv2_$r RBC_TX_PRIO=2 RBC_ENC_PRIO=0 --
run lv1_$r RBC_TX_PRIO=1 RBC_ENC_PRIO=0 --
run lv3rx3_$r RBC_TX_PRIO=2 RBC_ENC_PRIO=0 RBC_RX_PRIO=3 --
done
