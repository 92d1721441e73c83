# A/B on the occupancy-4 build: --pipeline 7 vs 1 at every config; priorities and block size under 7
set -o pipefail
O=gpurun_out/r02p7b; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['values_ok'], d['oracle_sample_ok'], d['config']['wave_priority'], d['stage_ms'])"
}
run p7 X=1 -- --pipeline 7
run p7_rx0 RBC_RX_PRIO=0 -- --pipeline 7
run p7_rx1 RBC_RX_PRIO=1 -- --pipeline 7
run p7_rx3 RBC_RX_PRIO=3 -- --pipeline 7
run p7_tpb256 RBC_RX_TPB=256 -- --pipeline 7
run p7_sets4 X=1 -- --pipeline 7 --sets 4
for c in c1 c3 c4; do
run ${c}_p7 X=1 -- --pipeline 7 --config $c
run ${c}_p1 X=1 -- --config $c
done
run p7_2k X=1 -- --pipeline 7 --instances 2048
run p7b X=1 -- --pipeline 7
