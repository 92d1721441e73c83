# A/B: --pipeline 6 (commit overlaps the receiver's rehash tail) vs the default
set -o pipefail
O=gpurun_out/r02p6; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['values_ok'], d['oracle_sample_ok'], d['config']['wave_priority'], d['stage_ms'])"
}
for r in 1 2; do
run p1_$r X=1 --
run p6_$r X=1 -- --pipeline 6
run p6_rx0_$r RBC_RX_PRIO=0 -- --pipeline 6
run p6_rx3_$r RBC_RX_PRIO=3 -- --pipeline 6
done
run p6_c1 X=1 -- --pipeline 6 --config c1
run p6_c4 X=1 -- --pipeline 6 --config c4
