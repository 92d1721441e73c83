# A/B after giving decode_prepare / compact_present / digest the receive priority too
set -o pipefail
O=gpurun_out/r02p7; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['values_ok'], d['oracle_sample_ok'], d['config']['wave_priority'], d['stage_ms'])"
}
for r in 1 2 3; do
run p1_$r X=1 --
run p6_$r X=1 -- --pipeline 6
done
run c4 X=1 -- --config c4
run c4_fuse RBC_FUSE_JOIN=1 -- --config c4
run c4_p6 X=1 -- --config c4 --pipeline 6
run c1 X=1 -- --config c1
run c1_p6 X=1 -- --config c1 --pipeline 6
