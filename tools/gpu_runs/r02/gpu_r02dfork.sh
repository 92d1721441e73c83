# GPU suite on the current code, then A/B: batch digest beside the root recheck (default) vs after it
set -o pipefail
O=gpurun_out/r02dfork; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['values_ok'], d['oracle_sample_ok'], d['config']['wave_priority'], d['stage_ms'])"
}
for r in 1 2; do
run fork$r RBC_DIGEST_FORK=1 --
run nofork$r RBC_DIGEST_FORK=0 --
run prio0_$r RBC_RX_PRIO=0 --
done
run c4 X=1 -- --config c4
run c1 X=1 -- --config c1
