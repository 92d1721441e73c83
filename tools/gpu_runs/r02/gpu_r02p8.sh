# receive_step: GPU parity test, then A/B --pipeline 7 vs the default
set -o pipefail
O=gpurun_out/r02p8; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "receive_step or phases_equal" > $O/test.log 2>&1 || { echo TESTFAIL; tail -40 $O/test.log; exit 1; }
grep -E "PASS|FAIL" $O/test.log | tail -8
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['values_ok'], d['oracle_sample_ok'], d['decoded_ok'], d['config']['wave_priority'], d['stage_ms'])"
}
for r in 1 2; do
run p1_$r X=1 --
run p7_$r X=1 -- --pipeline 7
run p7_rx0_$r RBC_RX_PRIO=0 -- --pipeline 7
done
run p7_rx3 RBC_RX_PRIO=3 -- --pipeline 7
run p7_c1 X=1 -- --pipeline 7 --config c1
run c1 X=1 -- --config c1
run p7_c4 X=1 -- --pipeline 7 --config c4
run c4 X=1 -- --config c4
run p7_c3 X=1 -- --pipeline 7 --config c3
run p6_1 X=1 -- --pipeline 6
