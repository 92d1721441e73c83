# SHA block loop unrolled x2 (ping-pong prefetch, default) vs one block per iteration (ab/librbc_gpu_u1.so)
set -o pipefail
O=gpurun_out/r02unroll; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { echo TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 60 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['values_ok'], 'iso leaf', d['roofline']['isolated']['avg_ms'], 'commit', d['commit_only']['ms_per_batch'], 'recv', d['receive_only']['ms_per_batch'])"
}
for r in 1 2 3; do
run new_$r X=1 --
run old_$r RBC_GPU_LIB_AB=ab/librbc_gpu_u1.so --
done
