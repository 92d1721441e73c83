# A/B of wave issue priorities: which receive-side kernels, and with the
# commit started at the receiver's verify (RBC_BENCH_PWAIT=verify, 3 sets)
set -o pipefail
O=gpurun_out/r02prio2; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['values_ok'], d['stage_ms'])"
}
run base RBC_RX_PRIO=0 --
run rx2 RBC_RX_PRIO=2 --
run rx2v0 RBC_RX_PRIO=2 RBC_RXV_PRIO=0 --
run rx3v0 RBC_RX_PRIO=3 RBC_RXV_PRIO=0 --
run rx3v1 RBC_RX_PRIO=3 RBC_RXV_PRIO=1 --
run pw_base RBC_BENCH_PWAIT=verify -- --sets 3
run pw_rx2 RBC_BENCH_PWAIT=verify RBC_RX_PRIO=2 -- --sets 3
run pw_rx3v0 RBC_BENCH_PWAIT=verify RBC_RX_PRIO=3 RBC_RXV_PRIO=0 -- --sets 3
run pw_rx3 RBC_BENCH_PWAIT=verify RBC_RX_PRIO=3 -- --sets 3
run base2 RBC_RX_PRIO=0 --
run rx2b RBC_RX_PRIO=2 --
run rx2v0b RBC_RX_PRIO=2 RBC_RXV_PRIO=0 --
