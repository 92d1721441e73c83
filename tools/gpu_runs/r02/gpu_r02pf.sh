# SHA block prefetch (default) vs none (ab/librbc_gpu_np.so: leaves 108 -> 95 VGPRs)
set -o pipefail
O=gpurun_out/r02pf; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 60 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['values_ok'], 'iso leaf', d['roofline']['isolated']['avg_ms'], 'commit', d['commit_only']['ms_per_batch'], 'recv', d['receive_only']['ms_per_batch'])"
}
for r in 1 2 3; do
run pf_$r X=1 --
run np_$r RBC_GPU_LIB_AB=ab/librbc_gpu_np.so --
done
run np_c1 RBC_GPU_LIB_AB=ab/librbc_gpu_np.so -- --config c1
run pf_c1 X=1 -- --config c1
run np_c4 RBC_GPU_LIB_AB=ab/librbc_gpu_np.so -- --config c4
run pf_c4 X=1 -- --config c4
