# A/B: receiver decode kernels' occupancy beside the proposer's leaf hashing
# (FFT decode at 4 waves/SIMD: ab/librbc_gpu_fdec4.so; GF missing-data rows per chunk: RBC_GF_MDRC)
set -o pipefail
O=gpurun_out/r02occ2; mkdir -p $O
run() {  # run <tag> <env...> -- [bench args]
    local tag=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 60 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])"
}
for r in 1 2; do
run base_$r X=1 --
run fdec4_$r RBC_GPU_LIB_AB=ab/librbc_gpu_fdec4.so --
run gd1_$r RBC_GPU_LIB_AB=ab/librbc_gpu_gd1.so --
run md4_$r RBC_GF_MDRC=4 --
run md6_$r RBC_GF_MDRC=6 --
run fdec4_md4_$r RBC_GPU_LIB_AB=ab/librbc_gpu_fdec4.so RBC_GF_MDRC=4 --
done
