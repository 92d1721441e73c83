# A/B: SHA kernel occupancy (waves per SIMD) under --pipeline 7 and the default schedule
set -o pipefail
O=gpurun_out/r02wpe; mkdir -p $O
run() {  # run <tag> <lib or -> [bench args]
    local tag=$1 lib=$2; shift 2
    local env=()
    [ "$lib" != "-" ] && env=(RBC_GPU_LIB_AB=$lib)
    env "${env[@]}" X=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --no-isolated --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])"
}
for r in 1 2; do
run w4_p7_$r - --pipeline 7
run w3_p7_$r ab/librbc_gpu_w3.so --pipeline 7
run w5_p7_$r ab/librbc_gpu_w5.so --pipeline 7
run w6_p7_$r ab/librbc_gpu_w6.so --pipeline 7
run r5_p7_$r ab/librbc_gpu_r5.so --pipeline 7
run w4_p1_$r -
run w5_p1_$r ab/librbc_gpu_w5.so
done
