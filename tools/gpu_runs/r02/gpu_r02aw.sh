set -o pipefail
mkdir -p gpurun_out/r02aw
B="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pcie --no-isolated"
for rc in 4 8; do RBC_GF_MDRC=$rc $B --config c4 --pipeline 0 > gpurun_out/r02aw/c4_s_$rc.json 2>/dev/null || exit 1; RBC_GF_MDRC=$rc $B --config c4 > gpurun_out/r02aw/c4_p_$rc.json 2>/dev/null || exit 1; done
for rc in 8 12 16; do RBC_GF_MDRC=$rc $B --pipeline 0 > gpurun_out/r02aw/c2_s_$rc.json 2>/dev/null || exit 1; RBC_GF_MDRC=$rc $B > gpurun_out/r02aw/c2_p_$rc.json 2>/dev/null || exit 1; done
for f in gpurun_out/r02aw/*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['stage_ms']['interp'], d['values_ok'])"; done
