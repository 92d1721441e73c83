#!/bin/bash
# Build A/B variants of librbc_gpu.so that differ in the kernel sources'
# compile flags (kernels.hip and rs_fft.hip):
#   tools/build_ab.sh <name> "<-D flags>" ... -> ab/librbc_gpu_<name>.so
# (select one with RBC_GPU_LIB=ab/librbc_gpu_<name>.so).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/cleisthenes_amd/csrc
mkdir -p $ROOT/ab
make -C $C -s
FL="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function"
while [ $# -ge 2 ]; do
    name=$1; defs=$2; shift 2
    /opt/rocm/bin/hipcc $FL $defs -c $C/kernels.hip -o $ROOT/ab/kernels_$name.o &
    /opt/rocm/bin/hipcc $FL $defs -c $C/rs_fft.hip -o $ROOT/ab/rs_fft_$name.o &
    /opt/rocm/bin/hipcc $FL $defs -c $C/gf_regen.hip -o $ROOT/ab/gf_regen_$name.o &
    wait
    /opt/rocm/bin/hipcc $FL -shared -o $ROOT/ab/librbc_gpu_$name.so $ROOT/ab/kernels_$name.o $ROOT/ab/rs_fft_$name.o \
        $ROOT/ab/gf_regen_$name.o $C/wire.o \
        $C/capi.o $C/batcher.o $C/rbc_node.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
    echo "built ab/librbc_gpu_$name.so"
done
