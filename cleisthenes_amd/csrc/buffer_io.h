// buffer_io.h -- raw-buffer access helpers shared by the HIP translation
// units of the batched RBC kernels (kernels.hip, gf_regen.hip): a buffer
// descriptor per instance (bounds-checked, base in SGPRs), loads with a
// wave-uniform row start as the scalar soffset, byte masks for the Split pad.
#pragma once
#include "device_common.h"

namespace {

using rsrc_t = __amdgpu_buffer_rsrc_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int RBC_RSRC_DW3 = 0x00020000;  // gfx9 raw buffer, bounds-checked

RBC_DEV rsrc_t make_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, RBC_RSRC_DW3);
}
RBC_DEV uint4 bload16(rsrc_t r, uint32_t off) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
// per-lane offset + a wave-uniform one (a row start), which the buffer
// instruction takes as its scalar soffset: no per-lane address arithmetic
RBC_DEV uint4 bload16s(rsrc_t r, uint32_t voff, uint32_t soff) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
RBC_DEV uint32_t uniform(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
RBC_DEV uint32_t inst_len(const uint32_t *lens, uint32_t uniform, int i) { return lens ? lens[i] : uniform; }

// byte mask keeping the first `nv` bytes (little-endian) of a word
RBC_DEV uint32_t keep_bytes(int nv) {
    return nv >= 4 ? 0xffffffffu : (nv <= 0 ? 0u : ((1u << (8 * nv)) - 1u));
}
RBC_DEV uint4 mask16(uint4 v, int nvalid) {
    v.x &= keep_bytes(nvalid);
    v.y &= keep_bytes(nvalid - 4);
    v.z &= keep_bytes(nvalid - 8);
    v.w &= keep_bytes(nvalid - 12);
    return v;
}
// gfx950 runs with unaligned global/buffer access enabled (hipcc itself
// emits dwordx4 for byte-aligned pointers), so a 16-byte row read at any
// byte offset is a single buffer_load_dwordx4; bounds are still checked by
// the buffer descriptor (out of range -> 0).

template <int V>
struct IntC {  // a compile-time int as a value (generic-lambda dispatch)
    static constexpr int value = V;
};

}  // namespace
