// wire.hip -- per-recipient VAL / ECHO marshaling in HBM (SURVEY §8f ranks 2
// and 4: the pb payload codec and the proposer's send path).
//
// A proposer's VAL fan-out is N messages per instance, each carrying one
// shard as base64 inside the Go-JSON request (rbc/request.go:9-17) inside a
// pb.Message (pb/message.proto:11-35): 4/3 of the committed shard bytes,
// i.e. ~4.3 GB per C2 batch of 1024 proposals.  Serialising that on the host
// costs seconds of CPU per batch; here one wave per message writes the exact
// bytes of rbc_pb_encode_rbc(type, rbc_json_encode_val(...)) (csrc/rbc_node.cpp)
// straight from the device-resident shards, branches and roots, so the host
// only copies finished messages out (or hands device buffers to a
// GPU-direct transport).
//
// Byte work, HBM-bound: every lane produces one aligned 16-byte chunk of its
// message per step.  Chunks wholly inside a base64 run (the shard, the
// branch) take the fast path: 3 dword loads' worth of source (5 dwords, one
// funnel shift), 5 base64 groups as packed sextets, SWAR ASCII mapping, one
// funnel shift to the chunk's phase and one 16-byte store.  The few chunks
// that straddle a header, a JSON literal or a run's end take a per-byte path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace {

__device__ __forceinline__ uint32_t b64_len(uint32_t n) { return (n + 2) / 3 * 4; }
__device__ __forceinline__ uint32_t varint_len(uint32_t v) {
    uint32_t l = 1;
    while (v >= 0x80) {
        v >>= 7;
        ++l;
    }
    return l;
}

// JSON literals of the request (rbc/request.go field order)
__constant__ const char kLit[] =
    "{\"RootHash\":\""                  // 0, 13
    "\",\"Branch\":\""                  // 13, 12
    "\",\"Block\":[\""                  // 25, 12
    "\"]}"                              // 37, 3
    "\",\"Branch\":null,\"Block\":[\""; // 40, 26

// Message layout for one (instance, row): piece start offsets.
struct Layout {
    uint32_t total;            // message bytes
    uint32_t hdr;              // 0x1a varint(R) 0x0a varint(J)
    uint32_t R, J;
    uint32_t root_off;         // base64 of the root (44 chars)
    uint32_t br_lit_off;       // '","Branch":"' or the null variant
    uint32_t br_off, br_len;   // base64 of the branch (br_len source bytes)
    uint32_t blk_lit_off;      // '","Block":["' (absent for a null branch)
    uint32_t blk_off, S;       // base64 of the shard
    uint32_t end_lit_off;      // '"]}'
    uint32_t type_off;         // 0x10 type, when type != 0
};

__device__ __forceinline__ Layout layout(uint32_t S, uint32_t br_len, int type) {
    Layout L;
    L.S = S;
    L.br_len = br_len;
    const uint32_t Bk = b64_len(S), Bb = b64_len(br_len);
    L.J = br_len ? 84 + Bb + Bk : 86 + Bk;
    L.R = 1 + varint_len(L.J) + L.J + (type ? 2 : 0);
    L.hdr = 1 + varint_len(L.R) + 1 + varint_len(L.J);
    L.total = 1 + varint_len(L.R) + L.R;
    L.root_off = L.hdr + 13;
    L.br_lit_off = L.root_off + 44;
    if (br_len) {
        L.br_off = L.br_lit_off + 12;
        L.blk_lit_off = L.br_off + Bb;
        L.blk_off = L.blk_lit_off + 12;
    } else {
        L.br_off = L.blk_lit_off = L.br_lit_off + 26;
        L.blk_off = L.br_lit_off + 26;
    }
    L.end_lit_off = L.blk_off + Bk;
    L.type_off = L.end_lit_off + 3;
    return L;
}

__device__ __forceinline__ uint32_t b64_char(uint32_t v) {
    return v < 26 ? 'A' + v : v < 52 ? 'a' + v - 26 : v < 62 ? '0' + v - 52 : v == 62 ? '+' : '/';
}

// character c of base64(src[0..len)) (standard alphabet, '=' padding)
__device__ __forceinline__ uint32_t b64_at(const uint8_t *src, uint32_t len, uint32_t c) {
    const uint32_t g = c >> 2, r = c & 3, b = 3 * g;
    const uint32_t n = len - b;  // source bytes in this group (>= 1)
    if (r >= 2 && n <= r - 1) return '=';
    const uint32_t b0 = src[b], b1 = n > 1 ? src[b + 1] : 0, b2 = n > 2 ? src[b + 2] : 0;
    const uint32_t w = b0 << 16 | b1 << 8 | b2;
    return b64_char((w >> (18 - 6 * r)) & 63);
}

__device__ __forceinline__ uint32_t varint_byte(uint32_t v, uint32_t i) {
    const uint32_t b = (v >> (7 * i)) & 0x7f;
    return (v >> (7 * (i + 1))) ? (b | 0x80) : b;
}

// byte p of the message (the slow, per-byte path)
__device__ uint32_t msg_byte(const Layout &L, uint32_t p, int type, const uint8_t *root, const uint8_t *br,
                             const uint8_t *blk) {
    if (p >= L.total) return 0;
    if (p < L.hdr) {
        const uint32_t vr = varint_len(L.R);
        if (p == 0) return 0x1a;
        if (p < 1 + vr) return varint_byte(L.R, p - 1);
        if (p == 1 + vr) return 0x0a;
        return varint_byte(L.J, p - 2 - vr);
    }
    if (p < L.root_off) return (uint8_t)kLit[p - L.hdr];
    if (p < L.br_lit_off) return b64_at(root, 32, p - L.root_off);
    if (!L.br_len) {
        if (p < L.blk_off) return (uint8_t)kLit[40 + p - L.br_lit_off];
    } else {
        if (p < L.br_off) return (uint8_t)kLit[13 + p - L.br_lit_off];
        if (p < L.blk_lit_off) return b64_at(br, L.br_len, p - L.br_off);
        if (p < L.blk_off) return (uint8_t)kLit[25 + p - L.blk_lit_off];
    }
    if (p < L.end_lit_off) return b64_at(blk, L.S, p - L.blk_off);
    if (p < L.type_off) return (uint8_t)kLit[37 + p - L.end_lit_off];
    return p == L.type_off ? 0x10u : (uint32_t)type;
}

// 4 sextets (already in output order, one per byte) -> 4 base64 ASCII bytes
__device__ __forceinline__ uint32_t b64_ascii4(uint32_t v) {
    const uint32_t t26 = (v + 0x66666666u) & 0x80808080u;  // byte >= 26
    const uint32_t t52 = (v + 0x4c4c4c4cu) & 0x80808080u;  // >= 52
    const uint32_t t62 = (v + 0x42424242u) & 0x80808080u;  // >= 62
    const uint32_t t63 = (v + 0x41414141u) & 0x80808080u;  // == 63
    // 'A' + v, +6 from 26 ('a'), -75 from 52 ('0'), -15 at 62 ('+'), +3 at 63 ('/');
    // additions first, so no byte borrows from its neighbour
    const uint32_t pos = v + 0x41414141u + (t26 >> 5) + (t26 >> 6) + (t63 >> 6) + (t63 >> 7);
    const uint32_t neg = (t52 >> 1) + (t52 >> 4) + (t52 >> 6) + (t52 >> 7) + (t62 >> 3) - (t62 >> 7);
    return pos - neg;
}

// 24-bit big-endian group w -> its 4 sextets, first in the lowest byte
__device__ __forceinline__ uint32_t sextets(uint32_t w) {
    return ((w >> 18) & 0x3fu) | ((w >> 4) & 0x3f00u) | ((w << 10) & 0x3f0000u) | ((w << 24) & 0x3f000000u);
}

// Fast path: the 16 characters of base64(src) starting at character c0, all
// from full groups and with 20 readable source bytes from 3*(c0/4) on.
__device__ __forceinline__ uint4 b64_chunk16(const uint8_t *src, uint32_t c0) {
    const uint32_t g0 = c0 >> 2, e = c0 & 3, sb = 3 * g0, a = sb & 3;
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(src) + (sb >> 2);
    const uint32_t d0 = s32[0], d1 = s32[1], d2 = s32[2], d3 = s32[3], d4 = s32[4];
    // E = source bytes sb .. sb+15
    const uint32_t e0 = __builtin_amdgcn_alignbyte(d1, d0, a), e1 = __builtin_amdgcn_alignbyte(d2, d1, a);
    const uint32_t e2 = __builtin_amdgcn_alignbyte(d3, d2, a), e3 = __builtin_amdgcn_alignbyte(d4, d3, a);
    // five groups as 24-bit big-endian words (byte-permute selectors: {hi:lo})
    const uint32_t w0 = __builtin_amdgcn_perm(e1, e0, 0x0c000102u);
    const uint32_t w1 = __builtin_amdgcn_perm(e1, e0, 0x0c030405u);
    const uint32_t w2 = __builtin_amdgcn_perm(e2, e1, 0x0c020304u);
    const uint32_t w3 = __builtin_amdgcn_perm(e3, e2, 0x0c010203u);
    const uint32_t w4 = __builtin_amdgcn_perm(e3, e3, 0x0c000102u);
    const uint32_t g[5] = {b64_ascii4(sextets(w0)), b64_ascii4(sextets(w1)), b64_ascii4(sextets(w2)),
                           b64_ascii4(sextets(w3)), b64_ascii4(sextets(w4))};
    // characters e .. e+15 of the 20
    return make_uint4(__builtin_amdgcn_alignbyte(g[1], g[0], e), __builtin_amdgcn_alignbyte(g[2], g[1], e),
                      __builtin_amdgcn_alignbyte(g[3], g[2], e), __builtin_amdgcn_alignbyte(g[4], g[3], e));
}

// is [p, p+16) a fast-path chunk of the base64 run of `len` bytes at `off`?
__device__ __forceinline__ bool fast_run(uint32_t p, uint32_t off, uint32_t len) {
    if (p < off) return false;
    const uint32_t c0 = p - off;
    const uint32_t full_chars = len / 3 * 4;
    if (c0 + 16 > full_chars) return false;
    const uint32_t w0 = (3 * (c0 >> 2)) >> 2;  // first source dword
    return 4 * (w0 + 5) <= len;                 // five dwords inside the run
}

// one wave per message; 4 waves (messages) per block
__global__ __launch_bounds__(256) void marshal_val_kernel(WireArgs a) {
    const uint32_t msg = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (msg >= (uint32_t)a.count * (uint32_t)a.n) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t inst = msg / a.n, j = msg - inst * a.n;
    const uint32_t S = a.lens ? a.lens[inst] : a.uniform_len;
    const bool empty0 = a.depth > 0 && (int)(j ^ 1u) >= a.n;
    const uint32_t br_len = 32u * (a.depth - (empty0 ? 1 : 0));
    const Layout L = layout(S, br_len, a.type);
    const uint8_t *root = a.roots + (size_t)inst * 32;
    const uint8_t *br = a.branches + ((size_t)inst * a.n + j) * a.depth * 32u + (empty0 ? 32u : 0u);
    const uint8_t *blk = a.shards + (size_t)inst * a.inst_pitch + (size_t)j * a.row_pitch;
    uint8_t *out = a.out + (size_t)msg * a.out_pitch;
    const uint32_t nchunks = (L.total + 15) >> 4;
    for (uint32_t q = lane; q < nchunks; q += 64) {
        const uint32_t p = q << 4;
        uint4 v;
        if (fast_run(p, L.blk_off, S)) {
            v = b64_chunk16(blk, p - L.blk_off);
        } else if (br_len && fast_run(p, L.br_off, br_len)) {
            v = b64_chunk16(br, p - L.br_off);
        } else {
            uint32_t d[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t x = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) x |= msg_byte(L, p + 4 * w + b, a.type, root, br, blk) << (8 * b);
                d[w] = x;
            }
            v = make_uint4(d[0], d[1], d[2], d[3]);
        }
        *reinterpret_cast<uint4 *>(out + p) = v;
    }
    if (lane == 0 && a.out_lens) a.out_lens[msg] = L.total;
}

}  // namespace

hipError_t rbc_launch_marshal_val(const WireArgs &a, hipStream_t st) {
    const uint64_t msgs = (uint64_t)a.count * a.n;
    if (!msgs) return hipSuccess;
    hipLaunchKernelGGL(marshal_val_kernel, dim3((unsigned)((msgs + 3) / 4)), dim3(256), 0, st, a);
    return hipGetLastError();
}


