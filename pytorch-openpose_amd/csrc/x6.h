// x6.h — device helpers of the split-bf16 ("X6") convolution kernels (conv_x6.hip, conv_win.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"

namespace opose {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

namespace x6 {

constexpr int x6_waves(int mt, int pt) { return mt * pt >= 32768 ? 8 : 4; }

__device__ __forceinline__ uint32_t bf16_rne(float x) {
    uint32_t u = __float_as_uint(x);
    u += 0x7fffu + ((u >> 16) & 1u);
    return u >> 16;
}

// x -> three bf16 pieces, x0 + x1 + x2 == x exactly (each remainder is exact by Sterbenz)
__device__ __forceinline__ void split3(float x, uint32_t& h0, uint32_t& h1, uint32_t& h2) {
    h0 = bf16_rne(x);
    const float r = x - __uint_as_float(h0 << 16);
    h1 = bf16_rne(r);
    const float r2 = r - __uint_as_float(h1 << 16);
    h2 = bf16_rne(r2);
}

__device__ __forceinline__ float join3(uint32_t h0, uint32_t h1, uint32_t h2) {
    return (__uint_as_float(h0 << 16) + __uint_as_float(h1 << 16)) + __uint_as_float(h2 << 16);
}

// write 4 consecutive channels (4hk .. 4hk+3 of a group) of one pixel, split, into the 3 planes
__device__ __forceinline__ void store4_x6(uint8_t* unit, uint32_t ps, const float (&v)[4]) {
    uint32_t h[3][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) split3(v[t], h[0][t], h[1][t], h[2][t]);
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
        uint2 w;
        w.x = h[pc][0] | (h[pc][1] << 16);
        w.y = h[pc][2] | (h[pc][3] << 16);
        *reinterpret_cast<uint2*>(unit + (size_t)pc * ps) = w;
    }
}

// Slab partials (X6Args::partial): per work unit of a multi-slab group an fp32 [MT/4][PT] array
// of channel quads -- quad q (channels 4q .. 4q+3 of the tile), pixel pl at float index
// (q * PT + pl) * 4.  A lane's accumulator block holds 4 consecutive channels of one pixel, so
// it leaves the kernel as one 16-byte write-through (sc1) store; conv_x6_fixup reads two quads
// per X6 unit.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(float* partial) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)partial, (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void store_slab_quad(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, f32x4 v) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)byte_off, 0, 16);  // aux 16: sc1
}

// unit index of (frame n, group g of the slice, y, x) in an X6 plane (common.h X6Layout)
__device__ __forceinline__ uint32_t x6_unit(const X6Layout& l, int n, int g, int y, int x) {
    return l.o0 + (uint32_t)n * l.fs + (uint32_t)g * l.gs + (uint32_t)y * l.rs + (uint32_t)x;
}

// group of a tile (groups are numbered in tile order, X6Group::t0)
__device__ __forceinline__ int x6_group_of(const X6Args& a, int tile) {
    int g = 0;
    for (int i = 1; i < a.ngroups; ++i) g = tile >= a.g[i].t0 ? i : g;
    return g;
}

// A work unit: chunks [c0, c1) of one tile, slab s of the group's `slabs` (common.h X6Group)
struct X6Unit {
    int g, tile, c0, c1;
    bool whole;  // the tile's only slab: the conv writes the output itself
};
__device__ __forceinline__ X6Unit x6_unit_of(const X6Args& a, int u) {
    int g = 0;
    for (int i = 1; i < a.ngroups; ++i) g = u >= a.g[i].u0 ? i : g;
    const int S = a.g[g].slabs, ul = u - a.g[g].u0, tl = ul / S, s = ul - tl * S;
    return X6Unit{g, a.g[g].t0 + tl, s * a.nK / S, (s + 1) * a.nK / S, S == 1};
}

// the unit list of workgroup w of gridDim.x: positions [k0, k1) of `list` (nullptr: the units
// themselves, a contiguous range)
struct X6Work {
    int k0, k1;
    const int* list;
};
__device__ __forceinline__ X6Work x6_work_of(const X6Args& a, int w) {
    const int G = gridDim.x;
    if (a.sched) return X6Work{a.sched[w], a.sched[w + 1], a.sched + G + 1};
    return X6Work{(int)((long long)w * a.units / G), (int)((long long)(w + 1) * a.units / G), nullptr};
}

}  // namespace x6
using namespace x6;

}  // namespace opose
