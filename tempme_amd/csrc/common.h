// Shared internals of libtempme_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/tempme.h"

namespace tmk {

void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

// test / diagnostic options (tm_debug_set, graph.cpp): process-wide, all 0 in the product path
int debug_opt(int opt);

// library-internal device scratch per (device, stream), grown on demand (scratch.cpp); nullptr on failure
void *scratch(size_t bytes, hipStream_t stream);

// per-kernel HIP-event timing (prof.cpp); no-ops unless tm_profile_enable(1)
hipEvent_t prof_begin(hipStream_t s);
void prof_end(const char *name, hipStream_t s, hipEvent_t a);

#define TM_HIP(expr)                                                                            \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return ::tmk::fail(TM_E_HIP, std::string(#expr ": ") + hipGetErrorString(_e));       \
    } while (0)

#define TM_CHECK_LAUNCH()                                                                       \
    do {                                                                                        \
        hipError_t _e = hipGetLastError();                                                      \
        if (_e != hipSuccess)                                                                   \
            return ::tmk::fail(TM_E_HIP, std::string("kernel launch: ") + hipGetErrorString(_e)); \
    } while (0)

// ------------------------------------------------------------------ device graph layout
// One 16-byte record per adjacency entry, so a sampled slot is one dwordx4 load: the neighbour, the
// edge id, the timestamp as the fp32 every sampled output carries, and the entry's rank inside its
// (node, neighbour) block (the number of earlier entries of the node with the same neighbour).  The
// fp64 timestamps the bisects compare live in their own array (8 B per entry: twice the density).
struct __attribute__((aligned(16))) Rec {
    int32_t ngh;
    int32_t eid;
    float ts;
    int32_t brank;
};

// e_idx -> (owner, slice length) for the (at most two) owners of an edge id.
// len = length of neighbors[:nodeedge2idx[owner][eid]] (the dict value, clamped the way
// Python slicing treats a negative stop).  node = -1: absent.
struct __attribute__((aligned(16))) EdgeEnds {
    int32_t node_a, len_a, node_b, len_b;
};

// (node, neighbour) -> that neighbour's block of the node: its n positions (ascending) stored as a
// 16-ary search tree at ppos[base..]: open addressing, linear probing, u = -1 marks an empty slot,
// capacity a power of two.
struct __attribute__((aligned(16))) PairBlk {
    int32_t u, x, base, n;
};

__host__ __device__ inline uint32_t pblk_hash(int32_t u, int32_t x) {
    uint32_t h = (uint32_t)u * 0x9E3779B1u ^ ((uint32_t)x + 0x7F4A7C15u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h;
}

// Block search tree (ppos), fan-out F = 2^kBlkLog.  A block of n <= F positions is its keys, padded
// with INT32_MAX to a multiple of 4 (16-B aligned).  A larger block stores levels L_h .. L_1, L_0 (in
// that order, 4F-B aligned, each padded with INT32_MAX to a multiple of F): L_0 = the positions,
// L_l[t] = L_(l-1)[F t], h = the first level with <= F entries.  A lower bound reads one F-key node per
// level (h + 1 lines instead of log2(n) dependent loads of a binary search).
// (fan-out 8 with 32-B nodes and 16 with 64-B nodes measured 1.5 % / 5 % slower than 4)
constexpr int32_t kBlkLog = 2, kBlkFan = 1 << kBlkLog;
__host__ __device__ inline int32_t blk_levels(int32_t n) {
    int32_t h = 0;
    while (n > kBlkFan) {
        n = (n + kBlkFan - 1) >> kBlkLog;
        ++h;
    }
    return h;
}
// padded length of level l of a block of n > F keys with h levels
__host__ __device__ inline int32_t blk_level_len(int32_t n, int32_t l, int32_t h) {
    if (l == h) return kBlkFan;
    const int32_t s = (int32_t)(((int64_t)n + ((int64_t)1 << (kBlkLog * l)) - 1) >> (kBlkLog * l));
    return (s + kBlkFan - 1) & ~(kBlkFan - 1);
}
// offset of the keys (L_0) from the block's base
__host__ __device__ inline int32_t blk_keys_off(int32_t n) {
    if (n <= kBlkFan) return 0;
    const int32_t h = blk_levels(n);
    int32_t o = 0;
    for (int32_t l = 1; l <= h; ++l) o += blk_level_len(n, l, h);
    return o;
}
// ints the block occupies
__host__ __device__ inline int32_t blk_region_len(int32_t n) {
    if (n <= kBlkFan) return (n + 3) & ~3;
    return blk_keys_off(n) + blk_level_len(n, 0, blk_levels(n));
}

struct DevGraph {
    int32_t n_nodes;
    int32_t max_eid;
    int64_t n_entries;
    const int32_t *off;     // [V+1]
    const int2 *span;       // [V] {off[u], off[u+1]}: a node's range in one 8-B load
    const Rec *rec;         // [n_entries]
    const double *tsd;      // [n_entries] fp64 timestamps (bisect keys)
    const EdgeEnds *ends;   // [max_eid+1]
    const int32_t *ppos;    // block search trees
    const double *ets;      // [max_eid+1] timestamp of each edge id (0 for absent ids)
    int32_t ts_unique;      // every record of an edge id carries the same timestamp
    const PairBlk *pblk;    // [pblk_mask+1] (node, neighbour) block table
    uint32_t pblk_mask;
    int32_t strict;         // strict_temporal view (tm_graph_strict_view): ends hold bisect_left(ts_u, t(e)),
                            // and final_step cuts an edge the node does not hold at t(e), not the whole list
};

// A uniform pointer moved into VGPRs: kernels with many pointer arguments otherwise overflow the
// scalar register file and spill it through v_readlane/v_writelane in their loops.
template <class T>
__device__ __forceinline__ T *vptr(T *p) {
    uint64_t v = reinterpret_cast<uint64_t>(p);
    asm volatile("" : "+v"(v));
    return reinterpret_cast<T *>(v);
}
// The same, typed as a global-address-space pointer: a pointer laundered through the asm loses its
// address space, and stores through a generic pointer are FLAT stores, which count on lgkmcnt as well
// as vmcnt (out of order), so every later LDS wait also waited for them.
template <class T>
using gptr = __attribute__((address_space(1))) T *;
template <class T>
__device__ __forceinline__ gptr<T> gvptr(T *p) {
    uint64_t v = reinterpret_cast<uint64_t>(p);
    asm volatile("" : "+v"(v));
    return (gptr<T>)v;
}
#define TM_OUTP(p) gvptr(p)

// ------------------------------------------------------------------ Philox4x32-10
// all four output words of one Philox4x32-10 block
__device__ __forceinline__ uint4 philox4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    // a wave-uniform key stays in SGPRs and its schedule is scalar adds (the keyed sampler kernels
    // fit it without spills; forcing the key into VGPRs cost 20 VALU per block: events_kernel 3 %)
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        // one 32x32->64 multiply (v_mad_u64_u32) per product instead of separate mul_hi and mul_lo:
        // integer multiplies are quarter rate and dominate the round
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ uint32_t philox_word(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                uint32_t k1, uint32_t w) {
    const uint4 r = philox4(c0, c1, c2, c3, k0, k1);
    return w == 0 ? r.x : w == 1 ? r.y : w == 2 ? r.z : r.w;
}

struct Key {
    uint32_t k0, k1, tagbase;  // tagbase = split << 16 | side << 8
};

__host__ __device__ inline Key make_key(uint64_t seed, uint32_t split, uint32_t side) {
    return Key{(uint32_t)seed, (uint32_t)(seed >> 32), (split << 16) | (side << 8)};
}

// the draw of word u for [0, high)
__device__ __forceinline__ int32_t scale_draw(uint32_t u, uint32_t high) {
    return (int32_t)(((uint64_t)u * (uint64_t)high) >> 32);
}

// the four words of block (stage, event, row, j >> 2): draws j = 4*(j>>2) .. +3 of the contract
__device__ __forceinline__ uint4 draw_block(Key k, uint32_t stage, uint32_t event, uint32_t row, uint32_t jb) {
    return philox4(event, k.tagbase | stage, row, jb, k.k0, k.k1);
}

// draw in [0, high) for (stage, event, row, j)
__device__ __forceinline__ int32_t draw(Key k, uint32_t stage, uint32_t event, uint32_t row, uint32_t j,
                                        uint32_t high) {
    uint32_t u = philox_word(event, k.tagbase | stage, row, j >> 2, k.k0, k.k1, j & 3);
    return (int32_t)(((uint64_t)u * (uint64_t)high) >> 32);
}

// cos of an fp32 argument, branch-free: the argument in revolutions, x / (2 pi), reduced to [-1/2, 1/2]
// in fp64 (relative error 2^-53: |x| < 2^40 keeps the reduced fraction exact to ~1e-9), then the
// hardware v_cos_f32 (input in revolutions).  Max abs error vs cos of the same fp32 argument 1.8e-7
// over the time encoder's whole argument range (micro/cosacc.hip, profiles/r03_cos_accuracy.txt: the
// round-2 fp64-reduction + r^12 polynomial form measured 1.5e-7 at about twice the VALU cost; torch's
// cosf 3.6e-8).  No slow path, so it interleaves with the MFMAs it feeds.  (An fp32-only reduction measured
// 0.8 % faster in walk_kernel at 3.0e-7 max error, not adopted: tools/patches/cos_fp32.patch.)
__device__ __forceinline__ float cos_rd(float xf) {
    const double u = (double)xf * 0.15915494309189533577;
    const double f = u - __builtin_rint(u);
    return __builtin_amdgcn_cosf((float)f);
}

// sin of an fp32 argument, the same branch-free reduction (fp64, in revolutions) and the hardware v_sin_f32
__device__ __forceinline__ float sin_rd(float xf) {
    const double u = (double)xf * 0.15915494309189533577;
    const double f = u - __builtin_rint(u);
    return __builtin_amdgcn_sinf((float)f);
}

// ------------------------------------------------------------------ lookups
// nodeedge2idx[u].get(e): slice length, or -1 for None
__device__ __forceinline__ int32_t edge_len(const DevGraph &g, int32_t u, int32_t e) {
    if (e < 0 || e > g.max_eid) return -1;
    EdgeEnds x = g.ends[e];
    if (x.node_a == u) return x.len_a;
    if (x.node_b == u) return x.len_b;
    return -1;
}

__device__ __forceinline__ int32_t deg(const DevGraph &g, int32_t u) { return g.off[u + 1] - g.off[u]; }

// bisect_left over node u's f64 timestamps (utils/graph.py:511-530)
__device__ __forceinline__ int32_t bisect_ts(const DevGraph &g, int32_t u, double x) {
    int32_t s = g.off[u], lo = 0, hi = g.off[u + 1] - s;
    while (lo < hi) {
        int32_t mid = (lo + hi) >> 1;
        if (g.tsd[s + mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

}  // namespace tmk

struct tm_graph {
    int device;
    tmk::DevGraph d;
    // device allocations
    int32_t *d_off;
    int2 *d_span;
    tmk::Rec *d_rec;
    double *d_tsd;
    tmk::EdgeEnds *d_ends;
    int32_t *d_ppos;
    double *d_ets;
    tmk::PairBlk *d_pblk;
    // device-built graphs (graph_dev.hip): the sorted CSR columns and get_ts2idx values stay on the device
    // until tm_graph_export asks for them
    int32_t *d_hngh, *d_heid, *d_dict;
    int dev_built;
    // a strict_temporal view (tm_graph_strict_view) owns only d_ends; everything else is the parent's
    const tm_graph *parent;
    // host copies (export)
    int64_t *h_off;
    int32_t *h_ngh, *h_eid, *h_dict;
    double *h_ts;
};
