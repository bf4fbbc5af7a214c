// Micro-benchmark: fp32-accurate layer chains on bf16 MFMA (each operand split into three bf16
// parts, the six products down to 2^-16 relative, fp32 accumulate) vs plain f32 MFMA.
// 16 activation columns per wave, 128 -> 128 layers, weights as the A operand.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short shortx8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int lane_id() {
    int l = threadIdx.x & 63;
    asm volatile("" : "+v"(l));
    return l;
}

struct Split3 { bf16x8 h, m, l; };

// 8 fp32 -> hi/mid/lo bf16 parts
__device__ __forceinline__ Split3 split8(const float (&v)[8]) {
    Split3 s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 h = (__bf16)v[j];
        const float r = v[j] - (float)h;
        const __bf16 m = (__bf16)r;
        const float r2 = r - (float)m;
        s.h[j] = h;
        s.m[j] = m;
        s.l[j] = (__bf16)r2;
    }
    return s;
}

#define MF(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0)

// y (8 tiles) = W (128x128, packed [t][kk][part][lane] bf16x8) * x (8 tiles)
template <int SPLITS>
__device__ __forceinline__ void layer_split(const bf16x8 *w, const floatx4 (&x)[8], floatx4 (&y)[8]) {
    Split3 xs[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const float v[8] = {x[2 * kk][0], x[2 * kk][1], x[2 * kk][2], x[2 * kk][3],
                            x[2 * kk + 1][0], x[2 * kk + 1][1], x[2 * kk + 1][2], x[2 * kk + 1][3]};
        xs[kk] = split8(v);
    }
    const bf16x8 *wp = w + lane_id();
    constexpr int N = 32, D = 2;   // (t, kk) steps, prefetch depth
    bf16x8 bh[D], bm[D], bl[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        bh[i] = wp[(i * 3 + 0) * 64];
        bm[i] = wp[(i * 3 + 1) * 64];
        bl[i] = wp[(i * 3 + 2) * 64];
    }
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int t = i / 4, kk = i % 4;
        const bf16x8 ah = bh[i % D], am = bm[i % D], al = bl[i % D];
        if (i + D < N) {
            bh[i % D] = wp[((i + D) * 3 + 0) * 64];
            bm[i % D] = wp[((i + D) * 3 + 1) * 64];
            bl[i % D] = wp[((i + D) * 3 + 2) * 64];
        }
        if (kk == 0) acc = floatx4{0.f, 0.f, 0.f, 0.f};
        acc = MF(ah, xs[kk].h, acc);
        acc = MF(ah, xs[kk].m, acc);
        acc = MF(am, xs[kk].h, acc);
        if (SPLITS == 6) {
            acc = MF(ah, xs[kk].l, acc);
            acc = MF(al, xs[kk].h, acc);
            acc = MF(am, xs[kk].m, acc);
        }
        if (kk == 3) y[t] = acc;
        __builtin_amdgcn_sched_barrier(0);
    }
}


// 6 products, output tiles processed in pairs with interleaved accumulators
__device__ __forceinline__ void layer_split_pair(const bf16x8 *w, const floatx4 (&x)[8], floatx4 (&y)[8]) {
    Split3 xs[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const float v[8] = {x[2 * kk][0], x[2 * kk][1], x[2 * kk][2], x[2 * kk][3],
                            x[2 * kk + 1][0], x[2 * kk + 1][1], x[2 * kk + 1][2], x[2 * kk + 1][3]};
        xs[kk] = split8(v);
    }
    const bf16x8 *wp = w + lane_id();
#pragma unroll
    for (int tp = 0; tp < 4; ++tp) {
        floatx4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int f0 = (2 * tp) * 4 + kk, f1 = (2 * tp + 1) * 4 + kk;
            const bf16x8 h0 = wp[(f0 * 3 + 0) * 64], m0 = wp[(f0 * 3 + 1) * 64], l0 = wp[(f0 * 3 + 2) * 64];
            const bf16x8 h1 = wp[(f1 * 3 + 0) * 64], m1 = wp[(f1 * 3 + 1) * 64], l1 = wp[(f1 * 3 + 2) * 64];
            a0 = MF(h0, xs[kk].h, a0); a1 = MF(h1, xs[kk].h, a1);
            a0 = MF(h0, xs[kk].m, a0); a1 = MF(h1, xs[kk].m, a1);
            a0 = MF(m0, xs[kk].h, a0); a1 = MF(m1, xs[kk].h, a1);
            a0 = MF(h0, xs[kk].l, a0); a1 = MF(h1, xs[kk].l, a1);
            a0 = MF(l0, xs[kk].h, a0); a1 = MF(l1, xs[kk].h, a1);
            a0 = MF(m0, xs[kk].m, a0); a1 = MF(m1, xs[kk].m, a1);
        }
        y[2 * tp] = a0;
        y[2 * tp + 1] = a1;
    }
}

__device__ __forceinline__ void layer_f32(const float4 *w, const floatx4 (&x)[8], floatx4 (&y)[8]) {
    const float4 *wp = w + lane_id();
    constexpr int N = 64, D = 3;
    float4 buf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) buf[i] = wp[i * 64];
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int t = i / 8, q = i % 8;
        const float4 wv = buf[i % D];
        if (i + D < N) buf[i % D] = wp[(i + D) * 64];
        if (q == 0) acc = floatx4{0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.x, x[q].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.y, x[q].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.z, x[q].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.w, x[q].w, acc, 0, 0, 0);
        if (q == 7) y[t] = acc;
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int MODE>   // 0: f32, 3: bf16 x3 (3 products), 6: bf16 x3 (6 products)
__global__ void __launch_bounds__(256, 2) chain(const void *w, int iters, float *out) {
    extern __shared__ float lds_pad[];
    if (threadIdx.x == 0) lds_pad[0] = 0.f;
    floatx4 x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = floatx4{1e-3f * q, 1e-3f, 2e-3f, 3e-3f};
#pragma nounroll
    for (int it = 0; it < iters; ++it) {
        floatx4 y[8];
        if (MODE == 0) layer_f32(reinterpret_cast<const float4 *>(w) + (it & 3) * 64 * 64, x, y);
        else if (MODE == 7) layer_split_pair(reinterpret_cast<const bf16x8 *>(w) + (it & 3) * 8 * 4 * 3 * 64, x, y);
        else layer_split<MODE>(reinterpret_cast<const bf16x8 *>(w) + (it & 3) * 8 * 4 * 3 * 64, x, y);
#pragma unroll
        for (int t = 0; t < 8; ++t)
            x[t] = floatx4{fmaxf(y[t][0], 0.f) + 1e-3f, fmaxf(y[t][1], 0.f), fmaxf(y[t][2], 0.f), fmaxf(y[t][3], 0.f)};
    }
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += x[q][0] + x[q][1] + x[q][2] + x[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
static void run(const char *name, const void *w, float *out, int blocks, int iters, int lds) {
    hipFuncSetAttribute((const void *)chain<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    chain<MODE><<<blocks, 256, lds>>>(w, iters, out);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) chain<MODE><<<blocks, 256, lds>>>(w, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double flop = 2.0 * 128 * 128 * 16 * (double)iters * blocks * 4;   // fp32-equivalent
    printf("%-18s lds=%6d  %.3f ms  %.1f TFLOP/s (fp32-equivalent)\n", name, lds, ms, flop / ms / 1e9);
}

int main() {
    void *w;
    const size_t bytes = 4 * 8 * 4 * 3 * 64 * 16;   // 4 layers, bf16x3 packing (largest)
    hipMalloc(&w, bytes);
    std::vector<unsigned short> h(bytes / 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3a80 + (i % 13);   // small bf16 / f32 halves
    hipMemcpy(w, h.data(), bytes, hipMemcpyHostToDevice);
    float *out;
    const int blocks = 256 * 2 * 8;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    for (int lds : {64 * 1024, 100 * 1024}) {
        run<0>("f32 16x16x4", w, out, blocks, 200, lds);
        run<6>("bf16x3 6-prod", w, out, blocks, 200, lds);
        run<3>("bf16x3 3-prod", w, out, blocks, 200, lds);
        run<7>("bf16x3 6-prod pair", w, out, blocks, 200, lds);
    }
    return 0;
}
