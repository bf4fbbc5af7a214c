// Micro-benchmark: register-resident MFMA layer chains (16x16x4 f32, weights as the A operand,
// 16 activation columns per wave) -- the structure of walk_kernel's GEMMs without its gathers.
// Usage: ./chain  -> one line per variant: ms, TFLOP/s
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int lane_id() {
    int l = threadIdx.x & 63;
    asm volatile("" : "+v"(l));
    return l;
}

// MODE 0: t-major (dependent chain per tile), MODE 1: pair-interleaved tiles, MODE 2/4: groups of 2/4
// tiles whose MFMAs alternate accumulators (consecutive MFMAs independent)
template <int NTO, int NQ, int D, int GS>
__device__ __forceinline__ void rgemm_alt(const float4 *w, const floatx4 (&x)[NQ], floatx4 (&o)[NTO]) {
    const float4 *wp = w + lane_id();
    constexpr int N = NTO * NQ;
#pragma unroll
    for (int t = 0; t < NTO; ++t) o[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 buf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) buf[i] = wp[i * 64];
    // fragment order: (group pr, step q, k): tile GS*pr + k
#pragma unroll
    for (int i0 = 0; i0 < N; i0 += GS) {
        float4 wv[GS];
#pragma unroll
        for (int k = 0; k < GS; ++k) {
            const int i = i0 + k;
            wv[k] = buf[i % D];
            if (i + D < N) buf[i % D] = wp[(i + D) * 64];
        }
        const int pr = i0 / (GS * NQ), q = (i0 % (GS * NQ)) / GS;
#pragma unroll
        for (int k = 0; k < GS; ++k) o[GS * pr + k] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[k].x, x[q].x, o[GS * pr + k], 0, 0, 0);
#pragma unroll
        for (int k = 0; k < GS; ++k) o[GS * pr + k] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[k].y, x[q].y, o[GS * pr + k], 0, 0, 0);
#pragma unroll
        for (int k = 0; k < GS; ++k) o[GS * pr + k] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[k].z, x[q].z, o[GS * pr + k], 0, 0, 0);
#pragma unroll
        for (int k = 0; k < GS; ++k) o[GS * pr + k] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[k].w, x[q].w, o[GS * pr + k], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int NTO, int NQ, int D, int MODE>
__device__ __forceinline__ void rgemm(const float4 *w, const floatx4 (&x)[NQ], floatx4 (&o)[NTO]) {
    if constexpr (MODE >= 2) {
        rgemm_alt<NTO, NQ, D, MODE>(w, x, o);
        return;
    }
    const float4 *wp = w + lane_id();
    constexpr int N = NTO * NQ;
#pragma unroll
    for (int t = 0; t < NTO; ++t) o[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 buf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) buf[i] = wp[i * 64];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        int t, q;
        if (MODE == 0) { t = i / NQ; q = i % NQ; }
        else { const int pr = i / (2 * NQ), r = i % (2 * NQ); t = 2 * pr + (r & 1); q = r >> 1; if (t >= NTO) { t = NTO - 1; } }
        const float4 wv = buf[i % D];
        if (i + D < N) buf[i % D] = wp[(i + D) * 64];
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.x, x[q].x, o[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.y, x[q].y, o[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.z, x[q].z, o[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.w, x[q].w, o[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// EPI 0: none (just pass D through), 1: bias (LDS) + relu
template <int D, int MODE, int EPI, int U = 1>
__global__ void __launch_bounds__(256, 2) chain_kernel(const float4 *w, int iters, float *out) {
    extern __shared__ float bias[];   // dynamic size sets blocks per CU (occupancy)
    if (threadIdx.x < 128) bias[threadIdx.x] = 0.001f * threadIdx.x;
    __syncthreads();
    floatx4 x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = floatx4{1e-3f * q, 1e-3f, 2e-3f, 3e-3f};
    const int g = threadIdx.x & 63 >> 4;
#pragma nounroll
    for (int it = 0; it < iters; it += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        floatx4 y[8];
        rgemm<8, 8, D, MODE>(w + ((it + u) & 3) * 64 * 64, x, y);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (EPI == 2 && t == 0) {
                // VALU block: 4 independent chains x 64 dependent FMAs (256 VALU) per layer
                float a0 = y[0][0], a1 = y[0][1], a2 = y[0][2], a3 = y[0][3];
#pragma unroll
                for (int r = 0; r < 64; ++r) {
                    a0 = __builtin_fmaf(a0, 0.999f, 1e-3f); a1 = __builtin_fmaf(a1, 0.999f, 1e-3f);
                    a2 = __builtin_fmaf(a2, 0.999f, 1e-3f); a3 = __builtin_fmaf(a3, 0.999f, 1e-3f);
                }
                x[0] = floatx4{a0, a1, a2, a3};
            } else if (EPI) {
                const float4 b = *reinterpret_cast<const float4 *>(bias + 16 * t + 4 * g);
                x[t] = floatx4{fmaxf(y[t][0] + b.x, 0.f), fmaxf(y[t][1] + b.y, 0.f), fmaxf(y[t][2] + b.z, 0.f),
                               fmaxf(y[t][3] + b.w, 0.f)};
            } else {
                x[t] = y[t];
            }
        }
    }
    }
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += x[q][0] + x[q][1] + x[q][2] + x[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int D, int MODE, int EPI, int U = 1>
static void run(const char *name, const float4 *w, float *out, int blocks, int iters, int lds = 64 * 1024) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipFuncSetAttribute((const void *)chain_kernel<D, MODE, EPI, U>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    chain_kernel<D, MODE, EPI, U><<<blocks, 256, lds>>>(w, iters, out);
    hipDeviceSynchronize();
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) chain_kernel<D, MODE, EPI, U><<<blocks, 256, lds>>>(w, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double flop = 2.0 * 16 * 16 * 4 * 4 * 64 * (double)iters * blocks * 4;   // 64 frags x 4 MFMA per layer
    printf("%-28s lds=%6d blocks=%d iters=%d  %.3f ms  %.1f TFLOP/s\n", name, lds, blocks, iters, ms, flop / ms / 1e9);
}

int main() {
    float4 *w;
    float *out;
    const int nw = 4 * 64 * 64;   // 4 layers of 64 fragments x 64 lanes
    hipMalloc(&w, sizeof(float4) * nw);
    std::vector<float4> h(nw);
    for (int i = 0; i < nw; ++i) h[i] = float4{1e-3f * (i % 7), -1e-3f, 2e-3f, 1e-4f};
    hipMemcpy(w, h.data(), sizeof(float4) * nw, hipMemcpyHostToDevice);
    const int blocks = 256 * 2 * 8;   // 8 rounds of 2 blocks per CU
    hipMalloc(&out, sizeof(float) * blocks * 256);
    const int iters = 200;
    run<3, 0, 0>("D3 tmajor noepi", w, out, blocks, iters);
    run<3, 0, 1>("D3 tmajor epi", w, out, blocks, iters);
    run<3, 1, 1>("D3 pairs epi", w, out, blocks, iters);
    run<6, 0, 1>("D6 tmajor epi", w, out, blocks, iters);
    run<1, 0, 1>("D1 tmajor epi", w, out, blocks, iters);
    run<3, 0, 2>("D3 tmajor valu256 2w", w, out, blocks, iters);
    run<3, 0, 2>("D3 tmajor valu256 1w", w, out, blocks, iters, 100 * 1024);
    run<3, 0, 2>("D3 tmajor valu256 4w", w, out, blocks, iters, 32 * 1024);
    run<3, 1, 2>("D3 pairs valu256 2w", w, out, blocks, iters);
    run<4, 2, 1>("D4 alt2 epi", w, out, blocks, iters);
    run<6, 2, 1>("D6 alt2 epi", w, out, blocks, iters);
    run<4, 4, 1>("D4 alt4 epi", w, out, blocks, iters);
    run<8, 4, 1>("D8 alt4 epi", w, out, blocks, iters);
    run<4, 2, 1>("D4 alt2 epi 1 wave/SIMD", w, out, blocks, iters, 100 * 1024);
    run<4, 2, 2>("D4 alt2 valu256 2w", w, out, blocks, iters);
    run<4, 2, 2>("D4 alt2 valu256 1w", w, out, blocks, iters, 100 * 1024);
    run<3, 0, 1>("D3 tmajor epi 1 wave/SIMD", w, out, blocks, iters, 100 * 1024);
    run<3, 0, 1>("D3 tmajor epi 4 waves/SIMD", w, out, blocks, iters, 32 * 1024);
    run<3, 1, 1>("D3 pairs epi 4 waves/SIMD", w, out, blocks, iters, 32 * 1024);
    return 0;
}
