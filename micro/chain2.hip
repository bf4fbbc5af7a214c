// Micro-benchmark round 3: what caps a register-resident fp32 MFMA layer chain (walk_kernel's GEMM
// structure) at ~0.8 of the fp32 peak?  128 -> 128 layers with a bias + relu epilogue, weights as the A
// operand streamed per wave (buffer loads, PF fragments ahead), activations as the B operand.
//   W16   : 16x16x4, 16 columns per wave, one weight fragment (1 KB/wave) per 4 MFMAs
//   W16x2 : 16x16x4, two 16-column sets through each fragment (1 KB per 8 MFMAs)
//   W32   : 32x32x2, 32 columns per wave, one float4 of A per lane per 4 MFMAs (1 KB per 4 MFMAs of 2x work)
// weight set: 256 KB (L2-streamed), 16 KB (L1-hot) or none (weights held in registers).
// Clock: s_memtime / s_memrealtime stamps around the loop of workgroups 2048..2303 -> effective GHz.
// Usage: ./chain2  -> one line per variant: ms, TFLOP/s, in-kernel GHz
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int lane_id() {
    int l = threadIdx.x & 63;
    asm volatile("" : "+v"(l));
    return l;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wrsrc(const float4 *w) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(w), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 wload(__amdgpu_buffer_rsrc_t r, int vo, int f4) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, f4 * 16, 0));
}

constexpr int PF = 3;

// ---- 16x16x4, CS column sets (1 or 2) through each weight fragment; WM = weight-set mask in fragments
// (-1: weights from registers)
template <int CS, int WM>
__device__ __forceinline__ void layer16(const float4 *w, int layer, const floatx4 (&x)[CS][8], floatx4 (&o)[CS][8],
                                        const float4 (&wr)[8]) {
    const auto rs = wrsrc(w);
    const int vo = lane_id() * 16;
    constexpr int N = 64;
#pragma unroll
    for (int c = 0; c < CS; ++c)
#pragma unroll
        for (int t = 0; t < 8; ++t) o[c][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 buf[PF];
    auto addr = [&](int i) { return ((layer * 64 + i) & (WM < 0 ? 0 : WM)) * 64; };
    if constexpr (WM >= 0) {
#pragma unroll
        for (int i = 0; i < PF; ++i) buf[i] = wload(rs, vo, addr(i));
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int t = i / 8, q = i % 8;
        float4 wv;
        if constexpr (WM >= 0) {
            wv = buf[i % PF];
            if (i + PF < N) buf[i % PF] = wload(rs, vo, addr(i + PF));
        } else {
            wv = wr[i & 7];
        }
        if constexpr (CS == 1) {
            o[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.x, x[0][q].x, o[0][t], 0, 0, 0);
            o[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.y, x[0][q].y, o[0][t], 0, 0, 0);
            o[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.z, x[0][q].z, o[0][t], 0, 0, 0);
            o[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.w, x[0][q].w, o[0][t], 0, 0, 0);
        } else {
            o[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.x, x[0][q].x, o[0][t], 0, 0, 0);
            o[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.x, x[1][q].x, o[1][t], 0, 0, 0);
            o[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.y, x[0][q].y, o[0][t], 0, 0, 0);
            o[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.y, x[1][q].y, o[1][t], 0, 0, 0);
            o[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.z, x[0][q].z, o[0][t], 0, 0, 0);
            o[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.z, x[1][q].z, o[1][t], 0, 0, 0);
            o[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.w, x[0][q].w, o[0][t], 0, 0, 0);
            o[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.w, x[1][q].w, o[1][t], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// pair-interleaved: tiles 2u, 2u+1 alternate so consecutive MFMAs write different accumulators
template <int WM>
__device__ __forceinline__ void layer16p(const float4 *w, int layer, const floatx4 (&x)[8], floatx4 (&o)[8]) {
    const auto rs = wrsrc(w);
    const int vo = lane_id() * 16;
    constexpr int N = 64, D = 4;
#pragma unroll
    for (int t = 0; t < 8; ++t) o[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 buf[D];
    // fragment order (pair u, step q, k): tile 2u + k
    auto frag = [&](int i) { const int u = i / 16, r = i % 16, q = r / 2, k = r % 2; return (2 * u + k) * 8 + q; };
    auto addr = [&](int i) { return ((layer * 64 + frag(i)) & WM) * 64; };
#pragma unroll
    for (int i = 0; i < D; ++i) buf[i] = wload(rs, vo, addr(i));
#pragma unroll
    for (int i = 0; i < N; i += 2) {
        const int u = i / 16, q = (i % 16) / 2;
        const float4 wa = buf[i % D], wb = buf[(i + 1) % D];
        if (i + D < N) buf[i % D] = wload(rs, vo, addr(i + D));
        if (i + 1 + D < N) buf[(i + 1) % D] = wload(rs, vo, addr(i + 1 + D));
        floatx4 &a = o[2 * u], &b = o[2 * u + 1];
        a = __builtin_amdgcn_mfma_f32_16x16x4f32(wa.x, x[q].x, a, 0, 0, 0);
        b = __builtin_amdgcn_mfma_f32_16x16x4f32(wb.x, x[q].x, b, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x4f32(wa.y, x[q].y, a, 0, 0, 0);
        b = __builtin_amdgcn_mfma_f32_16x16x4f32(wb.y, x[q].y, b, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x4f32(wa.z, x[q].z, a, 0, 0, 0);
        b = __builtin_amdgcn_mfma_f32_16x16x4f32(wb.z, x[q].z, b, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x4f32(wa.w, x[q].w, a, 0, 0, 0);
        b = __builtin_amdgcn_mfma_f32_16x16x4f32(wb.w, x[q].w, b, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int WM>
__global__ void __launch_bounds__(256) k16p(const float4 *w, int iters, float *out, unsigned long long *clk) {
    extern __shared__ float bias[];
    if (threadIdx.x < 128) bias[threadIdx.x] = 0.001f * threadIdx.x;
    __syncthreads();
    floatx4 x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = floatx4{1e-3f * q, 1e-3f, 2e-3f, 3e-3f};
    const int g = (threadIdx.x & 63) >> 4;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#pragma nounroll
    for (int it = 0; it < iters; ++it) {
        floatx4 y[8];
        layer16p<WM>(w, it & 3, x, y);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const float4 b = *reinterpret_cast<const float4 *>(bias + 16 * t + 4 * g);
            x[t] = floatx4{fmaxf(y[t][0] + b.x, 0.f), fmaxf(y[t][1] + b.y, 0.f), fmaxf(y[t][2] + b.z, 0.f),
                           fmaxf(y[t][3] + b.w, 0.f)};
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += x[q][0] + x[q][1] + x[q][2] + x[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x >= 2048 && blockIdx.x < 2304) {
        clk[2 * (blockIdx.x - 2048)] = t1 - t0;
        clk[2 * (blockIdx.x - 2048) + 1] = r1 - r0;
    }
}

template <int CS, int WM>
__global__ void __launch_bounds__(256) k16(const float4 *w, int iters, float *out, unsigned long long *clk) {
    extern __shared__ float bias[];
    if (threadIdx.x < 128) bias[threadIdx.x] = 0.001f * threadIdx.x;
    __syncthreads();
    floatx4 x[CS][8];
#pragma unroll
    for (int c = 0; c < CS; ++c)
#pragma unroll
        for (int q = 0; q < 8; ++q) x[c][q] = floatx4{1e-3f * q, 1e-3f * c, 2e-3f, 3e-3f};
    float4 wr[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) wr[i] = w[i * 64 + (threadIdx.x & 63)];
    const int g = (threadIdx.x & 63) >> 4;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#pragma nounroll
    for (int it = 0; it < iters; ++it) {
        floatx4 y[CS][8];
        layer16<CS, WM>(w, it & 3, x, y, wr);
#pragma unroll
        for (int c = 0; c < CS; ++c)
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const float4 b = *reinterpret_cast<const float4 *>(bias + 16 * t + 4 * g);
                x[c][t] = floatx4{fmaxf(y[c][t][0] + b.x, 0.f), fmaxf(y[c][t][1] + b.y, 0.f),
                                  fmaxf(y[c][t][2] + b.z, 0.f), fmaxf(y[c][t][3] + b.w, 0.f)};
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CS; ++c)
#pragma unroll
        for (int q = 0; q < 8; ++q) s += x[c][q][0] + x[c][q][1] + x[c][q][2] + x[c][q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x >= 2048 && blockIdx.x < 2304) {
        clk[2 * (blockIdx.x - 2048)] = t1 - t0;
        clk[2 * (blockIdx.x - 2048) + 1] = r1 - r0;
    }
}

// ---- 32x32x2: 4 output tiles of 32 features; K step s (of 64) = register s%16 of x tile s/16
// weight pack: [layer][t][s/4][lane] float4 (A operand of 4 consecutive K steps)
template <int WM>
__device__ __forceinline__ void layer32(const float4 *w, int layer, const floatx16 (&x)[4], floatx16 (&o)[4]) {
    const auto rs = wrsrc(w);
    const int vo = lane_id() * 16;
    constexpr int N = 64;   // 4 tiles x 16 float4 loads
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float4 buf[PF];
    auto addr = [&](int i) { return ((layer * 64 + i) & WM) * 64; };
#pragma unroll
    for (int i = 0; i < PF; ++i) buf[i] = wload(rs, vo, addr(i));
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int t = i / 16, s4 = i % 16;
        const float4 wv = buf[i % PF];
        if (i + PF < N) buf[i % PF] = wload(rs, vo, addr(i + PF));
        const int q = s4 * 4;
        o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, x[q / 16][q % 16], o[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, x[q / 16][q % 16 + 1], o[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, x[q / 16][q % 16 + 2], o[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, x[q / 16][q % 16 + 3], o[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int WM>
__global__ void __launch_bounds__(256) k32(const float4 *w, int iters, float *out, unsigned long long *clk) {
    extern __shared__ float bias[];
    if (threadIdx.x < 128) bias[threadIdx.x] = 0.001f * threadIdx.x;
    __syncthreads();
    floatx16 x[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) x[t][r] = 1e-3f * (r + t);
    const int h = (threadIdx.x & 63) >> 5;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#pragma nounroll
    for (int it = 0; it < iters; ++it) {
        floatx16 y[4];
        layer32<WM>(w, it & 3, x, y);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const float4 b = *reinterpret_cast<const float4 *>(bias + 32 * t + 8 * r4 + 4 * h);
                x[t][4 * r4 + 0] = fmaxf(y[t][4 * r4 + 0] + b.x, 0.f);
                x[t][4 * r4 + 1] = fmaxf(y[t][4 * r4 + 1] + b.y, 0.f);
                x[t][4 * r4 + 2] = fmaxf(y[t][4 * r4 + 2] + b.z, 0.f);
                x[t][4 * r4 + 3] = fmaxf(y[t][4 * r4 + 3] + b.w, 0.f);
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += x[t][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x >= 2048 && blockIdx.x < 2304) {
        clk[2 * (blockIdx.x - 2048)] = t1 - t0;
        clk[2 * (blockIdx.x - 2048) + 1] = r1 - r0;
    }
}

template <typename K>
static void run(const char *name, K kern, double flop_per_wave_iter, const float4 *w, float *out,
                unsigned long long *clk, int blocks, int iters, int lds) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int r = 0; r < 3; ++r) kern<<<blocks, 256, lds>>>(w, iters, out, clk);   // warm the clock
    hipDeviceSynchronize();
    hipEventRecord(a);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) kern<<<blocks, 256, lds>>>(w, iters, out, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    std::vector<unsigned long long> h(512);
    hipMemcpy(h.data(), clk, 512 * 8, hipMemcpyDeviceToHost);
    std::vector<double> ghz;
    for (int i = 0; i < 256; ++i)
        if (h[2 * i + 1]) ghz.push_back((double)h[2 * i] / h[2 * i + 1] * 0.1);
    std::sort(ghz.begin(), ghz.end());
    const double flop = flop_per_wave_iter * iters * blocks * 4.0;
    const int wps = (160 * 1024) / lds;   // workgroups per CU by LDS = waves per SIMD (if registers allow)
    printf("%-34s waves/SIMD=%d  %.3f ms  %6.1f TFLOP/s  (%.3f of 157.3)  clk %.2f GHz\n", name, wps, ms,
           flop / ms / 1e9, flop / ms / 1e9 / 157.3, ghz.empty() ? 0.0 : ghz[ghz.size() / 2]);
}

int main() {
    float4 *w;
    float *out;
    unsigned long long *clk;
    const int nw = 4 * 64 * 64;   // 4 layers x 64 fragments x 64 lanes = 256 KB
    hipMalloc(&w, sizeof(float4) * nw);
    std::vector<float4> h(nw);
    for (int i = 0; i < nw; ++i) h[i] = float4{1e-3f * (i % 7), -1e-3f * (i % 3), 2e-3f, 1e-4f * (i % 5)};
    hipMemcpy(w, h.data(), sizeof(float4) * nw, hipMemcpyHostToDevice);
    const int blocks = 256 * 2 * 16;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    hipMalloc(&clk, 512 * 8);
    const int iters = 200;
    const double f16 = 2.0 * 128 * 128 * 16, f32 = 2.0 * 128 * 128 * 32;
    const int L1W = 96 * 1024, L2W = 64 * 1024, L4W = 40 * 1024;   // dynamic LDS -> 1 / 2 / 4 waves per SIMD
    for (int rep = 0; rep < 2; ++rep) {
        run("W16 t-major streamed", k16<1, 255>, f16, w, out, clk, blocks, iters, L2W);
        run("W16 t-major streamed", k16<1, 255>, f16, w, out, clk, blocks, iters, L1W);
        run("W16 pairs streamed", k16p<255>, f16, w, out, clk, blocks, iters, L2W);
        run("W16 pairs streamed", k16p<255>, f16, w, out, clk, blocks, iters, L1W);
        run("W16x2 streamed", k16<2, 255>, 2 * f16, w, out, clk, blocks, iters, L1W);
        run("W32 streamed", k32<255>, f32, w, out, clk, blocks, iters, L1W);
    }
    return 0;
}
