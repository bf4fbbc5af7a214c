// Micro-benchmark: how much independent VALU work hides beside fp32 MFMAs (v_mfma_f32_16x16x4_f32)?
// 128 -> 128 layer chain (16 columns, weights streamed from a 16 KB L1-hot set), NV fp32 FMAs (or NV fp64 FMAs)
// on independent registers issued after every tile's 4 MFMAs.  2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));

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

template <int NV, bool F64>
__global__ void __launch_bounds__(256) kv(const float4 *w, int iters, float *out) {
    extern __shared__ float bias[];
    floatx4 x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = floatx4{1e-3f * q, 1e-3f, 2e-3f, 3e-3f};
    float a[8];
    double d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = 1e-3f * j + threadIdx.x; d[j] = a[j]; }
    const auto rs = wrsrc(w);
    const int vo = lane_id() * 16;
#pragma nounroll
    for (int it = 0; it < iters; ++it) {
        floatx4 o[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) o[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        float4 buf[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) buf[i] = wload(rs, vo, (i & 15) * 64);
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            const int t = i / 8, q = i % 8;
            const float4 wv = buf[i % 3];
            if (i + 3 < 64) buf[i % 3] = wload(rs, vo, ((i + 3) & 15) * 64);
            o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.x, x[q].x, o[t], 0, 0, 0);
            o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.y, x[q].y, o[t], 0, 0, 0);
            o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.z, x[q].z, o[t], 0, 0, 0);
            o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.w, x[q].w, o[t], 0, 0, 0);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                if (F64) d[v & 7] = __builtin_fma(d[v & 7], 0.999, 1e-3);
                else a[v & 7] = __builtin_fmaf(a[v & 7], 0.999f, 1e-3f);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) x[t] = floatx4{fmaxf(o[t][0], 0.f), fmaxf(o[t][1], 0.f), fmaxf(o[t][2], 0.f), fmaxf(o[t][3], 0.f)};
    }
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += x[q][0] + x[q][1] + x[q][2] + x[q][3];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + (float)d[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char *name, K kern, const float4 *w, float *out, int blocks, int iters, int lds) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int r = 0; r < 3; ++r) kern<<<blocks, 256, lds>>>(w, iters, out);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < 10; ++r) kern<<<blocks, 256, lds>>>(w, iters, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= 10;
    // per SIMD: blocks*4 waves / 1024 SIMDs, each wave iters*256 MFMAs
    const double mf = (double)blocks * 4 * iters * 256 / 1024.0;
    const double cyc = ms * 1e-3 * 2.4e9;
    printf("%-22s %.3f ms  %.1f cycles per MFMA per SIMD  (32 = peak)\n", name, ms, cyc / mf);
}

int main() {
    float4 *w;
    float *out;
    (void)hipMalloc(&w, sizeof(float4) * 64 * 64);
    std::vector<float4> h(64 * 64, float4{1e-3f, -1e-3f, 2e-3f, 1e-4f});
    (void)hipMemcpy(w, h.data(), sizeof(float4) * 64 * 64, hipMemcpyHostToDevice);
    const int blocks = 256 * 2 * 16, iters = 100;
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    const int L2W = 64 * 1024;
    for (int rep = 0; rep < 2; ++rep) {
        run("f32 valu/tile=0", kv<0, false>, w, out, blocks, iters, L2W);
        run("f32 valu/tile=4", kv<4, false>, w, out, blocks, iters, L2W);
        run("f32 valu/tile=8", kv<8, false>, w, out, blocks, iters, L2W);
        run("f32 valu/tile=16", kv<16, false>, w, out, blocks, iters, L2W);
        run("f32 valu/tile=32", kv<32, false>, w, out, blocks, iters, L2W);
        run("f64 valu/tile=4", kv<4, true>, w, out, blocks, iters, L2W);
        run("f64 valu/tile=8", kv<8, true>, w, out, blocks, iters, L2W);
        run("f64 valu/tile=16", kv<16, true>, w, out, blocks, iters, L2W);
    }
    return 0;
}
