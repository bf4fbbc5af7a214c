// Accuracy + cost of cos(x) evaluations for the time encoder's fp32 arguments x = fp32(fp32(dt*w) + phi):
//   rd : tempme's cos_rd (fp64 reduction by pi, even Taylor polynomial to r^12)
//   hw : v_cos_f32 on the fraction of x / (2 pi) computed in fp64 (__builtin_amdgcn_cosf takes revolutions)
// Max |err| vs fp64 cos over dt in [0, 1e8] (integers), every encoder frequency w_k = 10^(-9k/171), phi in
// [-1, 1]; then VALU cost per evaluation in a loop.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ float cos_rd(float xf) {
    const double x = (double)xf;
    const double t = __builtin_fma(x, 0.31830988618379067154, 6755399441055744.0);
    const double j = t - 6755399441055744.0;
    double r = __builtin_fma(-j, 3.141592653589793116, x);
    r = __builtin_fma(-j, 1.2246467991473532e-16, r);
    const float rf = (float)r, z = rf * rf;
    float c = 2.08767569878681e-09f;
    c = __builtin_fmaf(c, z, -2.755731922398589e-07f);
    c = __builtin_fmaf(c, z, 2.48015873015873e-05f);
    c = __builtin_fmaf(c, z, -1.388888888888889e-03f);
    c = __builtin_fmaf(c, z, 4.166666666666666e-02f);
    c = __builtin_fmaf(c, z, -0.5f);
    c = __builtin_fmaf(c, z, 1.0f);
    const uint32_t odd = (uint32_t)__double2loint(t) << 31;
    return __uint_as_float(__float_as_uint(c) ^ odd);
}

__device__ __forceinline__ float cos_hw(float xf) {
    const double u = (double)xf * 0.15915494309189533577;   // x / (2 pi), rel err 2^-53
    const double f = u - __builtin_rint(u);                   // in [-1/2, 1/2]
    return __builtin_amdgcn_cosf((float)f);
}

__global__ void acc_kernel(const float *x, int n, float *e_rd, float *e_hw, const double *ref) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    e_rd[i] = (float)fabs((double)cos_rd(x[i]) - ref[i]);
    e_hw[i] = (float)fabs((double)cos_hw(x[i]) - ref[i]);
}

template <int M>
__global__ void cost_kernel(const float *x, int iters, float *out) {
    float a = x[threadIdx.x], s = 0.f;
    for (int it = 0; it < iters; ++it) {
        float v = M == 0 ? cos_rd(a) : cos_hw(a);
        s += v;
        a = a * 1.0001f + 0.5f;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    std::vector<float> hx;
    std::vector<double> hr;
    uint64_t st = 12345;
    auto rnd = [&]() { st = st * 6364136223846793005ull + 1442695040888963407ull; return (st >> 11) * (1.0 / 9007199254740992.0); };
    for (int k = 0; k < 172; ++k) {
        const float w = (float)(1.0 / pow(10.0, 9.0 * k / 171.0));
        for (int s = 0; s < 20000; ++s) {
            const float dt = (float)(uint32_t)(rnd() * 1e8);
            const float ph = (float)(rnd() * 2 - 1) * (s & 1);
            const float x = __builtin_fmaf(0, 0, (float)(dt * w)) + ph;   // fp32 product, then + phi in fp32
            hx.push_back(x);
            hr.push_back(cos((double)x));
        }
    }
    const int n = (int)hx.size();
    float *x, *e1, *e2;
    double *r;
    (void)hipMalloc(&x, n * 4); (void)hipMalloc(&e1, n * 4); (void)hipMalloc(&e2, n * 4); (void)hipMalloc(&r, n * 8);
    (void)hipMemcpy(x, hx.data(), n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(r, hr.data(), n * 8, hipMemcpyHostToDevice);
    acc_kernel<<<(n + 255) / 256, 256>>>(x, n, e1, e2, r);
    std::vector<float> a(n), b(n);
    (void)hipMemcpy(a.data(), e1, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(b.data(), e2, n * 4, hipMemcpyDeviceToHost);
    double ma = 0, mb = 0, sa = 0, sb = 0;
    int worst_k = 0;
    for (int i = 0; i < n; ++i) {
        if (a[i] > ma) ma = a[i];
        if (b[i] > mb) { mb = b[i]; worst_k = i / 20000; }
        sa += a[i]; sb += b[i];
    }
    printf("samples %d: cos_rd max %.3g mean %.3g | cos_hw max %.3g (k=%d) mean %.3g\n", n, ma, sa / n, mb, worst_k, sb / n);
    // per-k max for hw
    for (int k = 0; k < 172; k += 19) {
        double m = 0;
        for (int i = k * 20000; i < (k + 1) * 20000; ++i) m = fmax(m, (double)b[i]);
        printf("  k=%3d hw max %.3g\n", k, m);
    }
    float *out;
    (void)hipMalloc(&out, 4 * 1024 * 256);
    hipEvent_t t0, t1;
    (void)hipEventCreate(&t0); (void)hipEventCreate(&t1);
    for (int m = 0; m < 2; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(t0);
            if (m == 0) cost_kernel<0><<<1024 * 8, 256>>>(x, 2000, out);
            else cost_kernel<1><<<1024 * 8, 256>>>(x, 2000, out);
            (void)hipEventRecord(t1);
            (void)hipEventSynchronize(t1);
            float ms;
            (void)hipEventElapsedTime(&ms, t0, t1);
            const double evals_per_simd = 1024.0 * 8 * 256 / 64 * 2000 / 1024;   // wave-evals per SIMD
            if (rep) printf("%s: %.3f ms, %.1f cycles per wave-eval per SIMD\n", m ? "cos_hw" : "cos_rd", ms, ms * 1e-3 * 2.4e9 / evals_per_simd);
        }
    }
    return 0;
}
