// The explainer's optimizer step (temp_exp_main.py:631-632, torch.optim.Adam(lr, betas, eps, weight_decay)) as ONE
// kernel over a flat fp32 bucket: every parameter of the explainer lives in one contiguous buffer, its gradient in
// another (tempme_amd/optim.py FusedAdam keeps the module's parameters and .grad as views of them), so the
// data-parallel gradient all-reduce (train.GradAllReduce) runs on the same bucket with no packing copies and the
// update is one grid-stride pass: m, v, bias corrections, the step.
//
// Per element, in torch.optim.Adam's single-tensor order (torch/optim/adam.py _single_tensor_adam, amsgrad off):
//   g = grad * grad_scale (+ weight_decay * p)
//   m = lerp(m, g, 1 - beta1)            v = v * beta2 + (1 - beta2) * g * g
//   p = p - step_size * m / (sqrt(v) / sqrt(bc2) + eps),  step_size = lr / bc1,  bc_i = 1 - beta_i^t
// The step count t lives on the device (capturable: a HIP-graph replay advances it): every workgroup reads the
// count before the step; the last workgroup to finish (a completion counter, reset by that workgroup) writes t.
#include <cmath>

#include "common.h"

namespace tmk {

struct AdamArgs {
    float *p;
    const float *g;
    float *m, *v;
    int64_t n;
    float lr, beta1, beta2, eps, weight_decay, grad_scale;
    float *step;          // device: the step count before this step (torch's state["step"])
    uint32_t *done;       // device: completion counter, 0 between launches
    int64_t head;         // elements before the first 16-byte-aligned one (the four buffers share the offset)
    int advance;          // this launch advances the step count (the last of a step's launches)
};

__device__ __forceinline__ void adam_elem(float &p, float g, float &m, float &v, const AdamArgs &a, float step_size,
                                          float bc2_sqrt) {
    g *= a.grad_scale;
    if (a.weight_decay != 0.f) g = __builtin_fmaf(a.weight_decay, p, g);
    m = m + (1.f - a.beta1) * (g - m);                    // torch.lerp with weight < 0.5
    v = __builtin_fmaf((1.f - a.beta2) * g, g, v * a.beta2);
    const float denom = sqrtf(v) / bc2_sqrt + a.eps;
    p = p + (-step_size) * (m / denom);
}

__global__ void __launch_bounds__(256) adam_kernel(AdamArgs a) {
    const double t = (double)(*a.step) + 1.0;
    const double bc1 = 1.0 - pow((double)a.beta1, t), bc2 = 1.0 - pow((double)a.beta2, t);
    const float step_size = (float)((double)a.lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    const int64_t h = a.head, n4 = (a.n - h) >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float4 *p4 = reinterpret_cast<float4 *>(a.p + h);
    float4 *m4 = reinterpret_cast<float4 *>(a.m + h);
    float4 *v4 = reinterpret_cast<float4 *>(a.v + h);
    const float4 *g4 = reinterpret_cast<const float4 *>(a.g + h);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 p = p4[i], m = m4[i], v = v4[i];
        const float4 g = g4[i];
        adam_elem(p.x, g.x, m.x, v.x, a, step_size, bc2_sqrt);
        adam_elem(p.y, g.y, m.y, v.y, a, step_size, bc2_sqrt);
        adam_elem(p.z, g.z, m.z, v.z, a, step_size, bc2_sqrt);
        adam_elem(p.w, g.w, m.w, v.w, a, step_size, bc2_sqrt);
        p4[i] = p;
        m4[i] = m;
        v4[i] = v;
    }
    // the unaligned head and the tail after the last float4 (at most 3 + 3 elements)
    const int64_t tail = (a.n - h) & 3;
    if (blockIdx.x == 0 && threadIdx.x < h + tail) {
        const int64_t i = threadIdx.x < h ? (int64_t)threadIdx.x : h + (n4 << 2) + (threadIdx.x - h);
        float p = a.p[i], m = a.m[i], v = a.v[i];
        adam_elem(p, a.g[i], m, v, a, step_size, bc2_sqrt);
        a.p[i] = p;
        a.m[i] = m;
        a.v[i] = v;
    }
    // the last workgroup advances the step count (every workgroup has read it by then) and resets the counter
    if (!a.advance) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(a.done, 1u) == gridDim.x - 1) {
            *a.step = (float)t;
            *a.done = 0u;
            __threadfence();
        }
    }
}

constexpr int kMaxCopyJobs = 32;

struct CopyArgs {
    tm_copy_job job[kMaxCopyJobs];
};

// blockIdx.y = job: dst[0:n) = src[0:n), grid-strided over blockIdx.x
__global__ void __launch_bounds__(256) copy_many_kernel(CopyArgs a) {
    const tm_copy_job &j = a.job[blockIdx.y];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < j.n; i += (int64_t)gridDim.x * blockDim.x)
        j.dst[i] = j.src[i];
}

}  // namespace tmk

using namespace tmk;

// The parameters' gradients into the flat bucket (FusedAdam.sync_grads: autograd's own gradient tensors, one launch
// per 32 parameters instead of an accumulation kernel per parameter per step)
extern "C" int tm_copy_many(const tm_copy_job *jobs, int32_t n_jobs, void *stream) {
    if (n_jobs < 0 || n_jobs > kMaxCopyJobs) return fail(TM_E_ARG, "tm_copy_many: bad job count");
    if (n_jobs == 0) return TM_OK;
    if (!jobs) return fail(TM_E_ARG, "tm_copy_many: NULL jobs");
    CopyArgs a{};
    int64_t most = 0;
    for (int i = 0; i < n_jobs; ++i) {
        if (jobs[i].n < 0 || (jobs[i].n > 0 && (!jobs[i].src || !jobs[i].dst)))
            return fail(TM_E_ARG, "tm_copy_many: bad job " + std::to_string(i));
        a.job[i] = jobs[i];
        most = std::max(most, jobs[i].n);
    }
    if (most == 0) return TM_OK;
    const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((most + 255) / 256, 256));
    copy_many_kernel<<<dim3(bx, (unsigned)n_jobs), 256, 0, (hipStream_t)stream>>>(a);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, float lr,
                            float beta1, float beta2, float eps, float weight_decay, float grad_scale, float *step,
                            uint32_t *done, int32_t advance, void *stream) {
    if (n < 0 || !(lr >= 0.f) || !(beta1 >= 0.f && beta1 < 1.f) || !(beta2 >= 0.f && beta2 < 1.f) || !(eps >= 0.f))
        return fail(TM_E_ARG, "tm_adam_step: bad arguments");
    if (n == 0) return TM_OK;
    if (!param || !grad || !exp_avg || !exp_avg_sq || !step || !done) return fail(TM_E_ARG, "tm_adam_step: NULL pointer");
    const uintptr_t mis = reinterpret_cast<uintptr_t>(param) & 15;
    for (const void *q : {(const void *)grad, (const void *)exp_avg, (const void *)exp_avg_sq})
        if ((reinterpret_cast<uintptr_t>(q) & 15) != mis || (mis & 3))
            return fail(TM_E_ARG, "tm_adam_step: the four buffers must share their offset within 16 bytes");
    const int64_t head = std::min<int64_t>(n, (int64_t)((16 - mis) & 15) / 4);
    AdamArgs a{param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay, grad_scale, step, done,
               head, advance ? 1 : 0};
    const int64_t n4 = (n - head) >> 2;
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 2048));
    hipEvent_t pe = prof_begin((hipStream_t)stream);
    adam_kernel<<<dim3(blocks), 256, 0, (hipStream_t)stream>>>(a);
    TM_CHECK_LAUNCH();
    prof_end("adam_kernel", (hipStream_t)stream, pe);
    return TM_OK;
}
