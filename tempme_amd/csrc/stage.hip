// Host arrays of the reference's eval loop read by the GPU in place (the drop-in's host-pack path: the reference's
// load_subgraph_margin / np.load arrays, utils/batch_loader.py:119-242, handed to TempME.forward /
// retrieve_explanation per batch as float64 / int64 numpy views, temp_exp_main.py:441-453).
//
// tm_host_register pins and maps a large host array once (hipHostRegister, page-rounded); tm_stage_cast then reads
// a call's views straight from that memory (no host-side cast and no pinned staging copy): one launch gathers every
// view of the call -- any dtype of the pack (int64 / float64 / int32 / float32), up to 5 dims with arbitrary byte
// strides -- converts it to the kernels' int32 / float32 (C conversions: truncation toward zero, round to nearest,
// as numpy's astype and torch's .to) and writes it contiguous on the device; a job with a bound clamps its int32
// row indices into the table (the caller checked them once per array: a guard, not a conversion).
#include <mutex>
#include <unistd.h>
#include <unordered_map>

#include "common.h"

namespace tmk {

constexpr int kMaxStageJobs = 16;

struct StageArgs {
    tm_stage_job job[kMaxStageJobs];
};

__device__ __forceinline__ double load_as_double(const char *p, int type) {
    switch (type) {
        case TM_I64: return (double)*reinterpret_cast<const int64_t *>(p);
        case TM_F64: return *reinterpret_cast<const double *>(p);
        case TM_I32: return (double)*reinterpret_cast<const int32_t *>(p);
        default: return (double)*reinterpret_cast<const float *>(p);
    }
}

// blockIdx.y = job; its elements (row-major over shape) grid-strided over blockIdx.x
__global__ void __launch_bounds__(256) stage_cast_kernel(StageArgs a) {
    const tm_stage_job &j = a.job[blockIdx.y];
    int64_t total = 1;
    for (int d = 0; d < j.ndim; ++d) total *= j.shape[d];
    const char *src = static_cast<const char *>(j.src);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t rem = i, off = 0;
        for (int d = j.ndim - 1; d >= 0; --d) {
            const int64_t c = rem % j.shape[d];
            rem /= j.shape[d];
            off += c * j.stride[d];
        }
        const char *p = src + off;
        if (j.dst_type == TM_I32) {
            int32_t v;
            if (j.src_type == TM_I64) v = (int32_t)*reinterpret_cast<const int64_t *>(p);
            else if (j.src_type == TM_I32) v = *reinterpret_cast<const int32_t *>(p);
            else v = (int32_t)load_as_double(p, j.src_type);
            if (j.bound > 0) v = min(max(v, 0), j.bound - 1);
            static_cast<int32_t *>(j.dst)[i] = v;
        } else if (j.dst_type == TM_F32) {
            static_cast<float *>(j.dst)[i] = j.src_type == TM_F32 ? *reinterpret_cast<const float *>(p)
                                                                   : (float)load_as_double(p, j.src_type);
        } else {
            static_cast<double *>(j.dst)[i] = load_as_double(p, j.src_type);
        }
    }
}

struct Reg {
    char *base;          // page-rounded host address
    size_t bytes;
    char *dev;           // its device address
};
static std::mutex g_reg_mu;
static std::unordered_map<uintptr_t, Reg> g_regs;   // key: the caller's pointer

}  // namespace tmk

using namespace tmk;

extern "C" int tm_host_register(void *ptr, int64_t bytes, void **dev_ptr) {
    if (!ptr || bytes <= 0 || !dev_ptr) return fail(TM_E_ARG, "tm_host_register: bad arguments");
    const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t p = reinterpret_cast<uintptr_t>(ptr);
    char *base = reinterpret_cast<char *>(p & ~(page - 1));
    const size_t len = (size_t)(((p + (uintptr_t)bytes + page - 1) & ~(page - 1)) - (uintptr_t)base);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    if (g_regs.count(p)) return fail(TM_E_ARG, "tm_host_register: already registered");
    // a refused registration (pages shared with another registered range, say) is an expected outcome here: clear
    // the runtime's sticky last error, which the caller's next HIP call (torch's launch checks) would report
    hipError_t e = hipHostRegister(base, len, hipHostRegisterMapped);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(TM_E_HIP, std::string("tm_host_register: ") + hipGetErrorString(e));
    }
    void *d = nullptr;
    e = hipHostGetDevicePointer(&d, base, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(base);
        (void)hipGetLastError();
        return fail(TM_E_HIP, std::string("tm_host_register: hipHostGetDevicePointer: ") + hipGetErrorString(e));
    }
    g_regs[p] = Reg{base, len, static_cast<char *>(d)};
    *dev_ptr = static_cast<char *>(d) + (p - reinterpret_cast<uintptr_t>(base));
    return TM_OK;
}

extern "C" int tm_host_unregister(void *ptr) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_regs.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == g_regs.end()) return fail(TM_E_ARG, "tm_host_unregister: not registered");
    const hipError_t e = hipHostUnregister(it->second.base);
    g_regs.erase(it);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(TM_E_HIP, std::string("tm_host_unregister: ") + hipGetErrorString(e));
    }
    return TM_OK;
}

extern "C" int tm_stage_cast(const tm_stage_job *jobs, int32_t n_jobs, void *stream) {
    if (n_jobs < 0 || n_jobs > kMaxStageJobs) return fail(TM_E_ARG, "tm_stage_cast: bad job count");
    if (n_jobs == 0) return TM_OK;
    if (!jobs) return fail(TM_E_ARG, "tm_stage_cast: NULL jobs");
    StageArgs a{};
    int64_t most = 0;
    for (int i = 0; i < n_jobs; ++i) {
        const tm_stage_job &j = jobs[i];
        if (!j.src || !j.dst || j.ndim < 1 || j.ndim > 5 || j.src_type < TM_I32 || j.src_type > TM_F64 ||
            j.dst_type < TM_I32 || j.dst_type > TM_F64 || j.bound < 0 || (j.bound > 0 && j.dst_type != TM_I32))
            return fail(TM_E_ARG, "tm_stage_cast: bad job " + std::to_string(i));
        int64_t n = 1;
        for (int d = 0; d < j.ndim; ++d) {
            if (j.shape[d] < 0) return fail(TM_E_ARG, "tm_stage_cast: negative extent");
            n *= j.shape[d];
        }
        most = std::max(most, n);
        a.job[i] = j;
    }
    if (most == 0) return TM_OK;
    const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((most + 255) / 256, 512));
    stage_cast_kernel<<<dim3(bx, (unsigned)n_jobs), 256, 0, (hipStream_t)stream>>>(a);
    TM_CHECK_LAUNCH();
    return TM_OK;
}
