// Row gather of several side-major arrays in one launch (tm_gather_rows): the training step's batch
// slice of the device-resident pack (utils/batch_loader.py get_item + get_item_edge, :203-242), which
// torch.index_select did with one kernel per array.
#include "common.h"

namespace tmk {

constexpr int kMaxGatherJobs = 24;

struct GatherArgs {
    tm_gather_job job[kMaxGatherJobs];
};

// blockIdx.y = job; the job's (side, row, 4-byte word) triples grid-strided over blockIdx.x
__global__ void __launch_bounds__(256) gather_rows_kernel(GatherArgs a, const int64_t *__restrict__ rows,
                                                          int64_t n_rows, int32_t *err) {
    const tm_gather_job &j = a.job[blockIdx.y];
    const int64_t words = j.row_bytes >> 2, per_side = n_rows * words, total = per_side * j.sides;
    const char *src = static_cast<const char *>(j.src);
    char *dst = static_cast<char *>(j.dst);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t side = i / per_side, rem = i - side * per_side, r = rem / words, w = rem - r * words;
        const int64_t sr = rows[r];
        if (sr < 0 || sr >= j.src_rows) {
            if (err) atomicCAS(err, 0, TM_E_ARG);
            continue;
        }
        const uint32_t v = *reinterpret_cast<const uint32_t *>(src + side * j.src_side_stride + sr * j.row_bytes + 4 * w);
        *reinterpret_cast<uint32_t *>(dst + side * j.dst_side_stride + r * j.row_bytes + 4 * w) = v;
    }
}

}  // namespace tmk

using namespace tmk;

extern "C" int tm_gather_rows(const tm_gather_job *jobs, int32_t n_jobs, const int64_t *rows, int64_t n_rows,
                              int32_t *err_flag, void *stream) {
    if (n_jobs < 0 || n_jobs > kMaxGatherJobs || n_rows < 0) return fail(TM_E_ARG, "tm_gather_rows: bad arguments");
    if (n_jobs == 0 || n_rows == 0) return TM_OK;
    if (!jobs || !rows) return fail(TM_E_ARG, "tm_gather_rows: NULL pointer");
    GatherArgs a{};
    int64_t most = 0;
    for (int i = 0; i < n_jobs; ++i) {
        const tm_gather_job &j = jobs[i];
        if (!j.src || !j.dst || j.row_bytes <= 0 || (j.row_bytes & 3) || j.sides <= 0 || j.src_rows < 0)
            return fail(TM_E_ARG, "tm_gather_rows: bad job " + std::to_string(i));
        a.job[i] = j;
        most = std::max<int64_t>(most, (int64_t)j.sides * n_rows * (j.row_bytes >> 2));
    }
    const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((most + 255) / 256, 1024));
    gather_rows_kernel<<<dim3(bx, (unsigned)n_jobs), 256, 0, (hipStream_t)stream>>>(a, rows, n_rows, err_flag);
    TM_CHECK_LAUNCH();
    return TM_OK;
}
