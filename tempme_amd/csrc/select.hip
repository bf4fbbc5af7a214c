// threshold_test masking on gfx950 (temp_exp_main.py:153-181, tgn / tgat branches).
//
// The reference picks the (n - topk) least important subgraph entries with
// torch.topk(imp, k, largest=False) on the CPU and zeroes their node ids.  Explanation scores tie
// often (the same edge id appears in several slots and gets the same score), so WHICH of several
// tied entries fall inside the cut is part of the result.  ATen's CPU top-k (TopKImpl.h) copies the
// row into (value, index) pairs and runs libstdc++'s std::nth_element(first, first + k - 1, last)
// -- or std::partial_sort(first, first + k, last) when 64*k <= n -- with a value-only comparator
// (NaN ordered last); the selected set is whatever those algorithms leave in front.  This kernel
// runs the same algorithms (introselect: median-of-three pivot, unguarded Hoare partition,
// 2*floor(log2 n) depth limit, heap-select fallback, insertion sort below 4 elements; heap select
// for partial_sort) step for step, so its set equals the reference's, ties included.
//
// One thread per (group, row): the pair array lives in that thread's slice of LDS.  The work is
// O(n log n) scalar steps per row over a few thousand rows: latency-bound, far below the contrast
// it feeds.
#include <algorithm>

#include "common.h"
#include "topk_select.h"

namespace tmk {

__global__ void __launch_bounds__(64) mask_least_kernel(const float *__restrict__ imp, int32_t rows, int32_t n,
                                                        const int32_t *__restrict__ k_of_group, int32_t n_groups,
                                                        const int32_t *__restrict__ node_in,
                                                        int32_t *__restrict__ node_out) {
    extern __shared__ float lds[];
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)rows * n_groups) return;
    const int32_t g = (int32_t)(t / rows), r = (int32_t)(t % rows);
    PairArr A{lds + (size_t)threadIdx.x * n, reinterpret_cast<int32_t *>(lds + (size_t)blockDim.x * n) +
                                                 (size_t)threadIdx.x * n};
    const float *row = imp + (int64_t)r * n;
    for (int j = 0; j < n; ++j) {
        A.v[j] = row[j];
        A.x[j] = j;
    }
    const int k = min(k_of_group[g], n);
    topk_smallest_select(A, n, k);
    const int32_t *in = node_in + (int64_t)r * n;
    int32_t *out = node_out + ((int64_t)g * rows + r) * n;
    for (int j = 0; j < n; ++j) out[j] = in[j];
    for (int j = 0; j < k; ++j) out[A.x[j]] = 0;
}

}  // namespace tmk

using namespace tmk;

extern "C" int tm_mask_least_important(const float *imp, int32_t rows, int32_t n, const int32_t *k_of_group,
                                       int32_t n_groups, const int32_t *node_in, int32_t *node_out, void *stream) {
    if (rows < 0 || n_groups < 0 || n <= 0 || n > 4096) return fail(TM_E_ARG, "tm_mask_least_important: bad sizes");
    const int64_t total = (int64_t)rows * n_groups;
    if (total == 0) return TM_OK;
    if (!imp || !k_of_group || !node_in || !node_out) return fail(TM_E_ARG, "tm_mask_least_important: NULL pointer");
    // threads per block: as many (value, index) slices of 8n bytes as fit in 64 KB of LDS
    int tpb = (int)std::min<int64_t>(64, (64 * 1024) / (8 * (int64_t)n));
    if (tpb < 1) tpb = 1;
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t pe = prof_begin(s);
    mask_least_kernel<<<dim3((unsigned)((total + tpb - 1) / tpb)), tpb, (size_t)8 * n * tpb, s>>>(
        imp, rows, n, k_of_group, n_groups, node_in, node_out);
    TM_CHECK_LAUNCH();
    prof_end("mask_least_kernel", s, pe);
    return TM_OK;
}
