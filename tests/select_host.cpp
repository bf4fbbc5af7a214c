// Host build of tempme_amd/csrc/topk_select.h for tests/test_select_host.py.
#include <vector>

#include "../tempme_amd/csrc/topk_select.h"

extern "C" void select_rows(const float *v, int64_t rows, int n, int k, int32_t *out) {
    std::vector<float> vv(n);
    std::vector<int32_t> xx(n);
    for (int64_t r = 0; r < rows; ++r) {
        for (int j = 0; j < n; ++j) {
            vv[j] = v[r * n + j];
            xx[j] = j;
        }
        tmk::PairArr A{vv.data(), xx.data()};
        tmk::topk_smallest_select(A, n, k);
        for (int j = 0; j < k; ++j) out[r * k + j] = xx[j];
    }
}
