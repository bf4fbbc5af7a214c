// Library-internal device scratch, one growing buffer per (device, stream): kernels that need a
// per-launch partials array (e.g. per-workgroup histogram bins) take it from here instead of
// widening the C ABI.  Work on one stream is ordered, so reuse across calls on it is safe.
#include <map>
#include <mutex>
#include <utility>

#include "common.h"

namespace tmk {
namespace {
std::mutex g_mu;
std::map<std::pair<int, hipStream_t>, std::pair<void *, size_t>> g_bufs;
}  // namespace

void *scratch(size_t bytes, hipStream_t stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_mu);
    auto &b = g_bufs[{dev, stream}];
    if (b.second < bytes) {
        if (b.first) {
            (void)hipStreamSynchronize(stream);   // the previous launch on this stream may still read it
            (void)hipFree(b.first);
        }
        b.first = nullptr;
        b.second = 0;
        size_t cap = 1 << 20;
        while (cap < bytes) cap <<= 1;
        if (hipMalloc(&b.first, cap) != hipSuccess) return nullptr;
        b.second = cap;
    }
    return b.first;
}
}  // namespace tmk
