// Per-kernel HIP-event timing, recorded on each kernel's own launch stream.  Enabled by
// bench.py (tm_profile_enable) to measure the live per-launch duration of every kernel
// over the timed region; off (one branch per launch) otherwise.
#include <map>
#include <string>
#include <vector>

#include "common.h"

namespace tmk {
namespace {
struct Rec2 {
    const char *name;
    hipEvent_t a, b;
};
bool g_on = false;
std::vector<Rec2> g_recs;
std::vector<hipEvent_t> g_pool;
std::map<std::string, std::pair<double, int64_t>> g_acc;
std::vector<std::string> g_names;

hipEvent_t get_event() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}
}  // namespace

hipEvent_t prof_begin(hipStream_t s) {
    if (!g_on) return nullptr;
    hipEvent_t a = get_event();
    (void)hipEventRecord(a, s);
    return a;
}

void prof_end(const char *name, hipStream_t s, hipEvent_t a) {
    if (!g_on || !a) return;
    hipEvent_t b = get_event();
    (void)hipEventRecord(b, s);
    g_recs.push_back({name, a, b});
}
}  // namespace tmk

using namespace tmk;

extern "C" int tm_profile_enable(int on) {
    g_on = on != 0;
    for (auto &r : g_recs) {
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    g_recs.clear();
    g_acc.clear();
    g_names.clear();
    return TM_OK;
}

extern "C" int tm_profile_sync(void) {
    for (auto &r : g_recs) {
        if (hipEventSynchronize(r.b) != hipSuccess) return fail(TM_E_HIP, "tm_profile_sync: event sync failed");
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, r.a, r.b);
        auto &x = g_acc[r.name];
        x.first += ms;
        x.second += 1;
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    g_recs.clear();
    g_names.clear();
    for (auto &kv : g_acc) g_names.push_back(kv.first);
    return (int)g_names.size();
}

extern "C" int tm_profile_entry(int i, const char **name, double *total_ms, int64_t *count) {
    if (i < 0 || i >= (int)g_names.size()) return fail(TM_E_ARG, "tm_profile_entry: index out of range");
    auto &x = g_acc[g_names[i]];
    if (name) *name = g_names[i].c_str();
    if (total_ms) *total_ms = x.first;
    if (count) *count = x.second;
    return TM_OK;
}
