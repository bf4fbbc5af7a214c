// Host side of the drop-in eval fast path (TempME.forward / retrieve_explanation on device-pack views,
// the call pattern of temp_exp_main.py:441-453): the per-call checks, the weight-version key, the
// side-stream output allocation, the gate-factor cache and the library calls that explainer.py's
// _dropin_forward / _dropin_retrieve do in Python, as one C++ call each (a Python extension on torch's
// C++ API).  The kernels are the C-ABI entry points of libtempme_hip.so (include/tempme.h), called
// through the function pointers the Python side hands over (no link-time dependency).  Every check
// that fails returns None and the caller takes the Python path, which gives the same results.
#include <Python.h>
#include <pybind11/pybind11.h>
#include <torch/csrc/autograd/python_variable.h>
#include <ATen/core/Tensor.h>
#include <ATen/ops/empty.h>
#include <c10/core/GradMode.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <deque>
#include <vector>

namespace py = pybind11;

namespace {

// include/tempme.h: tm_dropin_forward, tm_edge_importance_gf3, tm_edge_importance_gf3_bern
using FwdFn = int (*)(void *d, int32_t k, int32_t sync, const void *w, const float *n_feat, const float *e_feat,
                      const float *etab, int32_t B, int32_t W, const int32_t *node6, const int32_t *eid3,
                      const float *ts3, const int32_t *cat, const double *cut_host, const double *cut_dev,
                      const float *cnt, float *out_imp, float *out_gfac, void *stream);
using Gf3Fn = int (*)(int32_t B, int32_t W, int32_t N, const float *, const float *, const float *, const int32_t *,
                      const int32_t *, const int32_t *, const float *, const float *, const float *, const int32_t *,
                      const int32_t *, const int32_t *, const int32_t *, const int32_t *, const int32_t *,
                      const int32_t *, const int32_t *, const int32_t *, const int32_t *, const int32_t *,
                      const int32_t *, float *, float *, void *);
using Gf3BernFn = int (*)(int32_t B, int32_t W, int32_t N, const float *, const float *, const float *,
                          const int32_t *, const int32_t *, const int32_t *, const float *, const float *,
                          const float *, const int32_t *, const int32_t *, const int32_t *, const int32_t *,
                          const int32_t *, const int32_t *, const int32_t *, const int32_t *, const int32_t *,
                          const int32_t *, const int32_t *, const int32_t *, float *, float *, float *, float *,
                          void *);

constexpr int kSides = 3, kCache = 6, kMaxHostCut = 512;

// host-time split of Fast.forward (diagnostics: prof_enable / prof_read, tools/dropin_timing.py): nanoseconds per
// segment summed over the calls since enabled
bool g_prof_on = false;
int64_t g_prof[8] = {}, g_prof_n = 0;
inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

bool is_tensor(PyObject *o) { return THPVariable_Check(o); }

// contiguous, on the context's device, of the given type: what the kernels' pointer arithmetic assumes
bool plain(const at::Tensor &t, int device, at::ScalarType ty) {
    return t.is_cuda() && t.get_device() == device && t.scalar_type() == ty && t.is_contiguous();
}

// a tensor the device pack handed out (pack.DevicePack views carry _tm_resident = True)
bool resident(PyObject *o) {
    if (!is_tensor(o)) return false;
    PyObject *a = PyObject_GetAttrString(o, "_tm_resident");
    if (!a) {
        PyErr_Clear();
        return false;
    }
    const bool r = PyObject_IsTrue(a) == 1;
    Py_DECREF(a);
    return r;
}

struct Watched {   // one tensor of the weight-version key
    at::Tensor t;
    const void *ptr;
    int64_t version;
    bool rg, track_rg;
};

// one forward's gate factors, for retrieve_explanation with the very same walk tensors
struct GfEntry {
    at::Tensor e3, t3, out;   // the walk eid / ts views (identity + version) and [imp | gate factors]
    int64_t v_e3, v_t3;
    int64_t B, W;
};

class Fast {
  public:
    Fast(py::list watched, py::list track_rg, py::object reg_gen, int64_t reg_gen_value, int64_t ctx, int64_t fwd,
         int64_t gf3, int64_t gf3b, int64_t wts, int64_t nt, int64_t et, int64_t etab, py::list side_ids, int device,
         bool enc_grad)
        : reg_gen_(reg_gen), reg_gen_value_(reg_gen_value), ctx_(reinterpret_cast<void *>(ctx)),
          fwd_(reinterpret_cast<FwdFn>(fwd)), gf3_(reinterpret_cast<Gf3Fn>(gf3)),
          gf3b_(reinterpret_cast<Gf3BernFn>(gf3b)), wts_(reinterpret_cast<const void *>(wts)),
          nt_(reinterpret_cast<const float *>(nt)), et_(reinterpret_cast<const float *>(et)),
          etab_(reinterpret_cast<const float *>(etab)), device_(device), enc_grad_(enc_grad) {
        for (size_t i = 0; i < watched.size(); ++i) {
            const at::Tensor &t = THPVariable_Unpack(watched[i].ptr());
            const bool tr = py::cast<bool>(track_rg[i]);
            watched_.push_back(Watched{t, t.data_ptr(), t._version(), t.requires_grad(), tr});
        }
        for (size_t k = 0; k < side_ids.size() && k < (size_t)kSides; ++k) {
            py::tuple s = side_ids[k];
            // torch's ROCm build hands out HIP streams typed as CUDA streams (masquerading); the c10::hip
            // stream object wants the HIP device type for the same (index, id)
            side_[k] = c10::hip::HIPStream(c10::Stream(c10::Stream::UNSAFE,
                                                       c10::Device(c10::DeviceType::HIP,
                                                                   static_cast<c10::DeviceIndex>(py::cast<int64_t>(s[1]))),
                                                       static_cast<c10::StreamId>(py::cast<int64_t>(s[0]))));
        }
    }

    // the weights, tables and module registrations the state was built from are unchanged
    bool current() const {
        PyObject *g = PyList_GetItem(reg_gen_.ptr(), 0);
        if (!g || PyLong_AsLongLong(g) != reg_gen_value_) {
            PyErr_Clear();
            return false;
        }
        for (const Watched &w : watched_)
            if (w.t.data_ptr() != w.ptr || w.t._version() != w.version || (w.track_rg && w.t.requires_grad() != w.rg))
                return false;
        return true;
    }

    // TempME.forward (eval) on device-pack views of one batch: (imp [B, W, 1], rc, needs_grad) or None
    py::object forward(py::handle node_idx, py::handle edge_idx, py::handle time_idx, py::handle cat_feat,
                       py::handle cut_time, py::handle edge_identify) {
        int64_t T[8];
        const bool pr = g_prof_on;
        if (pr) T[0] = now_ns();
        if (!(resident(edge_idx.ptr()) && resident(node_idx.ptr()) && resident(time_idx.ptr()) &&
              resident(cat_feat.ptr()) && resident(edge_identify.ptr())))
            return py::none();
        if (pr) T[1] = now_ns();
        const at::Tensor &e3 = THPVariable_Unpack(edge_idx.ptr());
        const at::Tensor &n6 = THPVariable_Unpack(node_idx.ptr());
        const at::Tensor &t3 = THPVariable_Unpack(time_idx.ptr());
        const at::Tensor &ct = THPVariable_Unpack(cat_feat.ptr());
        const at::Tensor &cn = THPVariable_Unpack(edge_identify.ptr());
        if (e3.dim() != 3 || e3.size(2) != 3) return py::none();
        const int64_t B = e3.size(0), W = e3.size(1);
        if (B == 0 || n6.dim() != 3 || n6.size(0) != B || n6.size(1) != W || n6.size(2) != 6 || t3.dim() != 3 ||
            t3.size(0) != B || t3.size(1) != W || t3.size(2) != 3 || ct.dim() < 2 || ct.size(0) != B ||
            ct.size(1) != W || cn.dim() != 4 || cn.size(0) != B || cn.size(1) != W || cn.size(2) != 3 ||
            cn.size(3) != 3 || !plain(e3, device_, at::kInt) || !plain(t3, device_, at::kFloat) ||
            !plain(n6, device_, at::kInt) || !plain(ct, device_, at::kInt) || !plain(cn, device_, at::kFloat))
            return py::none();
        // cut times: a host float64 array (sent as kernel arguments) or a device float64 tensor
        const double *cut_h = nullptr, *cut_d = nullptr;
        if (is_tensor(cut_time.ptr())) {
            const at::Tensor &c = THPVariable_Unpack(cut_time.ptr());
            if (!c.is_cuda() || c.get_device() != device_ || c.scalar_type() != at::kDouble || c.numel() != B ||
                !c.is_contiguous())
                return py::none();
            cut_d = c.data_ptr<double>();
        } else {
            Py_buffer view;
            if (PyObject_GetBuffer(cut_time.ptr(), &view, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) {
                PyErr_Clear();
                return py::none();
            }
            const bool ok = view.format && view.format[0] == 'd' && view.format[1] == 0 && view.itemsize == 8 &&
                            view.len == (Py_ssize_t)(8 * B) && B <= kMaxHostCut;
            cut_h = static_cast<const double *>(view.buf);
            PyBuffer_Release(&view);   // the array object itself stays alive for this call (the caller holds it)
            if (!ok) return py::none();
        }
        if (pr) T[2] = now_ns();
        if (!current()) return py::none();
        if (pr) T[3] = now_ns();
        const int k = next_k_;
        next_k_ = (k + 1) % kSides;
        c10::hip::HIPStream cur = c10::hip::getCurrentHIPStream(device_);
        at::Tensor out;
        {
            // the outputs come from side stream k's pool (its kernels write them) and are recorded as used by
            // the caller's stream, which reads them after the wait tm_dropin_forward enqueues
            c10::hip::HIPStreamGuard g(side_[k]);
            out = at::empty({B * W * 4}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
        }
        if (pr) T[4] = now_ns();
        c10::hip::HIPCachingAllocator::recordStream(out.storage().data_ptr(), cur);
        if (pr) T[5] = now_ns();
        const int sync = (cut_d != nullptr || dirty_) ? 1 : 0;
        dirty_ = false;
        float *o = out.data_ptr<float>();
        const int rc = fwd_(ctx_, k, sync, wts_, nt_, et_, etab_, (int32_t)B, (int32_t)W, n6.data_ptr<int32_t>(),
                            e3.data_ptr<int32_t>(), t3.data_ptr<float>(), ct.data_ptr<int32_t>(), cut_h, cut_d,
                            cn.data_ptr<float>(), o, o + B * W, cur.stream());
        if (rc != 0) return py::make_tuple(py::none(), rc, false);
        if (pr) T[6] = now_ns();
        at::Tensor imp = out.as_strided({B, W, 1}, {W, 1, 1});
        cache_.push_back(GfEntry{e3, t3, out, e3._version(), t3._version(), B, W});
        if (cache_.size() > kCache) cache_.pop_front();
        ++hits_;
        const bool grad = enc_grad_ && c10::GradMode::is_enabled();
        py::object res = py::make_tuple(py::reinterpret_steal<py::object>(THPVariable_Wrap(imp)), 0, grad);
        if (pr) {
            T[7] = now_ns();
            for (int i = 0; i < 7; ++i) g_prof[i] += T[i + 1] - T[i];
            ++g_prof_n;
        }
        return res;
    }

    // retrieve_explanation for the three sides' (subgraph, graphlet_imp, walks) whose walks went through
    // forward(): one launch.  Returns (out, rc, side tensors) -- out = [hop-1 | hop-2] concatenated, or with
    // bern [p | keep] -- or None.
    py::object retrieve(py::sequence sides, bool bern) {
        if (sides.size() != kSides || cache_.empty() || !current()) return py::none();
        struct Side {
            const GfEntry *h;
            at::Tensor imp, n1, x1, n2, x2;
        } sd[kSides];
        for (int s = 0; s < kSides; ++s) {
            py::object side = sides[s];
            py::object subgraph = side[py::int_(0)], imp = side[py::int_(1)], walks = side[py::int_(2)];
            py::object e3o = walks[py::int_(1)], t3o = walks[py::int_(2)];
            if (!is_tensor(e3o.ptr()) || !is_tensor(t3o.ptr()) || !is_tensor(imp.ptr())) return py::none();
            const at::Tensor &e3 = THPVariable_Unpack(e3o.ptr());
            const at::Tensor &t3 = THPVariable_Unpack(t3o.ptr());
            const GfEntry *h = nullptr;
            for (auto it = cache_.rbegin(); it != cache_.rend(); ++it)
                if (it->e3.unsafeGetTensorImpl() == e3.unsafeGetTensorImpl() &&
                    it->t3.unsafeGetTensorImpl() == t3.unsafeGetTensorImpl()) {
                    h = &*it;
                    break;
                }
            if (!h || e3._version() != h->v_e3 || t3._version() != h->v_t3) return py::none();
            py::object nodes = subgraph[py::int_(0)], eids = subgraph[py::int_(1)];
            py::object n1o = nodes[py::int_(0)], n2o = nodes[py::int_(1)], x1o = eids[py::int_(0)],
                       x2o = eids[py::int_(1)];
            if (!(resident(n1o.ptr()) && resident(x1o.ptr()) && resident(n2o.ptr()) && resident(x2o.ptr())))
                return py::none();
            sd[s].h = h;
            sd[s].imp = THPVariable_Unpack(imp.ptr());
            sd[s].n1 = THPVariable_Unpack(n1o.ptr());
            sd[s].x1 = THPVariable_Unpack(x1o.ptr());
            sd[s].n2 = THPVariable_Unpack(n2o.ptr());
            sd[s].x2 = THPVariable_Unpack(x2o.ptr());
        }
        const int64_t B = sd[0].h->B, W = sd[0].h->W;
        if (sd[0].n1.dim() != 2) return py::none();
        const int64_t N = sd[0].n1.size(1);
        for (int s = 0; s < kSides; ++s) {
            const Side &x = sd[s];
            if (x.h->B != B || x.h->W != W || !plain(x.imp, device_, at::kFloat) || x.imp.numel() != B * W ||
                x.n1.dim() != 2 || x.n1.size(0) != B || x.n1.size(1) != N || !plain(x.n1, device_, at::kInt) ||
                !x.x1.sizes().equals(x.n1.sizes()) || !plain(x.x1, device_, at::kInt) || x.n2.dim() != 2 ||
                x.n2.size(0) != B || x.n2.size(1) != N * N || !plain(x.n2, device_, at::kInt) ||
                !x.x2.sizes().equals(x.n2.sizes()) || !plain(x.x2, device_, at::kInt))
                return py::none();
        }
        const int64_t n_out = 3 * B * (N + N * N);
        at::Tensor o = at::empty({n_out * (bern ? 2 : 1)}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
        float *p1 = o.data_ptr<float>(), *p2 = p1 + 3 * B * N;
        auto gf = [&](int s) { return sd[s].h->out.data_ptr<float>() + B * W; };
        auto i32 = [](const at::Tensor &t) { return t.data_ptr<int32_t>(); };
        hipStream_t st = c10::hip::getCurrentHIPStream(device_).stream();
        int rc;
        if (bern) {
            float *k1 = p1 + n_out, *k2 = k1 + 3 * B * N;
            rc = gf3b_((int32_t)B, (int32_t)W, (int32_t)N, gf(0), gf(1), gf(2), i32(sd[0].h->e3), i32(sd[1].h->e3),
                       i32(sd[2].h->e3), sd[0].imp.data_ptr<float>(), sd[1].imp.data_ptr<float>(),
                       sd[2].imp.data_ptr<float>(), i32(sd[0].n1), i32(sd[1].n1), i32(sd[2].n1), i32(sd[0].x1),
                       i32(sd[1].x1), i32(sd[2].x1), i32(sd[0].n2), i32(sd[1].n2), i32(sd[2].n2), i32(sd[0].x2),
                       i32(sd[1].x2), i32(sd[2].x2), p1, p2, k1, k2, st);
        } else {
            rc = gf3_((int32_t)B, (int32_t)W, (int32_t)N, gf(0), gf(1), gf(2), i32(sd[0].h->e3), i32(sd[1].h->e3),
                      i32(sd[2].h->e3), sd[0].imp.data_ptr<float>(), sd[1].imp.data_ptr<float>(),
                      sd[2].imp.data_ptr<float>(), i32(sd[0].n1), i32(sd[1].n1), i32(sd[2].n1), i32(sd[0].x1),
                      i32(sd[1].x1), i32(sd[2].x1), i32(sd[0].n2), i32(sd[1].n2), i32(sd[2].n2), i32(sd[0].x2),
                      i32(sd[1].x2), i32(sd[2].x2), p1, p2, st);
        }
        py::list args;
        for (int s = 0; s < kSides; ++s) {
            auto w = [](const at::Tensor &t) { return py::reinterpret_steal<py::object>(THPVariable_Wrap(t)); };
            args.append(py::make_tuple(w(sd[s].h->e3), w(sd[s].h->t3), w(sd[s].n1), w(sd[s].x1), w(sd[s].n2),
                                       w(sd[s].x2), B, W, N));
        }
        ++hits_;
        return py::make_tuple(py::reinterpret_steal<py::object>(THPVariable_Wrap(o)), rc, args);
    }

    // a forward the Python path ran (the call that built this state): its gate factors join the cache
    void push(py::handle edge_idx, py::handle time_idx, py::handle out, int64_t B, int64_t W) {
        const at::Tensor &e3 = THPVariable_Unpack(edge_idx.ptr());
        const at::Tensor &t3 = THPVariable_Unpack(time_idx.ptr());
        cache_.push_back(GfEntry{e3, t3, THPVariable_Unpack(out.ptr()), e3._version(), t3._version(), B, W});
        if (cache_.size() > kCache) cache_.pop_front();
    }

    int64_t hits() const { return hits_; }
    size_t cached() const { return cache_.size(); }

  private:
    std::vector<Watched> watched_;
    py::object reg_gen_;
    int64_t reg_gen_value_;
    void *ctx_;
    FwdFn fwd_;
    Gf3Fn gf3_;
    Gf3BernFn gf3b_;
    const void *wts_;
    const float *nt_, *et_, *etab_;
    int device_;
    bool enc_grad_;
    bool dirty_ = true;   // a new state follows new weights / tables / context: every side stream waits once
    int next_k_ = 0;
    int64_t hits_ = 0;
    c10::hip::HIPStream side_[kSides] = {c10::hip::getDefaultHIPStream(), c10::hip::getDefaultHIPStream(),
                                         c10::hip::getDefaultHIPStream()};
    std::deque<GfEntry> cache_;
};

// include/tempme.h tm_stage_job / tm_stage_cast (the host-pack staging of hoststage.stage)
struct StageJob {
    const void *src;
    void *dst;
    int32_t src_type, dst_type, ndim, bound;
    int64_t shape[5];
    int64_t stride[5];
};
using StageFn = int (*)(const StageJob *jobs, int32_t n_jobs, void *stream);
constexpr int kI32 = 1, kF32 = 2, kI64 = 3, kF64 = 4, kMaxStage = 16;

int buffer_type(const char *f, Py_ssize_t itemsize) {
    if (!f) return 0;
    while (*f == '<' || *f == '=' || *f == '@') ++f;
    if (f[0] == 0 || f[1] != 0) return 0;
    switch (f[0]) {
        case 'd': return itemsize == 8 ? kF64 : 0;
        case 'f': return itemsize == 4 ? kF32 : 0;
        case 'i': return itemsize == 4 ? kI32 : 0;
        case 'l': case 'q': return itemsize == 8 ? kI64 : 0;
        default: return 0;
    }
}

// hoststage.stage's per-call work for views of registered host arrays, on the current stream of `device`:
// items = [(array, dst type 1 int32 | 2 float32, bound, registered start, registered length, its device address)].
// Every view must lie inside its registration; one allocation, one tm_stage_cast launch.  The outputs (torch
// tensors shaped as the views) or None when any item does not qualify (the Python path then decides).
py::object stage_host(py::list items, int device, int64_t fn) {
    const size_t n = items.size();
    if (n == 0 || n > (size_t)kMaxStage) return py::none();
    StageJob jobs[kMaxStage] = {};
    std::vector<std::vector<int64_t>> shapes(n);
    int64_t off[kMaxStage], total = 0;
    for (size_t i = 0; i < n; ++i) {
        py::tuple it = items[i].cast<py::tuple>();
        Py_buffer v;
        if (PyObject_GetBuffer(it[0].ptr(), &v, PyBUF_RECORDS_RO) != 0) {
            PyErr_Clear();
            return py::none();
        }
        const int st = buffer_type(v.format, v.itemsize);
        const int dt = it[1].cast<int>();
        const int64_t bound = it[2].cast<int64_t>(), lo = it[3].cast<int64_t>(), len = it[4].cast<int64_t>(),
                      dev = it[5].cast<int64_t>();
        bool ok = st != 0 && (dt == kI32 || dt == kF32) && v.ndim <= 5 && bound >= 0 && bound < INT32_MAX;
        const uintptr_t p = reinterpret_cast<uintptr_t>(v.buf);
        intptr_t a = (intptr_t)p, b = (intptr_t)p;
        int64_t elems = 1;
        StageJob &j = jobs[i];
        j.ndim = v.ndim > 0 ? v.ndim : 1;
        j.shape[0] = 1;
        for (int d = 0; ok && d < v.ndim; ++d) {
            const int64_t e = v.shape[d], s = v.strides ? v.strides[d] : 0;
            if (e <= 0) ok = false;
            a += std::min<int64_t>(0, (e - 1) * s);
            b += std::max<int64_t>(0, (e - 1) * s);
            j.shape[d] = e;
            j.stride[d] = s;
            elems *= e;
            shapes[i].push_back(e);
        }
        b += v.itemsize;
        PyBuffer_Release(&v);   // the array stays alive: the caller holds it (and the registry holds its base)
        if (!ok || a < lo || b > lo + len) return py::none();
        j.src = reinterpret_cast<const void *>(dev + ((intptr_t)p - lo));
        j.src_type = st;
        j.dst_type = dt;
        j.bound = dt == kI32 ? (int32_t)bound : 0;
        off[i] = total;
        total += (elems * 4 + 15) & ~int64_t(15);
    }
    c10::hip::HIPGuard g(device);
    at::Tensor buf = at::empty({std::max<int64_t>(total, 16)}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, device));
    char *base = static_cast<char *>(buf.data_ptr());
    for (size_t i = 0; i < n; ++i) jobs[i].dst = base + off[i];
    const int rc = reinterpret_cast<StageFn>(fn)(jobs, (int32_t)n, c10::hip::getCurrentHIPStream(device).stream());
    if (rc != 0) return py::make_tuple(py::none(), rc);
    py::list out;
    for (size_t i = 0; i < n; ++i) {
        int64_t elems = 1;
        for (int64_t e : shapes[i]) elems *= e;
        at::Tensor t = buf.narrow(0, off[i], elems * 4).view(jobs[i].dst_type == kI32 ? at::kInt : at::kFloat);
        out.append(py::reinterpret_steal<py::object>(THPVariable_Wrap(t.view(shapes[i]))));
    }
    return py::make_tuple(out, 0);
}

// the data address of a buffer-protocol object (a numpy view), or -1
int64_t buf_addr(py::handle o) {
    Py_buffer v;
    if (PyObject_GetBuffer(o.ptr(), &v, PyBUF_RECORDS_RO) != 0) {
        PyErr_Clear();
        return -1;
    }
    const int64_t a = (int64_t) reinterpret_cast<uintptr_t>(v.buf);
    PyBuffer_Release(&v);
    return a;
}

}  // namespace

PYBIND11_MODULE(_dropin_ext, m) {
    m.def("stage_host", &stage_host);
    m.def("prof_enable", [](bool on) {
        g_prof_on = on;
        for (auto &x : g_prof) x = 0;
        g_prof_n = 0;
    });
    m.def("prof_read", []() {
        py::list l;
        for (int i = 0; i < 7; ++i) l.append(g_prof_n ? (double)g_prof[i] / g_prof_n / 1e3 : 0.0);
        return py::make_tuple(l, g_prof_n);
    });
    m.def("buf_addr", &buf_addr);
    m.doc() = "C++ host side of TempME's drop-in eval fast path (tempme_amd/csrc/dropin_ext.cpp)";
    py::class_<Fast>(m, "Fast")
        .def(py::init<py::list, py::list, py::object, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                      int64_t, int64_t, py::list, int, bool>())
        .def("current", &Fast::current)
        .def("forward", &Fast::forward)
        .def("retrieve", &Fast::retrieve)
        .def("push", &Fast::push)
        .def_property_readonly("hits", &Fast::hits)
        .def_property_readonly("cached", &Fast::cached);
}
