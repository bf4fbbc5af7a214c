// host-side cost of the HIP calls one drop-in forward makes (launch, event record, stream wait)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ void empty_kernel(int *p) { if (p && threadIdx.x == 1000) p[0] = 1; }
struct Big { double v[256]; };
__global__ void big_kernel(int *p, Big b) { if (p && threadIdx.x == 1000) p[0] = (int)b.v[3]; }
int main() {
    hipStream_t s1, s2;
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t e;
    hipEventCreateWithFlags(&e, hipEventDisableTiming);
    const int n = 2000;
    auto t = [] { return std::chrono::high_resolution_clock::now(); };
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    for (int r = 0; r < 2; ++r) {
        hipDeviceSynchronize();
        auto a = t();
        for (int i = 0; i < n; ++i) empty_kernel<<<1, 64, 0, s1>>>(nullptr);
        auto b = t();
        hipDeviceSynchronize();
        auto c = t();
        for (int i = 0; i < n; ++i) empty_kernel<<<256, 256, 0, s1>>>(nullptr);
        auto d = t();
        hipDeviceSynchronize();
        Big big{};
        auto e0 = t();
        for (int i = 0; i < n; ++i) big_kernel<<<1, 64, 0, s1>>>(nullptr, big);
        auto e1 = t();
        hipDeviceSynchronize();
        auto f0 = t();
        for (int i = 0; i < n; ++i) hipEventRecord(e, s1);
        auto f1 = t();
        hipDeviceSynchronize();
        auto g0 = t();
        for (int i = 0; i < n; ++i) hipStreamWaitEvent(s2, e, 0);
        auto g1 = t();
        hipDeviceSynchronize();
        auto h0 = t();
        for (int i = 0; i < n; ++i) { hipEventRecord(e, s1); hipStreamWaitEvent(s2, e, 0); empty_kernel<<<1, 64, 0, s2>>>(nullptr); }
        auto h1 = t();
        hipDeviceSynchronize();
        printf("round %d: launch(1 wg) %.2f us, launch(256 wg) %.2f us, launch(2KB args) %.2f us, eventRecord %.2f us, "
               "streamWaitEvent %.2f us, record+wait+launch %.2f us\n", r, us(a, b) / n, us(c, d) / n, us(e0, e1) / n,
               us(f0, f1) / n, us(g0, g1) / n, us(h0, h1) / n);
    }
    return 0;
}
