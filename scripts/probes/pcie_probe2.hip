// PCIe transfer rates on the MI355X box for planning the chunked host path (boundary 2):
// pageable (pre-touched) vs pinned host memory, one direction at a time and both directions
// concurrently from two host threads on two streams. Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O2 -o scripts/probes/pcie_probe2 scripts/probes/pcie_probe2.hip -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void copy_kernel(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        d[i] = s[i];
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t nb = 512ull << 20, chunk = 64ull << 20;
    const int reps = 4;
    char* pg_in = (char*)malloc(nb);
    char* pg_out = (char*)malloc(nb);
    memset(pg_in, 1, nb);
    memset(pg_out, 2, nb);
    char *pin_in, *pin_out;
    CK(hipHostMalloc((void**)&pin_in, nb, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&pin_out, nb, hipHostMallocDefault));
    memset(pin_in, 1, nb);
    memset(pin_out, 2, nb);
    char *d_in, *d_out;
    CK(hipMalloc((void**)&d_in, nb));
    CK(hipMalloc((void**)&d_out, nb));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));

    auto h2d = [&](const char* src, hipStream_t s) {
        for (size_t o = 0; o < nb; o += chunk) CK(hipMemcpyAsync(d_in + o, src + o, chunk, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    };
    auto d2h = [&](char* dst, hipStream_t s) {
        for (size_t o = 0; o < nb; o += chunk) CK(hipMemcpyAsync(dst + o, d_out + o, chunk, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    };
    auto rate = [&](auto fn) {
        fn();
        double t0 = now();
        for (int r = 0; r < reps; ++r) fn();
        return (double)nb * reps / (now() - t0) / 1e9;
    };
    double h2d_pg = rate([&] { h2d(pg_in, s1); });
    double h2d_pin = rate([&] { h2d(pin_in, s1); });
    double d2h_pg = rate([&] { d2h(pg_out, s2); });
    double d2h_pin = rate([&] { d2h(pin_out, s2); });
    // host time of an async pageable H2D call (does it return before the copy is done?)
    double t0 = now();
    CK(hipMemcpyAsync(d_in, pg_in, nb, hipMemcpyHostToDevice, s1));
    double call_pg = now() - t0;
    CK(hipStreamSynchronize(s1));
    double done_pg = now() - t0;
    t0 = now();
    CK(hipMemcpyAsync(d_in, pin_in, nb, hipMemcpyHostToDevice, s1));
    double call_pin = now() - t0;
    CK(hipStreamSynchronize(s1));
    double done_pin = now() - t0;
    // both directions at once, one host thread each
    auto both = [&](const char* src, char* dst) {
        double ta = 0, tb = 0;
        std::thread a([&] { double s = now(); for (int r = 0; r < reps; ++r) h2d(src, s1); ta = now() - s; });
        std::thread b([&] { double s = now(); for (int r = 0; r < reps; ++r) d2h(dst, s2); tb = now() - s; });
        a.join();
        b.join();
        return std::make_pair((double)nb * reps / ta / 1e9, (double)nb * reps / tb / 1e9);
    };
    both(pg_in, pg_out);
    auto bp = both(pg_in, pg_out);
    auto bn = both(pin_in, pin_out);
    // both directions from one thread, async on two streams (pinned only: truly async)
    t0 = now();
    for (int r = 0; r < reps; ++r) {
        for (size_t o = 0; o < nb; o += chunk) {
            CK(hipMemcpyAsync(d_in + o, pin_in + o, chunk, hipMemcpyHostToDevice, s1));
            CK(hipMemcpyAsync(pin_out + o, d_out + o, chunk, hipMemcpyDeviceToHost, s2));
        }
    }
    CK(hipStreamSynchronize(s1));
    CK(hipStreamSynchronize(s2));
    double bidir_async = (double)nb * reps / (now() - t0) / 1e9;
    // host memcpy pageable -> pinned, 1 and 8 threads
    auto hcopy = [&](int nt) {
        double s = now();
        for (int r = 0; r < reps; ++r) {
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t)
                th.emplace_back([&, t] {
                    size_t per = nb / nt;
                    memcpy(pin_in + t * per, pg_in + t * per, per);
                });
            for (auto& x : th) x.join();
        }
        return (double)nb * reps / (now() - s) / 1e9;
    };
    double hc1 = hcopy(1), hc8 = hcopy(8);
    // D2H variants: synchronous hipMemcpy in 8 MB chunks (pageable, pinned); two streams at once;
    // a kernel storing straight into mapped pinned memory (zero-copy write over PCIe)
    auto d2h_sync = [&](char* dst) {
        for (size_t o = 0; o < nb; o += (8u << 20)) CK(hipMemcpy(dst + o, d_out + o, 8u << 20, hipMemcpyDeviceToHost));
    };
    double d2h_sync_pg = rate([&] { d2h_sync(pg_out); });
    double d2h_sync_pin = rate([&] { d2h_sync(pin_out); });
    double d2h_2s = rate([&] {
        for (size_t o = 0; o < nb; o += chunk) CK(hipMemcpyAsync(pin_out + o, d_out + o, chunk, hipMemcpyDeviceToHost, (o / chunk) & 1 ? s2 : s1));
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
    });
    char* mapped = nullptr;
    CK(hipHostGetDevicePointer((void**)&mapped, pin_out, 0));
    double d2h_kernel = rate([&] {
        hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, s1, (const uint4*)d_out, (uint4*)mapped, nb / 16);
        CK(hipStreamSynchronize(s1));
    });
    double h2d_kernel = rate([&] {
        const char* mi = nullptr;
        CK(hipHostGetDevicePointer((void**)&mi, pin_in, 0));
        hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, s1, (const uint4*)mi, (uint4*)d_in, nb / 16);
        CK(hipStreamSynchronize(s1));
    });
    printf("{\"bytes\": %zu, \"chunk\": %zu, \"h2d_pageable_GBps\": %.2f, \"h2d_pinned_GBps\": %.2f, "
           "\"d2h_pageable_GBps\": %.2f, \"d2h_pinned_GBps\": %.2f, \"async_call_pageable_ms\": %.3f, "
           "\"async_done_pageable_ms\": %.3f, \"async_call_pinned_ms\": %.3f, \"async_done_pinned_ms\": %.3f, "
           "\"both_threads_pageable_h2d_GBps\": %.2f, \"both_threads_pageable_d2h_GBps\": %.2f, "
           "\"both_threads_pinned_h2d_GBps\": %.2f, \"both_threads_pinned_d2h_GBps\": %.2f, "
           "\"bidir_async_pinned_GBps_each\": %.2f, \"host_memcpy_1t_GBps\": %.2f, \"host_memcpy_8t_GBps\": %.2f, "
           "\"d2h_sync8MB_pageable_GBps\": %.2f, \"d2h_sync8MB_pinned_GBps\": %.2f, "
           "\"d2h_async_2streams_pinned_GBps\": %.2f, \"d2h_kernel_zero_copy_GBps\": %.2f, "
           "\"h2d_kernel_zero_copy_GBps\": %.2f}\n",
           nb, chunk, h2d_pg, h2d_pin, d2h_pg, d2h_pin, call_pg * 1e3, done_pg * 1e3, call_pin * 1e3,
           done_pin * 1e3, bp.first, bp.second, bn.first, bn.second, bidir_async, hc1, hc8, d2h_sync_pg, d2h_sync_pin,
           d2h_2s, d2h_kernel, h2d_kernel);
    return 0;
}
