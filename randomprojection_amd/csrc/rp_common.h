// rp_common.h — host-side helpers shared by librp's translation units (error plumbing, device
// buffers, dtype codes). Internal; the public interface is include/rp.h.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>
#include <thread>

#include "../../include/rp.h"

namespace rpd {

// ------------------------------------------------------------------------------------------
// error plumbing
inline thread_local std::string g_err;

inline int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(RP_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),     \
                        __FILE__, __LINE__);                                                   \
    } while (0)


struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int device = -1;
    ~DevBuf() { release(); }
    void release() {
        if (p) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(device);
            (void)hipFree(p);
            (void)hipSetDevice(cur);
        }
        p = nullptr;
        bytes = 0;
    }
    int ensure(size_t n, int dev) {
        if (n <= bytes && p) return RP_OK;
        release();
        device = dev;
        size_t want = std::max<size_t>(n, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(RP_ERR_NOMEM, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        }
        bytes = want;
        return RP_OK;
    }
    // for buffers resized per chunk of a stream: 1/8 headroom, so sizes that drift up do not
    // reallocate every chunk (hipFree / hipMalloc synchronise the whole device)
    int grow(size_t n, int dev) { return n <= bytes && p ? RP_OK : ensure(n + n / 8, dev); }
};


// Waits of the streaming pipelines' threads: poll instead of hipStreamSynchronize /
// hipEventSynchronize, which measured as serialising the other threads' HIP calls (a chunk's upload
// started only once the compute stream drained: uploads and kernels did not overlap)
inline hipError_t poll_event(hipEvent_t e) {
    for (;;) {
        const hipError_t r = hipEventQuery(e);
        if (r != hipErrorNotReady) return r;
        std::this_thread::yield();
    }
}
inline hipError_t poll_stream(hipStream_t st) {
    hipEvent_t e = nullptr;
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (r != hipSuccess) return r;
    r = hipEventRecord(e, st);
    if (r == hipSuccess) r = poll_event(e);
    (void)hipEventDestroy(e);
    return r;
}

inline int dtype_size(int t) {
    switch (t) {
        case RP_I32: case RP_F32: return 4;
        case RP_I64: case RP_F64: return 8;
        default: return 0;
    }
}

template <typename I>
inline int64_t idx_at(const void* a, int64_t i) { return (int64_t)((const I*)a)[i]; }
inline int64_t ptr_at(const void* a, int t, int64_t i) {
    return t == RP_I64 ? idx_at<int64_t>(a, i) : idx_at<int32_t>(a, i);
}
inline double val_at(const void* a, int t, int64_t i) {
    return t == RP_F64 ? ((const double*)a)[i] : (double)((const float*)a)[i];
}


// inclusive prefix sum of n int64 values in place on `st` (defined in rp_spgemm.hip)
int inclusive_scan_i64(int64_t* a, int64_t n, hipStream_t st, DevBuf& tmp, int device);

// libsvm parse (rp_libsvm.hip) with caller-kept scratch buffers, so a chunked pipeline allocates
// once (hipFree of a per-call buffer would synchronise the device and stall the other streams).
// Same contract as rp_libsvm_parse_device, on stream st.
struct LibsvmScratch {
    DevBuf counts, tmp, nl, keep, items, errb, slow;
    // the line structure of the last text counted into this scratch (newline positions, kept-line
    // and item prefix sums): a call with reuse_counts parses that same text without counting again
    bool counted = false;
    int64_t n_nl = 0, n_lines = 0, rows = 0, total = 0, bytes = -1;
};
int libsvm_parse(LibsvmScratch& s, int device, const char* text, int64_t n_bytes, int64_t num_features,
                 double* labels, void* indptr, int32_t indptr_type, int32_t* indices, float* data, int64_t cap_rows,
                 int64_t cap_nnz, hipStream_t st, int64_t* n_rows, int64_t* nnz, int64_t* err_line,
                 bool reuse_counts = false);

}  // namespace rpd
