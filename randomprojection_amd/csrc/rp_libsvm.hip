// rp_libsvm.hip — libsvm text -> CSR on the MI355X.
//
// Reference: spark.read.format("libsvm").load(DATA_DIR, numFeatures=N_FEATURES)
// (code/clustermode/randomProjection.py:71, code/localmode/randomProjection.py:92-96), i.e. Spark's
// MLUtils.parseLibSVMRecord (Scala, not in the container; restated from its published source):
//   * lines are trimmed; empty lines and lines starting with '#' are skipped;
//   * items = line.split(' ') (single spaces; empty items after the label are dropped);
//   * label = items(0).toDouble;
//   * each item "i:v" -> index = i.toInt - 1, value = v.toDouble (extra ":x" parts are ignored,
//     a missing value is an error); indices must be strictly ascending (so 1-based: "0:v" fails)
//     and < numFeatures.
// Values are parsed as doubles and stored as float32, which is what the partition function does
// next (features.values.astype(np.float32), clustermode/randomProjection.py:38). Labels stay f64.
//
// Kernels: newline count/mark per 4 KiB block (16 B per lane loads), one thread per line for
// tokenising/counting and for parsing (numbers by Clinger's exact fast path: <= 15 significant
// digits and |exp10| <= 22, plus NaN/Infinity). A literal outside that path is reported, never
// guessed (error code 7).
#include "rp_common.h"

#include <vector>

using namespace rpd;

namespace {

constexpr int kLB = 256;              // threads per block
constexpr int kBytesPerThread = 16;
constexpr int kBytesPerBlock = kLB * kBytesPerThread;

enum : int {
    E_LABEL = 1, E_INDEX = 2, E_NOVALUE = 3, E_VALUE = 4, E_ORDER = 5, E_RANGE = 6, E_LITERAL = 7
};

__device__ __forceinline__ bool is_ws(unsigned char c) { return c <= ' '; }  // Java String.trim

__global__ void nl_count_kernel(const unsigned char* __restrict__ t, int64_t n, int64_t* __restrict__ counts) {
    __shared__ int64_t s[kLB / 64];
    const int64_t base = (int64_t)blockIdx.x * kBytesPerBlock + (int64_t)threadIdx.x * kBytesPerThread;
    int c = 0;
    if (base + kBytesPerThread <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(t + base);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int b = 0; b < 4; ++b) c += ((w[q] >> (8 * b)) & 0xff) == '\n';
    } else {
        for (int64_t i = base; i < n && i < base + kBytesPerThread; ++i) c += t[i] == '\n';
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t tot = 0;
        for (int i = 0; i < kLB / 64; ++i) tot += s[i];
        counts[blockIdx.x] = tot;
    }
}

// positions of every '\n', in order: block offset (scanned counts) + in-block exclusive prefix
__global__ void nl_mark_kernel(const unsigned char* __restrict__ t, int64_t n,
                               const int64_t* __restrict__ block_incl, int64_t* __restrict__ nl_pos) {
    __shared__ int s_w[kLB / 64];
    const int64_t base = (int64_t)blockIdx.x * kBytesPerBlock + (int64_t)threadIdx.x * kBytesPerThread;
    unsigned char b[kBytesPerThread];
    int c = 0;
#pragma unroll
    for (int i = 0; i < kBytesPerThread; ++i) {
        b[i] = (base + i < n) ? t[base + i] : 0;
        c += b[i] == '\n';
    }
    // block exclusive scan of c
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int inc = c;
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    int off = 0;
    for (int i = 0; i < w; ++i) off += s_w[i];
    int64_t pos = (blockIdx.x ? block_incl[blockIdx.x - 1] : 0) + off + inc - c;
#pragma unroll
    for (int i = 0; i < kBytesPerThread; ++i)
        if (b[i] == '\n') nl_pos[pos++] = base + i;
}

__device__ __forceinline__ void line_span(const int64_t* __restrict__ nl_pos, int64_t n_nl, int64_t n,
                                          int64_t i, int64_t& s, int64_t& e) {
    s = i == 0 ? 0 : nl_pos[i - 1] + 1;
    e = i < n_nl ? nl_pos[i] : n;
}

// per line: kept (not blank, not a comment) and number of feature items
__global__ void line_count_kernel(const unsigned char* __restrict__ t, int64_t n,
                                  const int64_t* __restrict__ nl_pos, int64_t n_nl, int64_t n_lines,
                                  int64_t* __restrict__ keep, int64_t* __restrict__ items) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_lines;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t s, e;
        line_span(nl_pos, n_nl, n, i, s, e);
        while (s < e && is_ws(t[s])) ++s;
        while (e > s && is_ws(t[e - 1])) --e;
        const bool k = s < e && t[s] != '#';
        int64_t tokens = 0;
        if (k) {
            bool in_tok = false;
            for (int64_t q = s; q < e; ++q) {
                const bool sp = t[q] == ' ';
                if (!sp && !in_tok) ++tokens;
                in_tok = !sp;
            }
        }
        keep[i + 1] = k ? 1 : 0;
        // the label is the first split item even when it is empty (line starting with ' ' cannot
        // happen after trim); feature items = non-empty tokens after it
        items[i + 1] = k ? (tokens > 0 ? tokens - 1 : 0) : 0;
    }
}

// Java Double.parseDouble subset: [+-]? (digits [. digits?] | . digits) ([eE] [+-]? digits)?,
// NaN, Infinity. Exact (correctly rounded) via Clinger's fast path; *ok = 0 for a syntax error,
// 2 for a valid literal outside the exact path.
__device__ double parse_double(const unsigned char* p, const unsigned char* end, int* ok) {
    *ok = 1;
    bool neg = false;
    if (p < end && (*p == '+' || *p == '-')) {
        neg = *p == '-';
        ++p;
    }
    if (end - p == 3 && p[0] == 'N' && p[1] == 'a' && p[2] == 'N') return __longlong_as_double(0x7ff8000000000000ll);
    if (end - p == 8 && p[0] == 'I' && p[1] == 'n' && p[2] == 'f' && p[3] == 'i' && p[4] == 'n' &&
        p[5] == 'i' && p[6] == 't' && p[7] == 'y')
        return neg ? -__longlong_as_double(0x7ff0000000000000ll) : __longlong_as_double(0x7ff0000000000000ll);
    uint64_t mant = 0;
    int sig = 0, exp10 = 0, nd = 0;
    bool lost = false;
    while (p < end && *p >= '0' && *p <= '9') {
        const int d = *p - '0';
        if (sig > 0 || d != 0) {
            if (sig < 19) { mant = mant * 10 + d; ++sig; } else { ++exp10; lost |= d != 0; }
        }
        ++nd;
        ++p;
    }
    if (p < end && *p == '.') {
        ++p;
        while (p < end && *p >= '0' && *p <= '9') {
            const int d = *p - '0';
            if (sig > 0 || d != 0) {
                if (sig < 19) { mant = mant * 10 + d; ++sig; --exp10; } else { lost |= d != 0; }
            } else {
                --exp10;
            }
            ++nd;
            ++p;
        }
    }
    if (nd == 0) { *ok = 0; return 0.0; }
    if (p < end && (*p == 'e' || *p == 'E')) {
        ++p;
        bool eneg = false;
        if (p < end && (*p == '+' || *p == '-')) { eneg = *p == '-'; ++p; }
        if (p >= end || *p < '0' || *p > '9') { *ok = 0; return 0.0; }
        int ev = 0;
        while (p < end && *p >= '0' && *p <= '9') { ev = ev < 100000 ? ev * 10 + (*p - '0') : ev; ++p; }
        exp10 += eneg ? -ev : ev;
    }
    if (p != end) {  // trailing characters: type suffix [fFdD] is valid Java but outside this path
        *ok = (end - p == 1 && (*p == 'f' || *p == 'F' || *p == 'd' || *p == 'D')) ? 2 : 0;
        return 0.0;
    }
    if (mant == 0) return neg ? -0.0 : 0.0;
    while (mant % 10 == 0) {  // 1e21 written out in full is still exact
        mant /= 10;
        ++exp10;
    }
    // Clinger's extended fast path: move surplus powers of ten into the mantissa while it stays exact
    while (exp10 > 22 && mant <= (1ull << 53) / 10) {
        mant *= 10;
        --exp10;
    }
    if (lost || mant > (1ull << 53) || exp10 < -22 || exp10 > 22) { *ok = 2; return 0.0; }
    const double pw[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                           1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    double v = (double)mant;  // exact: mant <= 2^53
    v = exp10 >= 0 ? __dmul_rn(v, pw[exp10]) : __ddiv_rn(v, pw[-exp10]);
    return neg ? -v : v;
}

// Java Integer.parseInt: [+-]? digits, int32 range
__device__ bool parse_int(const unsigned char* p, const unsigned char* end, int64_t* out) {
    bool neg = false;
    if (p < end && (*p == '+' || *p == '-')) { neg = *p == '-'; ++p; }
    if (p >= end) return false;
    int64_t v = 0;
    for (; p < end; ++p) {
        if (*p < '0' || *p > '9') return false;
        v = v * 10 + (*p - '0');
        if (v > 2147483648ll) return false;
    }
    v = neg ? -v : v;
    if (v > 2147483647ll || v < -2147483648ll) return false;
    *out = v;
    return true;
}

template <typename IP>
__global__ void line_parse_kernel(const unsigned char* __restrict__ t, int64_t n,
                                  const int64_t* __restrict__ nl_pos, int64_t n_nl, int64_t n_lines,
                                  const int64_t* __restrict__ row_of, const int64_t* __restrict__ off_of,
                                  int64_t num_features, double* __restrict__ labels, IP* __restrict__ indptr,
                                  int32_t* __restrict__ indices, float* __restrict__ data,
                                  unsigned long long* __restrict__ err) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_lines;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (row_of[i + 1] == row_of[i]) continue;  // blank or comment line
        const int64_t row = row_of[i];
        int64_t out = off_of[i];
        int64_t s, e;
        line_span(nl_pos, n_nl, n, i, s, e);
        while (s < e && is_ws(t[s])) ++s;
        while (e > s && is_ws(t[e - 1])) --e;
        int code = 0;
        // label: first split(' ') item
        int64_t q = s;
        while (q < e && t[q] != ' ') ++q;
        {
            // Double.parseDouble trims the item itself
            int64_t a = s, b = q;
            while (a < b && is_ws(t[a])) ++a;
            while (b > a && is_ws(t[b - 1])) --b;
            int ok;
            const double lab = parse_double(t + a, t + b, &ok);
            if (ok != 1) code = ok == 2 ? E_LITERAL : E_LABEL;
            labels[row] = lab;
        }
        indptr[row] = (IP)out;
        int64_t prev = -1;
        while (code == 0 && q < e) {
            while (q < e && t[q] == ' ') ++q;
            if (q >= e) break;
            int64_t a = q;
            while (q < e && t[q] != ' ') ++q;
            // item [a, q): split(':') -> parts[0] index, parts[1] value (further parts ignored)
            int64_t c1 = a;
            while (c1 < q && t[c1] != ':') ++c1;
            int64_t c2 = c1 < q ? c1 + 1 : q;
            while (c2 < q && t[c2] != ':') ++c2;
            if (c1 >= q || c2 == c1 + 1) { code = E_NOVALUE; break; }
            int64_t idx;
            if (!parse_int(t + a, t + c1, &idx)) { code = E_INDEX; break; }
            int64_t va = c1 + 1, vb = c2;
            while (va < vb && is_ws(t[va])) ++va;
            while (vb > va && is_ws(t[vb - 1])) --vb;
            int ok;
            const double v = parse_double(t + va, t + vb, &ok);
            if (ok != 1) { code = ok == 2 ? E_LITERAL : E_VALUE; break; }
            const int64_t j = idx - 1;
            if (j <= prev) { code = E_ORDER; break; }
            if (j >= num_features) { code = E_RANGE; break; }
            prev = j;
            indices[out] = (int32_t)j;
            data[out] = (float)v;
            ++out;
        }
        if (code) atomicMin(err, ((unsigned long long)i << 8) | (unsigned long long)code);
    }
}

const char* reason(int c) {
    switch (c) {
        case E_LABEL: return "label is not a number";
        case E_INDEX: return "feature index is not an int";
        case E_NOVALUE: return "item without ':value'";
        case E_VALUE: return "feature value is not a number";
        case E_ORDER: return "indices should be one-based and in ascending order";
        case E_RANGE: return "feature index >= numFeatures";
        case E_LITERAL: return "numeric literal outside the exact GPU parser (hex, type suffix, >15 digits or |exp| > 22)";
        default: return "parse error";
    }
}

}  // namespace

extern "C" int rp_libsvm_parse_device(int device, const char* text, int64_t n_bytes, int64_t num_features,
                                      double* labels, void* indptr, int32_t indptr_type, int32_t* indices,
                                      float* data, int64_t cap_rows, int64_t cap_nnz, void* stream,
                                      int64_t* n_rows, int64_t* nnz, int64_t* err_line) {
    if (!n_rows || !nnz || n_bytes < 0 || (n_bytes > 0 && !text)) return fail(RP_ERR_INVALID, "bad argument");
    if (indptr && indptr_type != RP_I32 && indptr_type != RP_I64) return fail(RP_ERR_INVALID, "bad indptr type");
    if (err_line) *err_line = -1;
    HIP_TRY(hipSetDevice(device));
    hipStream_t st = (hipStream_t)stream;
    const unsigned char* t = (const unsigned char*)text;
    if (((uintptr_t)t & 15) != 0) return fail(RP_ERR_INVALID, "text must be 16-byte aligned");
    const int64_t nblk = std::max<int64_t>((n_bytes + kBytesPerBlock - 1) / kBytesPerBlock, 1);
    DevBuf counts, tmp, nl, keep, items, errb;
    int rc;
    if ((rc = counts.ensure(8 * (size_t)nblk, device))) return rc;
    hipLaunchKernelGGL(nl_count_kernel, dim3((unsigned)nblk), dim3(kLB), 0, st, t, n_bytes, (int64_t*)counts.p);
    HIP_TRY(hipGetLastError());
    if ((rc = inclusive_scan_i64((int64_t*)counts.p, nblk, st, tmp, device))) return rc;
    int64_t n_nl = 0;
    HIP_TRY(hipMemcpyAsync(&n_nl, (int64_t*)counts.p + nblk - 1, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    unsigned char last = '\n';
    if (n_bytes > 0) {
        HIP_TRY(hipMemcpyAsync(&last, t + n_bytes - 1, 1, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    const int64_t n_lines = n_nl + (last != '\n' ? 1 : 0);
    if ((rc = nl.ensure(8 * (size_t)std::max<int64_t>(n_nl, 1), device))) return rc;
    if (n_nl > 0) {
        hipLaunchKernelGGL(nl_mark_kernel, dim3((unsigned)nblk), dim3(kLB), 0, st, t, n_bytes,
                           (const int64_t*)counts.p, (int64_t*)nl.p);
        HIP_TRY(hipGetLastError());
    }
    if ((rc = keep.ensure(8 * (size_t)(n_lines + 1), device)) || (rc = items.ensure(8 * (size_t)(n_lines + 1), device)) ||
        (rc = errb.ensure(8, device)))
        return rc;
    HIP_TRY(hipMemsetAsync(keep.p, 0, 8, st));
    HIP_TRY(hipMemsetAsync(items.p, 0, 8, st));
    HIP_TRY(hipMemsetAsync(errb.p, 0xff, 8, st));
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>((n_lines + 255) / 256, 1), 65536);
    if (n_lines > 0) {
        hipLaunchKernelGGL(line_count_kernel, dim3(grid), dim3(256), 0, st, t, n_bytes, (const int64_t*)nl.p, n_nl,
                           n_lines, (int64_t*)keep.p, (int64_t*)items.p);
        HIP_TRY(hipGetLastError());
        if ((rc = inclusive_scan_i64((int64_t*)keep.p + 1, n_lines, st, tmp, device))) return rc;
        if ((rc = inclusive_scan_i64((int64_t*)items.p + 1, n_lines, st, tmp, device))) return rc;
    }
    int64_t rows = 0, total = 0;
    HIP_TRY(hipMemcpyAsync(&rows, (int64_t*)keep.p + n_lines, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&total, (int64_t*)items.p + n_lines, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *n_rows = rows;
    *nnz = total;  // upper bound until parsed: items counted; every parsed item is stored
    if (!indices) return RP_OK;
    if (!labels || !indptr || !data) return fail(RP_ERR_INVALID, "NULL output buffer");
    if (rows > cap_rows || total > cap_nnz)
        return fail(RP_ERR_CAPACITY, "need %lld rows / %lld entries", (long long)rows, (long long)total);
    if (indptr_type == RP_I32 && total >= ((int64_t)1 << 31))
        return fail(RP_ERR_UNSUPPORTED, "nnz %lld needs int64 indptr", (long long)total);
    if (n_lines > 0) {
        if (indptr_type == RP_I64)
            hipLaunchKernelGGL((line_parse_kernel<int64_t>), dim3(grid), dim3(256), 0, st, t, n_bytes,
                               (const int64_t*)nl.p, n_nl, n_lines, (const int64_t*)keep.p, (const int64_t*)items.p,
                               num_features, labels, (int64_t*)indptr, indices, data, (unsigned long long*)errb.p);
        else
            hipLaunchKernelGGL((line_parse_kernel<int32_t>), dim3(grid), dim3(256), 0, st, t, n_bytes,
                               (const int64_t*)nl.p, n_nl, n_lines, (const int64_t*)keep.p, (const int64_t*)items.p,
                               num_features, labels, (int32_t*)indptr, indices, data, (unsigned long long*)errb.p);
        HIP_TRY(hipGetLastError());
    }
    // indptr[rows] = total
    if (indptr_type == RP_I64)
        HIP_TRY(hipMemcpyAsync((int64_t*)indptr + rows, &total, 8, hipMemcpyHostToDevice, st));
    else {
        const int32_t t32 = (int32_t)total;
        HIP_TRY(hipMemcpyAsync((int32_t*)indptr + rows, &t32, 4, hipMemcpyHostToDevice, st));
    }
    unsigned long long e = 0;
    HIP_TRY(hipMemcpyAsync(&e, errb.p, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (e != ~0ull) {
        if (err_line) *err_line = (int64_t)(e >> 8);
        return fail(RP_ERR_INVALID, "libsvm line %lld: %s", (long long)(e >> 8), reason((int)(e & 0xff)));
    }
    return RP_OK;
}
