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
// counting items (16-byte words, SWAR space masks), and a workgroup-cooperative parser (lines staged
// in LDS, one thread per token; coop_parse_kernel). Every literal Double.parseDouble accepts converts correctly
// rounded: Clinger's fast path, Eisel-Lemire for any exponent, hex literals, and an exact
// decimal-shifting slow path (slow_line_kernel) for the rare long literals the first two cannot
// settle.
#include "rp_common.h"
#include "rp_pow5.h"

#include <vector>

using namespace rpd;

namespace {

constexpr int kLB = 256;              // threads per block
constexpr int kBytesPerThread = 16;
constexpr int kBytesPerBlock = kLB * kBytesPerThread;

enum : int {
    E_LABEL = 1, E_INDEX = 2, E_NOVALUE = 3, E_VALUE = 4, E_ORDER = 5, E_RANGE = 6
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

// bit j set where byte j of the 4-byte word w is ' ' (SWAR zero-byte test on w ^ 0x20202020)
__device__ __forceinline__ uint32_t space_bits4(uint32_t w) {
    const uint32_t m = w ^ 0x20202020u;
    const uint32_t zb = ~(((m & 0x7f7f7f7fu) + 0x7f7f7f7fu) | m) & 0x80808080u;
    return ((zb >> 7) & 1u) | ((zb >> 14) & 2u) | ((zb >> 21) & 4u) | ((zb >> 28) & 8u);
}

// per line: kept (not blank, not a comment) and number of feature items. One thread per line; the
// line's bytes are read as aligned 16-byte words (the text is 16-byte aligned, so a word holding a
// byte of the text never crosses its allocation's end) and its tokens counted 16 bytes at a time:
// a token starts at a non-space byte whose predecessor is a space or the line's (trimmed) start.
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
            uint32_t carry = 1u;  // "the byte before is a space": true at the line's start
            for (int64_t a = s & ~int64_t(15); a < e; a += 16) {
                const uint4 v = *reinterpret_cast<const uint4*>(t + a);
                uint32_t sp = space_bits4(v.x) | (space_bits4(v.y) << 4) | (space_bits4(v.z) << 8) |
                              (space_bits4(v.w) << 12);
                const int lo = a < s ? (int)(s - a) : 0, hi = e < a + 16 ? (int)(e - a) : 16;
                const uint32_t valid = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
                sp |= (1u << lo) - 1u;  // bytes before the line's start count as spaces
                const uint32_t starts = valid & ~sp & ((sp << 1) | carry);
                tokens += __builtin_popcount(starts);
                carry = (sp >> 15) & 1u;
            }
        }
        keep[i + 1] = k ? 1 : 0;
        // the label is the first split item even when it is empty (line starting with ' ' cannot
        // happen after trim); feature items = non-empty tokens after it
        items[i + 1] = k ? (tokens > 0 ? tokens - 1 : 0) : 0;
    }
}

// ---- decimal/hex text -> binary64, correctly rounded (Java Double.parseDouble, every literal):
//   [+-]? (NaN | Infinity | digits [. digits?] | . digits) ([eE] [+-]? digits)? [fFdD]?
//   [+-]? 0[xX] (hexdigits [.]? | hexdigits? . hexdigits) [pP] [+-]? digits [fFdD]?
// Decimal literals with <= 19 significant digits: the Eisel-Lemire algorithm (Lemire 2021), exact
// with no fallback for such mantissas (Mushtak & Lemire 2023). More digits: the first 19 give a
// truncated mantissa w; if w and w + 1 round to the same double it is the answer, else the line is
// handed to slow_line_kernel, which converts every digit exactly (decimal shifting, below).

// m * 2^e2 correctly rounded to binary64 (round to nearest even); sticky: nonzero bits below m
__device__ uint64_t round_bin64(uint64_t m, int e2, bool sticky) {
    if (m == 0) return 0;
    const int lz = __clzll(m);
    m <<= lz;
    e2 -= lz;
    const int E = e2 + 63;  // exponent of the leading bit
    if (E > 1023) return 0x7ff0000000000000ull;
    const int shift = E >= -1022 ? 11 : 11 + (-1022 - E);
    if (shift > 64) return 0;
    const uint64_t kept = shift == 64 ? 0 : m >> shift;
    const uint64_t rem = shift == 64 ? m : m << (64 - shift);  // dropped bits, top-aligned
    const bool half = rem >> 63, rest = (rem << 1) != 0 || sticky;
    uint64_t k = kept + ((half && (rest || (kept & 1))) ? 1 : 0);
    if (E >= -1022) {
        int Eo = E;
        if (k == (1ull << 53)) {
            k >>= 1;
            ++Eo;
            if (Eo > 1023) return 0x7ff0000000000000ull;
        }
        return ((uint64_t)(Eo + 1023) << 52) | (k & ((1ull << 52) - 1));
    }
    return k;  // subnormal (k == 2^52: the smallest normal, exponent field 1)
}

// Eisel-Lemire: w * 10^q (w != 0 exact) -> binary64 bits, no sign
__device__ uint64_t eisel_lemire(int q, uint64_t w) {
    if (q < kPow5Min) return 0;
    if (q > kPow5Max) return 0x7ff0000000000000ull;
    const int lz = __clzll(w);
    w <<= lz;
    const int idx = 2 * (q - kPow5Min);
    uint64_t hi = __umul64hi(w, kPow5[idx]), lo = w * kPow5[idx];
    constexpr uint64_t kPrecMask = 0xFFFFFFFFFFFFFFFFull >> 55;
    if ((hi & kPrecMask) == kPrecMask) {
        const uint64_t hi2 = __umul64hi(w, kPow5[idx + 1]);
        lo += hi2;
        if (hi2 > lo) ++hi;
    }
    const int upper = (int)(hi >> 63);
    const int shift = upper + 64 - 52 - 3;
    uint64_t mant = hi >> shift;
    int p2 = (int)((((152170 + 65536) * (int64_t)q) >> 16) + 63) + upper - lz + 1023;
    if (p2 <= 0) {  // subnormal
        if (-p2 + 1 >= 64) return 0;
        mant >>= -p2 + 1;
        mant += mant & 1;
        mant >>= 1;
        return mant;  // mant == 2^52: the smallest normal
    }
    if (lo <= 1 && q >= -4 && q <= 23 && (mant & 3) == 1 && (mant << shift) == hi) mant &= ~1ull;
    mant += mant & 1;
    mant >>= 1;
    if (mant >= (2ull << 52)) {
        mant = 1ull << 52;
        ++p2;
    }
    if (p2 >= 0x7ff) return 0x7ff0000000000000ull;
    return ((uint64_t)p2 << 52) | (mant & ((1ull << 52) - 1));
}

__device__ __forceinline__ int hexval(unsigned char c) {
    return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
}

// hex literal after "0x": value bits (no sign); *ok = 0 on a syntax error
__device__ uint64_t parse_hex(const unsigned char* p, const unsigned char* end, int* ok) {
    uint64_t m = 0;
    int e2 = 0, nd = 0;
    bool sticky = false, seen_nz = false;
    auto digit = [&](int v, bool frac) {
        ++nd;
        if (!seen_nz && v == 0) {
            if (frac) e2 -= 4;
            return;
        }
        seen_nz = true;
        if (m >> 60) {  // 64 bits kept: the rest only rounds
            sticky |= v != 0;
            if (!frac) e2 += 4;
        } else {
            m = (m << 4) | (uint64_t)v;
            if (frac) e2 -= 4;
        }
    };
    while (p < end && hexval(*p) >= 0) digit(hexval(*p++), false);
    if (p < end && *p == '.') {
        ++p;
        while (p < end && hexval(*p) >= 0) digit(hexval(*p++), true);
    }
    if (nd == 0 || p >= end || (*p != 'p' && *p != 'P')) { *ok = 0; return 0; }
    ++p;
    bool eneg = false;
    if (p < end && (*p == '+' || *p == '-')) { eneg = *p == '-'; ++p; }
    if (p >= end || *p < '0' || *p > '9') { *ok = 0; return 0; }
    int ev = 0;
    while (p < end && *p >= '0' && *p <= '9') { ev = ev < 100000 ? ev * 10 + (*p - '0') : ev; ++p; }
    if (p < end && (*p == 'f' || *p == 'F' || *p == 'd' || *p == 'D')) ++p;
    if (p != end) { *ok = 0; return 0; }
    *ok = 1;
    if (m == 0) return 0;
    const int64_t e = (int64_t)e2 + (eneg ? -ev : ev);
    return round_bin64(m, (int)std::max<int64_t>(std::min<int64_t>(e, 4000), -4000), sticky);
}

// *ok: 1 parsed, 0 syntax error, 3 valid but needs the exact slow path (slow_line_kernel)
__device__ double parse_double(const unsigned char* p, const unsigned char* end, int* ok) {
    *ok = 1;
    bool neg = false;
    if (p < end && (*p == '+' || *p == '-')) {
        neg = *p == '-';
        ++p;
    }
    const uint64_t sgn = neg ? 0x8000000000000000ull : 0ull;
    if (end - p == 3 && p[0] == 'N' && p[1] == 'a' && p[2] == 'N') return __longlong_as_double(0x7ff8000000000000ll);
    if (end - p == 8 && p[0] == 'I' && p[1] == 'n' && p[2] == 'f' && p[3] == 'i' && p[4] == 'n' &&
        p[5] == 'i' && p[6] == 't' && p[7] == 'y')
        return __longlong_as_double((long long)(sgn | 0x7ff0000000000000ull));
    if (end - p >= 2 && p[0] == '0' && (p[1] == 'x' || p[1] == 'X')) {
        const uint64_t b = parse_hex(p + 2, end, ok);
        return __longlong_as_double((long long)(sgn | b));
    }
    uint64_t mant = 0;
    int sig = 0, nd = 0;
    int64_t exp10 = 0;
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
        int64_t ev = 0;
        while (p < end && *p >= '0' && *p <= '9') { ev = ev < 100000 ? ev * 10 + (*p - '0') : ev; ++p; }
        exp10 += eneg ? -ev : ev;
    }
    if (p < end && (*p == 'f' || *p == 'F' || *p == 'd' || *p == 'D')) ++p;  // Java type suffix
    if (p != end) { *ok = 0; return 0.0; }
    if (mant == 0) return __longlong_as_double((long long)sgn);
    const int q = (int)std::max<int64_t>(std::min<int64_t>(exp10, 100000), -100000);
    uint64_t b;
    if (!lost && mant <= (1ull << 53) && q >= -22 && q <= 22) {  // Clinger: one exact operation
        const double pw[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
        const double v = q >= 0 ? __dmul_rn((double)mant, pw[q]) : __ddiv_rn((double)mant, pw[-q]);
        b = (uint64_t)__double_as_longlong(v);
    } else {
        b = eisel_lemire(q, mant);
        if (lost && eisel_lemire(q, mant + 1) != b) {  // the dropped digits decide: exact path
            *ok = 3;
            return 0.0;
        }
    }
    return __longlong_as_double((long long)(sgn | b));
}

// ---- exact slow path: the literal as a decimal digit string (up to kDecDigits significant digits,
// `trunc` if nonzero digits were dropped), scaled by powers of two until it lies in [1/2, 1), then
// 53 bits extracted with round-half-even (the classic decimal-shifting conversion).
constexpr int kDecDigits = 800;
struct Dec {
    uint8_t d[kDecDigits + 24];
    int nd, dp;
    bool trunc;
};

__device__ void dec_trim(Dec& a) {
    while (a.nd > 0 && a.d[a.nd - 1] == 0) --a.nd;
    if (a.nd == 0) a.dp = 0;
}

__device__ void dec_rshift(Dec& a, int k) {  // a /= 2^k, k <= 60
    int r = 0, w = 0;
    uint64_t n = 0;
    for (; (n >> k) == 0; ++r) {
        if (r >= a.nd) {
            if (n == 0) { a.nd = 0; return; }
            while ((n >> k) == 0) { n *= 10; ++r; }
            break;
        }
        n = n * 10 + a.d[r];
    }
    a.dp -= r - 1;
    const uint64_t mask = (1ull << k) - 1;
    for (; r < a.nd; ++r) {
        const uint64_t c = a.d[r];
        const uint64_t dig = n >> k;
        n &= mask;
        a.d[w++] = (uint8_t)dig;
        n = n * 10 + c;
    }
    while (n > 0) {
        const uint64_t dig = n >> k;
        n &= mask;
        if (w < kDecDigits) a.d[w++] = (uint8_t)dig;
        else if (dig > 0) a.trunc = true;
        n *= 10;
    }
    a.nd = w;
    dec_trim(a);
}

__device__ void dec_lshift(Dec& a, int k) {  // a *= 2^k, k <= 60: at most 19 new leading digits
    constexpr int kGrow = 20;
    int w = a.nd + kGrow;
    uint64_t n = 0;
    for (int r = a.nd - 1; r >= 0; --r) {
        n += (uint64_t)a.d[r] << k;
        const uint64_t quo = n / 10, rem = n - 10 * quo;
        --w;
        a.d[w] = (uint8_t)rem;
        n = quo;
    }
    while (n > 0) {
        const uint64_t quo = n / 10, rem = n - 10 * quo;
        --w;
        a.d[w] = (uint8_t)rem;
        n = quo;
    }
    int nn = a.nd + kGrow - w;  // digits now in d[w, w + nn)
    for (int i = 0; i < nn; ++i) a.d[i] = a.d[w + i];
    a.dp += kGrow - w;
    if (nn > kDecDigits) {
        for (int i = kDecDigits; i < nn; ++i) a.trunc |= a.d[i] != 0;
        nn = kDecDigits;
    }
    a.nd = nn;
    dec_trim(a);
}

__device__ void dec_shift(Dec& a, int k) {
    if (a.nd == 0) return;
    while (k > 60) { dec_lshift(a, 60); k -= 60; }
    if (k > 0) dec_lshift(a, k);
    while (k < -60) { dec_rshift(a, 60); k += 60; }
    if (k < 0) dec_rshift(a, -k);
}

__device__ bool dec_round_up(const Dec& a, int nd) {
    if (nd < 0 || nd >= a.nd) return false;
    if (a.d[nd] == 5 && nd + 1 == a.nd) {  // exactly half-way (unless digits were dropped)
        if (a.trunc) return true;
        return nd > 0 && (a.d[nd - 1] & 1);
    }
    return a.d[nd] >= 5;
}

__device__ uint64_t dec_to_bits(Dec& a) {
    constexpr int kBias = -1023, kMant = 52;
    const int powtab[9] = {1, 3, 6, 9, 13, 16, 19, 23, 26};
    if (a.nd == 0 || a.dp < -330) return 0;
    if (a.dp > 310) return 0x7ff0000000000000ull;
    int exp = 0;
    while (a.dp > 0) {
        const int n = a.dp >= 9 ? 27 : powtab[a.dp];
        dec_shift(a, -n);
        exp += n;
    }
    while (a.dp < 0 || (a.dp == 0 && a.d[0] < 5)) {
        const int n = -a.dp >= 9 ? 27 : powtab[-a.dp];
        dec_shift(a, n);
        exp -= n;
    }
    --exp;  // [1/2, 1) -> [1, 2)
    if (exp < kBias + 1) {
        const int n = kBias + 1 - exp;
        dec_shift(a, -n);
        exp += n;
    }
    if (exp - kBias >= 0x7ff) return 0x7ff0000000000000ull;
    dec_shift(a, 1 + kMant);
    uint64_t mant = 0;
    {
        int i = 0;
        for (; i < a.dp && i < a.nd; ++i) mant = mant * 10 + a.d[i];
        for (; i < a.dp; ++i) mant *= 10;
        if (dec_round_up(a, a.dp)) ++mant;
    }
    if (mant == (2ull << kMant)) {
        mant >>= 1;
        ++exp;
        if (exp - kBias >= 0x7ff) return 0x7ff0000000000000ull;
    }
    if (!(mant & (1ull << kMant))) exp = kBias;
    return (mant & ((1ull << kMant) - 1)) | ((uint64_t)((exp - kBias) & 0x7ff) << kMant);
}

// the exact conversion of a decimal literal already validated by parse_double (ok == 3 there)
__device__ double parse_double_exact(const unsigned char* p, const unsigned char* end) {
    Dec a;
    a.nd = 0;
    a.dp = 0;
    a.trunc = false;
    bool neg = false;
    if (p < end && (*p == '+' || *p == '-')) { neg = *p == '-'; ++p; }
    bool saw_dot = false, saw_nz = false;
    int64_t dp = 0;
    for (; p < end; ++p) {
        const unsigned char c = *p;
        if (c == '.') { saw_dot = true; continue; }
        if (c < '0' || c > '9') break;
        if (!saw_nz && c == '0') {
            if (saw_dot) --dp;
            continue;
        }
        saw_nz = true;
        if (a.nd < kDecDigits) a.d[a.nd++] = (uint8_t)(c - '0');
        else a.trunc |= c != '0';
        if (!saw_dot) ++dp;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
        ++p;
        bool eneg = false;
        if (p < end && (*p == '+' || *p == '-')) { eneg = *p == '-'; ++p; }
        int64_t ev = 0;
        while (p < end && *p >= '0' && *p <= '9') { ev = ev < 100000 ? ev * 10 + (*p - '0') : ev; ++p; }
        dp += eneg ? -ev : ev;
    }
    a.dp = (int)std::max<int64_t>(std::min<int64_t>(dp, 100000), -100000);
    dec_trim(a);
    const uint64_t b = dec_to_bits(a);
    return __longlong_as_double((long long)((neg ? 0x8000000000000000ull : 0ull) | b));
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

// one line -> its row (label, indptr, entries). EXACT = false: a literal that needs the exact slow
// path (ok == 3) is left for slow_line_kernel (*slow = true); EXACT = true converts it here.
template <typename IP, bool EXACT>
__device__ int parse_line(const unsigned char* __restrict__ t, int64_t n, const int64_t* __restrict__ nl_pos,
                          int64_t n_nl, int64_t i, const int64_t* __restrict__ row_of,
                          const int64_t* __restrict__ off_of, int64_t num_features, double* __restrict__ labels,
                          IP* __restrict__ indptr, int32_t* __restrict__ indices, float* __restrict__ data,
                          bool* slow) {
    const int64_t row = row_of[i];
    int64_t out = off_of[i];
    int64_t s, e;
    line_span(nl_pos, n_nl, n, i, s, e);
    while (s < e && is_ws(t[s])) ++s;
    while (e > s && is_ws(t[e - 1])) --e;
    int code = 0;
    auto number = [&](int64_t a, int64_t b, int* ok) {
        double v = parse_double(t + a, t + b, ok);
        if (*ok == 3) {
            if (EXACT) {
                v = parse_double_exact(t + a, t + b);
                *ok = 1;
            } else {
                *slow = true;
                *ok = 1;  // placeholder; the exact kernel rewrites the whole line
            }
        }
        return v;
    };
    // label: first split(' ') item
    int64_t q = s;
    while (q < e && t[q] != ' ') ++q;
    {
        // Double.parseDouble trims the item itself
        int64_t a = s, b = q;
        while (a < b && is_ws(t[a])) ++a;
        while (b > a && is_ws(t[b - 1])) --b;
        int ok;
        const double lab = number(a, b, &ok);
        if (ok != 1) code = E_LABEL;
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
        const double v = number(va, vb, &ok);
        if (ok != 1) { code = E_VALUE; break; }
        const int64_t j = idx - 1;
        if (j <= prev) { code = E_ORDER; break; }
        if (j >= num_features) { code = E_RANGE; break; }
        prev = j;
        indices[out] = (int32_t)j;
        data[out] = (float)v;  // double -> float32 rounding, as features.values.astype(np.float32)
        ++out;
    }
    return code;
}

// error key of the first failure: line, then the failing item's rank in the line (0 = the label),
// then the code; the smallest key is what a sequential parse meets first
__device__ __forceinline__ unsigned long long err_key(int64_t line, uint32_t rank, int code) {
    return ((unsigned long long)line << 20) | ((unsigned long long)std::min<uint32_t>(rank, 4095u) << 8) |
           (unsigned long long)code;
}

// Workgroup-cooperative parse (the default). Workgroup b owns the lines that START in text bytes
// [b kPB, (b + 1) kPB) and stages them whole into LDS with 16-byte loads; token starts (a byte other
// than ' ' / '\n' after one of them) and newlines are counted per thread slice, block-scanned, and
// listed in LDS; then one thread per token parses it from LDS: the line's first token is its label,
// the others "index:value" items stored at off_of[line] + rank. Order and range checks read the
// neighbouring token's index after a barrier. A block whose window holds other control bytes
// (tab, CR), a token starting with '#' (comment lines), more than kWin bytes, kMaxTok tokens or
// kMaxLn lines parses its lines one thread per line from global memory instead (parse_line).
constexpr int kPB = 8192;             // text bytes per workgroup (two line-count blocks)
constexpr int kWin = 12288;           // staged window: the block's lines, whole
constexpr int kMaxTok = 2048, kMaxLn = 512;

template <typename IP>
__global__ void __launch_bounds__(kLB)
coop_parse_kernel(const unsigned char* __restrict__ t, int64_t n, const int64_t* __restrict__ counts,
                  const int64_t* __restrict__ nl_pos, int64_t n_nl, int64_t n_lines,
                  const int64_t* __restrict__ row_of, const int64_t* __restrict__ off_of, int64_t num_features,
                  double* __restrict__ labels, IP* __restrict__ indptr, int32_t* __restrict__ indices,
                  float* __restrict__ data, unsigned long long* __restrict__ err,
                  unsigned long long* __restrict__ n_slow, int64_t* __restrict__ slow_lines) {
    __shared__ __align__(16) unsigned char s_txt[kWin + 32];
    __shared__ uint16_t s_tok[kMaxTok], s_tln[kMaxTok];
    __shared__ int32_t s_j[kMaxTok];
    __shared__ uint8_t s_code[kMaxTok];
    __shared__ uint16_t s_lfirst[kMaxLn];
    __shared__ uint32_t s_lslow[kMaxLn];
    __shared__ uint32_t s_w[2][kLB / 64];
    __shared__ int s_bad;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t B0 = (int64_t)blockIdx.x * kPB, B1 = std::min<int64_t>(n, B0 + kPB);
    if (B0 >= n) return;
    auto nl_lt = [&](int64_t x) -> int64_t {  // newlines before byte x (x a multiple of 4096, or n)
        return x >= n ? n_nl : (x == 0 ? 0 : counts[x / kBytesPerBlock - 1]);
    };
    const int64_t i0 = B0 == 0 ? 0 : nl_lt(B0) - (t[B0 - 1] == '\n' ? 1 : 0) + 1;
    const int64_t i1 = std::min<int64_t>(n_lines, nl_lt(B1) - (t[B1 - 1] == '\n' ? 1 : 0) + 1);
    if (i0 >= i1) return;  // uniform
    const int64_t S = i0 == 0 ? 0 : nl_pos[i0 - 1] + 1;
    const int64_t E = i1 - 1 < n_nl ? nl_pos[i1 - 1] + 1 : n;
    const int64_t W64 = E - S;
    const int nlines = (int)(i1 - i0);
    auto fallback = [&]() {
        for (int64_t i = i0 + tid; i < i1; i += kLB) {
            if (row_of[i + 1] == row_of[i]) continue;  // blank or comment line
            bool slow = false;
            const int code = parse_line<IP, false>(t, n, nl_pos, n_nl, i, row_of, off_of, num_features, labels,
                                                   indptr, indices, data, &slow);
            if (code) atomicMin(err, err_key(i, 0, code));
            else if (slow) slow_lines[atomicAdd(n_slow, 1ull)] = i;
        }
    };
    if (W64 > kWin || nlines > kMaxLn) {  // uniform
        fallback();
        return;
    }
    const int W = (int)W64;
    const int64_t a0 = S & ~int64_t(15);
    const int o0 = (int)(S - a0);
    const int nw = (int)((((E + 15) & ~int64_t(15)) - a0) / 16);
    for (int w = tid; w < nw; w += kLB)
        *reinterpret_cast<uint4*>(s_txt + 16 * w) = *reinterpret_cast<const uint4*>(t + a0 + 16 * w);
    if (tid == 0) s_bad = 0;
    __syncthreads();
    const unsigned char* b = s_txt + o0;
    const int per = (W + kLB - 1) / kLB, p0 = std::min(W, tid * per), p1 = std::min(W, p0 + per);
    auto is_sep = [](unsigned char c) { return c == ' ' || c == '\n'; };
    uint32_t ntok = 0, nnl = 0;
    bool bad = false;
    {
        bool prev = p0 == 0 || is_sep(b[p0 - 1]);
        for (int p = p0; p < p1; ++p) {
            const unsigned char c = b[p];
            const bool sp = is_sep(c);
            bad |= c < ' ' && c != '\n';
            if (!sp && prev) {
                ++ntok;
                bad |= c == '#';
            }
            nnl += c == '\n';
            prev = sp;
        }
    }
    if (bad) s_bad = 1;
    // block exclusive scan of (tokens, newlines) over the thread slices, in text order
    uint32_t it = ntok, il = nnl;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t yt = __shfl_up(it, o, 64), yl = __shfl_up(il, o, 64);
        if (lane >= o) { it += yt; il += yl; }
    }
    if (lane == 63) { s_w[0][wv] = it; s_w[1][wv] = il; }
    __syncthreads();
    uint32_t tb = it - ntok, lb = il - nnl, T = 0;
#pragma unroll
    for (int q = 0; q < kLB / 64; ++q) {
        if (q < wv) { tb += s_w[0][q]; lb += s_w[1][q]; }
        T += s_w[0][q];
    }
    if (s_bad || T > (uint32_t)kMaxTok) {  // uniform
        fallback();
        return;
    }
    {
        bool prev = p0 == 0 || is_sep(b[p0 - 1]);
        uint32_t k = tb, L = lb;
        for (int p = p0; p < p1; ++p) {
            const unsigned char c = b[p];
            const bool sp = is_sep(c);
            if (!sp && prev) {
                s_tok[k] = (uint16_t)p;
                s_tln[k] = (uint16_t)L;
                ++k;
            }
            L += c == '\n';
            prev = sp;
        }
    }
    for (int L = tid; L < nlines; L += kLB) s_lslow[L] = 0u;
    __syncthreads();
    for (uint32_t k = tid; k < T; k += kLB)
        if (k == 0 || s_tln[k - 1] != s_tln[k]) s_lfirst[s_tln[k]] = (uint16_t)k;
    __syncthreads();
    // one thread per token
    for (uint32_t k = tid; k < T; k += kLB) {
        const int p = s_tok[k];
        int q = p;
        while (q < W && !is_sep(b[q])) ++q;
        const int L = s_tln[k];
        const int64_t i = i0 + L;
        const int64_t row = row_of[i];
        const uint32_t f = s_lfirst[L];
        int ok = 1;
        if (f == k) {  // the label
            const double lab = parse_double(b + p, b + q, &ok);
            labels[row] = lab;
            indptr[row] = (IP)off_of[i];
            if (ok == 3) atomicOr(&s_lslow[L], 1u);
            if (ok == 0) atomicMin(err, err_key(i, 0, E_LABEL));
            s_code[k] = 0;
            continue;
        }
        const int64_t out = off_of[i] + (k - f - 1);
        int c1 = p;
        while (c1 < q && b[c1] != ':') ++c1;
        int c2 = c1 < q ? c1 + 1 : q;
        while (c2 < q && b[c2] != ':') ++c2;
        int code = 0;
        int64_t idx = 0;
        if (c1 >= q || c2 == c1 + 1) {
            code = E_NOVALUE;
        } else if (!parse_int(b + p, b + c1, &idx)) {
            code = E_INDEX;
        } else {
            const double v = parse_double(b + c1 + 1, b + c2, &ok);
            if (ok == 0) {
                code = E_VALUE;
            } else {
                if (ok == 3) atomicOr(&s_lslow[L], 1u);
                const int64_t j = idx - 1;
                s_j[k] = (int32_t)std::max<int64_t>(std::min<int64_t>(j, INT32_MAX), -1);
                indices[out] = (int32_t)j;
                data[out] = (float)v;  // double -> float32 rounding, as features.values.astype(np.float32)
            }
        }
        s_code[k] = (uint8_t)code;
    }
    __syncthreads();
    // order (first) and range checks against the item before, errors keyed by (line, rank)
    for (uint32_t k = tid; k < T; k += kLB) {
        const int L = s_tln[k];
        const uint32_t f = s_lfirst[L];
        if (f == k) continue;
        int code = s_code[k];
        if (code == 0) {
            const int64_t j = s_j[k], prevj = k - 1 == f ? -1 : s_j[k - 1];
            if (j <= prevj) code = E_ORDER;
            else if (j >= num_features) code = E_RANGE;
        }
        if (code) atomicMin(err, err_key(i0 + L, k - f, code));
    }
    for (int L = tid; L < nlines; L += kLB)
        if (s_lslow[L]) slow_lines[atomicAdd(n_slow, 1ull)] = i0 + L;
}

// lines holding a literal the fast parser could not settle: parsed again, every literal exact
template <typename IP>
__global__ void slow_line_kernel(const unsigned char* __restrict__ t, int64_t n, const int64_t* __restrict__ nl_pos,
                                 int64_t n_nl, const int64_t* __restrict__ row_of, const int64_t* __restrict__ off_of,
                                 int64_t num_features, double* __restrict__ labels, IP* __restrict__ indptr,
                                 int32_t* __restrict__ indices, float* __restrict__ data,
                                 const unsigned long long* __restrict__ n_slow, const int64_t* __restrict__ slow_lines) {
    const unsigned long long ns = *n_slow;
    for (unsigned long long k = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; k < ns;
         k += (unsigned long long)gridDim.x * blockDim.x) {
        bool slow = false;
        (void)parse_line<IP, true>(t, n, nl_pos, n_nl, slow_lines[k], row_of, off_of, num_features, labels, indptr,
                                   indices, data, &slow);
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
        default: return "parse error";
    }
}

}  // namespace

int rpd::libsvm_parse(LibsvmScratch& sc, int device, const char* text, int64_t n_bytes, int64_t num_features,
                      double* labels, void* indptr, int32_t indptr_type, int32_t* indices, float* data,
                      int64_t cap_rows, int64_t cap_nnz, hipStream_t st, int64_t* n_rows, int64_t* nnz,
                      int64_t* err_line, bool reuse_counts) {
    if (!n_rows || !nnz || n_bytes < 0 || (n_bytes > 0 && !text)) return fail(RP_ERR_INVALID, "bad argument");
    if (indptr && indptr_type != RP_I32 && indptr_type != RP_I64) return fail(RP_ERR_INVALID, "bad indptr type");
    if (err_line) *err_line = -1;
    HIP_TRY(hipSetDevice(device));
    const unsigned char* t = (const unsigned char*)text;
    if (((uintptr_t)t & 15) != 0) return fail(RP_ERR_INVALID, "text must be 16-byte aligned");
    const int64_t nblk = std::max<int64_t>((n_bytes + kBytesPerBlock - 1) / kBytesPerBlock, 1);
    DevBuf &counts = sc.counts, &tmp = sc.tmp, &nl = sc.nl, &keep = sc.keep, &items = sc.items, &errb = sc.errb,
           &slow = sc.slow;
    int rc;
    int64_t n_nl = 0, n_lines = 0, rows = 0, total = 0;
    auto count = [&]() -> int {  // newline positions, kept lines, items per line (prefix sums)
        if ((rc = counts.grow(8 * (size_t)nblk, device))) return rc;
        hipLaunchKernelGGL(nl_count_kernel, dim3((unsigned)nblk), dim3(kLB), 0, st, t, n_bytes, (int64_t*)counts.p);
        HIP_TRY(hipGetLastError());
        if ((rc = inclusive_scan_i64((int64_t*)counts.p, nblk, st, tmp, device))) return rc;
        HIP_TRY(hipMemcpyAsync(&n_nl, (int64_t*)counts.p + nblk - 1, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(poll_stream(st));
        unsigned char last = '\n';
        if (n_bytes > 0) {
            HIP_TRY(hipMemcpyAsync(&last, t + n_bytes - 1, 1, hipMemcpyDeviceToHost, st));
            HIP_TRY(poll_stream(st));
        }
        n_lines = n_nl + (last != '\n' ? 1 : 0);
        if ((rc = nl.grow(8 * (size_t)std::max<int64_t>(n_nl, 1), device))) return rc;
        if (n_nl > 0) {
            hipLaunchKernelGGL(nl_mark_kernel, dim3((unsigned)nblk), dim3(kLB), 0, st, t, n_bytes,
                               (const int64_t*)counts.p, (int64_t*)nl.p);
            HIP_TRY(hipGetLastError());
        }
        if ((rc = keep.grow(8 * (size_t)(n_lines + 1), device)) || (rc = items.grow(8 * (size_t)(n_lines + 1), device)) ||
            (rc = errb.grow(16, device)))
            return rc;
        HIP_TRY(hipMemsetAsync(keep.p, 0, 8, st));
        HIP_TRY(hipMemsetAsync(items.p, 0, 8, st));
        HIP_TRY(hipMemsetAsync(errb.p, 0xff, 8, st));
        HIP_TRY(hipMemsetAsync((char*)errb.p + 8, 0, 8, st));  // lines for the exact slow path
        if (n_lines > 0) {
            const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>((n_lines + 255) / 256, 1), 65536);
            hipLaunchKernelGGL(line_count_kernel, dim3(grid), dim3(256), 0, st, t, n_bytes, (const int64_t*)nl.p, n_nl,
                               n_lines, (int64_t*)keep.p, (int64_t*)items.p);
            HIP_TRY(hipGetLastError());
            if ((rc = inclusive_scan_i64((int64_t*)keep.p + 1, n_lines, st, tmp, device))) return rc;
            if ((rc = inclusive_scan_i64((int64_t*)items.p + 1, n_lines, st, tmp, device))) return rc;
        }
        HIP_TRY(hipMemcpyAsync(&rows, (int64_t*)keep.p + n_lines, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&total, (int64_t*)items.p + n_lines, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(poll_stream(st));
        sc.counted = true;
        sc.n_nl = n_nl;
        sc.n_lines = n_lines;
        sc.rows = rows;
        sc.total = total;
        sc.bytes = n_bytes;
        return RP_OK;
    };
    if (reuse_counts && sc.counted && sc.bytes == n_bytes) {  // the same text, counted by the call before
        n_nl = sc.n_nl;
        n_lines = sc.n_lines;
        rows = sc.rows;
        total = sc.total;
    } else {
        sc.counted = false;
        if ((rc = count())) return rc;
    }
    *n_rows = rows;
    *nnz = total;  // upper bound until parsed: items counted; every parsed item is stored
    if (!indices) return RP_OK;
    sc.counted = false;
    if (!labels || !indptr || !data) return fail(RP_ERR_INVALID, "NULL output buffer");
    if (rows > cap_rows || total > cap_nnz)
        return fail(RP_ERR_CAPACITY, "need %lld rows / %lld entries", (long long)rows, (long long)total);
    if (indptr_type == RP_I32 && total >= ((int64_t)1 << 31))
        return fail(RP_ERR_UNSUPPORTED, "nnz %lld needs int64 indptr", (long long)total);
    if (n_lines > 0) {
        if ((rc = slow.grow(8 * (size_t)n_lines, device))) return rc;
        unsigned long long* ns = (unsigned long long*)errb.p + 1;
        const unsigned sgrid = (unsigned)std::min<int64_t>(std::max<int64_t>((n_lines + 255) / 256, 1), 1024);
        const unsigned pgrid = (unsigned)std::max<int64_t>((n_bytes + kPB - 1) / kPB, 1);
        if (indptr_type == RP_I64) {
            hipLaunchKernelGGL((coop_parse_kernel<int64_t>), dim3(pgrid), dim3(kLB), 0, st, t, n_bytes,
                               (const int64_t*)counts.p, (const int64_t*)nl.p, n_nl, n_lines, (const int64_t*)keep.p,
                               (const int64_t*)items.p, num_features, labels, (int64_t*)indptr, indices, data,
                               (unsigned long long*)errb.p, ns, (int64_t*)slow.p);
            hipLaunchKernelGGL((slow_line_kernel<int64_t>), dim3(sgrid), dim3(64), 0, st, t, n_bytes,
                               (const int64_t*)nl.p, n_nl, (const int64_t*)keep.p, (const int64_t*)items.p,
                               num_features, labels, (int64_t*)indptr, indices, data, ns, (const int64_t*)slow.p);
        } else {
            hipLaunchKernelGGL((coop_parse_kernel<int32_t>), dim3(pgrid), dim3(kLB), 0, st, t, n_bytes,
                               (const int64_t*)counts.p, (const int64_t*)nl.p, n_nl, n_lines, (const int64_t*)keep.p,
                               (const int64_t*)items.p, num_features, labels, (int32_t*)indptr, indices, data,
                               (unsigned long long*)errb.p, ns, (int64_t*)slow.p);
            hipLaunchKernelGGL((slow_line_kernel<int32_t>), dim3(sgrid), dim3(64), 0, st, t, n_bytes,
                               (const int64_t*)nl.p, n_nl, (const int64_t*)keep.p, (const int64_t*)items.p,
                               num_features, labels, (int32_t*)indptr, indices, data, ns, (const int64_t*)slow.p);
        }
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
    HIP_TRY(poll_stream(st));
    if (e != ~0ull) {
        if (err_line) *err_line = (int64_t)(e >> 20);
        return fail(RP_ERR_INVALID, "libsvm line %lld: %s", (long long)(e >> 20), reason((int)(e & 0xff)));
    }
    return RP_OK;
}

extern "C" int rp_libsvm_parse_device(int device, const char* text, int64_t n_bytes, int64_t num_features,
                                      double* labels, void* indptr, int32_t indptr_type, int32_t* indices,
                                      float* data, int64_t cap_rows, int64_t cap_nnz, void* stream,
                                      int64_t* n_rows, int64_t* nnz, int64_t* err_line) {
    LibsvmScratch sc;
    return libsvm_parse(sc, device, text, n_bytes, num_features, labels, indptr, indptr_type, indices, data,
                        cap_rows, cap_nnz, (hipStream_t)stream, n_rows, nnz, err_line);
}

// ------------------------------------------------------------------------------------------
// Synthetic libsvm text (benchmarks of boundary 3; the reference reads kdd12.tr, not available
// offline): row i of a device CSR as "<label> <j+1>:<value> ...\n", label 0/1, every value a
// decimal literal of 6-17 significant digits (first digit 1-9, a decimal point after a random
// digit or none, a minus sign on a quarter of them) — the literal shapes that exercise both the
// fast and the exact paths of the parser. Deterministic in (seed, entry index).
namespace {
__device__ __forceinline__ uint64_t sx_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ int sx_digits(uint64_t v) {
    int d = 1;
    while (v >= 10) {
        v /= 10;
        ++d;
    }
    return d;
}
struct SxValue {
    uint64_t r;  // digit source
    int k, q;    // significant digits, digits before the point (q == k: no point)
    bool neg;
    __device__ SxValue(uint64_t seed, int64_t e) {
        const uint64_t h = sx_mix(seed ^ ((uint64_t)e * 0xD1B54A32D192ED03ull));
        k = 6 + (int)(h % 12u);
        q = 1 + (int)((h >> 8) % (uint64_t)k);
        neg = ((h >> 20) & 3u) == 0;
        r = sx_mix(h);
    }
    __device__ int len() const { return (neg ? 1 : 0) + k + (q < k ? 1 : 0); }
};

__global__ void sx_len_kernel(int64_t n_rows, const int64_t* __restrict__ Ap, const int32_t* __restrict__ Aj,
                              uint64_t seed, int64_t* __restrict__ len) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t L = 2;  // label + newline
        for (int64_t e = Ap[i]; e < Ap[i + 1]; ++e)
            L += 2 + sx_digits((uint64_t)Aj[e] + 1) + SxValue(seed, e).len();
        len[i + 1] = L;
    }
}

__global__ void sx_write_kernel(int64_t n_rows, const int64_t* __restrict__ Ap, const int32_t* __restrict__ Aj,
                                uint64_t seed, const int64_t* __restrict__ off, char* __restrict__ text) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows; i += (int64_t)gridDim.x * blockDim.x) {
        char* o = text + off[i];
        *o++ = (sx_mix(seed + 0x51ED27ull * (uint64_t)i) & 1u) ? '1' : '0';
        for (int64_t e = Ap[i]; e < Ap[i + 1]; ++e) {
            *o++ = ' ';
            const uint64_t j = (uint64_t)Aj[e] + 1;
            const int dj = sx_digits(j);
            uint64_t v = j;
            for (int d = dj - 1; d >= 0; --d) {
                o[d] = (char)('0' + v % 10);
                v /= 10;
            }
            o += dj;
            *o++ = ':';
            SxValue x(seed, e);
            if (x.neg) *o++ = '-';
            uint64_t r = x.r;
            for (int d = 0; d < x.k; ++d) {
                if (d == x.q) *o++ = '.';
                const uint32_t dig = d == 0 ? 1u + (uint32_t)(r % 9u) : (uint32_t)(r % 10u);
                r = d % 16 == 15 ? sx_mix(r) : r / 10;
                *o++ = (char)('0' + dig);
            }
        }
        *o = '\n';
    }
}
}  // namespace

extern "C" int rp_synth_libsvm_device(int device, int64_t n_rows, const int64_t* indptr, const int32_t* indices,
                                      uint64_t seed, int64_t* line_offsets, char* text, int64_t cap_bytes,
                                      void* stream, int64_t* n_bytes) {
    if (n_rows < 0 || !indptr || !line_offsets || !n_bytes) return fail(RP_ERR_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(device));
    hipStream_t st = (hipStream_t)stream;
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>((n_rows + 255) / 256, 1), 65536);
    HIP_TRY(hipMemsetAsync(line_offsets, 0, 8, st));
    if (n_rows > 0) {
        hipLaunchKernelGGL(sx_len_kernel, dim3(grid), dim3(256), 0, st, n_rows, indptr, indices, seed, line_offsets);
        HIP_TRY(hipGetLastError());
        DevBuf tmp;
        if (int rc = inclusive_scan_i64(line_offsets + 1, n_rows, st, tmp, device)) return rc;
    }
    int64_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, line_offsets + n_rows, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *n_bytes = total;
    if (!text) return RP_OK;
    if (total > cap_bytes) return fail(RP_ERR_CAPACITY, "text needs %lld bytes", (long long)total);
    if (n_rows > 0) {
        hipLaunchKernelGGL(sx_write_kernel, dim3(grid), dim3(256), 0, st, n_rows, indptr, indices, seed, line_offsets,
                           text);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipStreamSynchronize(st));
    return RP_OK;
}
