// rp_spgemm.hip — MI355X (gfx950) projection step C = A @ R of afcarl/RandomProjection.
//
// Reference path (paths relative to /root/reference):
//   code/clustermode/randomProjection.py:46  projected_features = features_matrix.dot(local_csr_matrix)
//   -> scipy/sparse/_compressed.py:546-604 _matmul_sparse -> _sparsetools csr_matmat_maxnnz + csr_matmat
// Semantics reproduced bit for bit: for every A row, products Ax[jj]*Bx[kk] in
// (jj, kk) storage order, each multiply rounded, then added into sums[k] (starting at +0); output
// entries = distinct touched k with sums[k] != 0, in reverse first-touch order (or ascending).
//
// Pipelines (rp_project_plan reports which one a launch runs):
//   row-lane (lpr_*, short rows over a packed R, the KDD2012 default): tiles of 256 rows, one wave
//     per 64-row unit, one flat pass per wave builds its rows' output in a fixed slot in
//     first-touch order (Bloom-flagged rows recomputed exactly), rows stored in final order; then
//     one scan and one contiguous copy place the runs. R descriptors come either straight from W32
//     (direct: lpr_main_flat_kernel) or from the staged gather (reserve / partition / gather:
//     bucket-major segments streamed against an L2-resident W32 slice; lpr_wave_kernel reads its
//     unit's parts of the runs and puts the descriptors back in entry order in LDS); in auto mode
//     lpr_choose_kernel samples the feature ids and the host launches the chosen branch only.
//   tile (spgemm_lookback_kernel, long rows / generic R): one workgroup per tile, products in LDS,
//     first-touch leaders sum their column groups, decoupled look-back for the tile's offset,
//     deferred output for tiles whose prefix is late (defer_copy_kernel).
// Tiles past the LDS caps in either pipeline run scipy's dense sums/next accumulator exactly
// (heavy_tile), so any input is handled.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <atomic>
#include <cstdarg>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rp.h"
#include "rp_common.h"

using namespace rpd;

namespace {

// ------------------------------------------------------------------------------------------
// constants
constexpr int kBlock = 256;          // threads per workgroup = max rows per tile
constexpr int kMaxE = 16;            // strided A entries held per thread in stage 1
constexpr int kCapAMax = kBlock * kMaxE;  // 4096 entries per tile at most on the fast path
constexpr int kRowProdMax = 1024;    // a row with more products goes to the exact dense path

constexpr uint64_t kFlagA = 1ull << 62;   // tile aggregate published
constexpr uint64_t kFlagP = 2ull << 62;   // tile inclusive prefix published
typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // 16-byte buffer loads / stores
constexpr uint64_t kValMask = (1ull << 62) - 1;
constexpr long kSpinLimit = 1l << 27;     // bounded waits (with s_sleep): seconds, never minutes

struct Workspace {              // device memory header; tile states follow at +64 bytes
    unsigned int tile_counter;
    unsigned int error;
    unsigned long long total;
    unsigned int n_deferred;    // heavy tiles listed (exact slow path after the main kernel)
    unsigned int staged_used;   // written last in a call: 1 = the staged gather ran (rp_project_choice)
    unsigned long long pool_used;  // (unused)
    unsigned long long pad[4];     // tile slots: [0] scan ticket, [1] zero (scan base), [2] scan total
};

// Tile slots: with the full workspace, no tile waits for its predecessors. Each
// tile writes its finished output (columns u16, values T, in final order) to its own slot of
// `slot` entries (= cap_p, the tile's product cap: a bound on its outputs) and its row offsets to
// its header; a scan of the tiles' counts gives their offsets and slot_copy_kernel moves every
// slot to C. A tile past the caps (exact slow path) only counts, lists itself and marks its
// header; tile_heavy_write_kernel writes it after the scan. (Round 5 published prefixes by a
// decoupled look-back and parked late tiles in a pool: 55 ms of configs[3]'s 198 went to the
// look-back and 10 ms to the pool copy.) cols == NULL: no slots (a small caller workspace), every
// tile waits for its prefix (blocking look-back) and writes C itself.
struct DeferSpace {
    unsigned int* list;          // n_tiles: heavy tiles, count in ws->n_deferred
    unsigned long long* toff;    // n_tiles: the tile's output offset (scan of tcnt)
    uint16_t* hdr;               // n_tiles x (rpt + 1): row offsets in the tile, [rows] = count (0xffff: heavy)
    uint16_t* cols;              // n_tiles x slot, or NULL
    unsigned char* vals;         // n_tiles x slot x sizeof(T)
    uint32_t* tcnt;              // n_tiles: the tile's output entries
    unsigned long long slot;     // entries per tile slot
};
constexpr uint16_t kHdrHeavy = 0xffffu;

// ------------------------------------------------------------------------------------------
// R layouts
//
// Packed (single magnitude, p <= 16384): one 64-bit word per feature j
//   bits 61..63 = n, the feature's entry count, if n <= 4: entry t in bits [15t, 15t + 15) as
//                 (sign << 14) | column (14 bits), in R's storage order;
//   bits 61..63 = 7: more than 4 entries, bits 0..60 = offset of a record in O (u16):
//                 O[rec] = n, O[rec+1..rec+n] = (sign << 15) | column.
// One gather serves the whole R row for 99.97% of KDD2012 features (every L2 miss costs a whole
// line whatever its width, so the wide word is free and no dependent record load is needed).
// Value of an entry = sign ? -mag : mag, so x * value == x * Bx bitwise (IEEE negation symmetry).
struct PackedR {
    const uint64_t* W;
    const uint16_t* O;
    const uint64_t* SW;  // side table: W words of the features with > 2 entries (W32 code 3), or NULL
    const uint32_t* BM;  // nonempty-feature bitmap (1 bit per feature, m <= 2^26), or NULL
    uint32_t w_bytes;    // bytes of W when BM is set (the tile kernel's buffer loads)
};
constexpr uint64_t kOvf = 7ull << 61;
constexpr uint32_t kW32J = (1u << 26) - 1;  // side-table index bits of a code-3 W32 word (m <= 2^26)
constexpr uint64_t kLow61 = (1ull << 61) - 1;
// Generic CSR (any values): Bp int32 (m + 1), Bj uint16, Bx in the compute type.
template <typename T>
struct GenericR {
    const int32_t* Bp;
    const uint16_t* Bj;
    const T* Bx;
};

// descriptor of the R row of one A entry, produced in stage 1
//   packed : d = the word itself, or kOvf | (record offset + 1) (first entry) for long rows
//   generic: d = Bp[j]
template <typename T>
__device__ __forceinline__ uint64_t r_describe(const PackedR& R, int32_t j, uint32_t& cnt) {
    const uint64_t w = R.W[j];
    const uint32_t n = (uint32_t)(w >> 61);
    if (n == 7) {
        const uint64_t rec = w & kLow61;
        cnt = R.O[rec];
        return kOvf | (rec + 1);
    }
    cnt = n;
    return w;
}
template <typename T>
__device__ __forceinline__ uint64_t r_describe(const GenericR<T>& R, int32_t j, uint32_t& cnt) {
    int32_t b0 = R.Bp[j];
    cnt = (uint32_t)(R.Bp[j + 1] - b0);
    return (uint64_t)(uint32_t)b0;
}

template <typename T>
__device__ __forceinline__ T tmul(T a, T b);
template <>
__device__ __forceinline__ float tmul<float>(float a, float b) { return __fmul_rn(a, b); }
template <>
__device__ __forceinline__ double tmul<double>(double a, double b) { return __dmul_rn(a, b); }
template <typename T>
__device__ __forceinline__ T tadd(T a, T b);
template <>
__device__ __forceinline__ float tadd<float>(float a, float b) { return __fadd_rn(a, b); }
template <>
__device__ __forceinline__ double tadd<double>(double a, double b) { return __dadd_rn(a, b); }

// one T from a raw buffer (out-of-range offsets read 0 without a memory access)
template <typename T>
__device__ __forceinline__ T buf_load_t(__amdgpu_buffer_rsrc_t r, uint32_t off);
template <>
__device__ __forceinline__ float buf_load_t<float>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
template <>
__device__ __forceinline__ double buf_load_t<double>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return __longlong_as_double((long long)(((uint64_t)v[1] << 32) | v[0]));
}

// t-th product (column, x * value) of an entry described by d
template <typename T>
__device__ __forceinline__ void r_product(const PackedR& R, T mag, uint64_t d, uint32_t t, T x,
                                          uint32_t& col, T& v) {
    if ((d >> 61) == 7) {
        const uint32_t e = R.O[(d & kLow61) + t];
        col = e & 0x7fffu;
        v = tmul<T>(x, (e & 0x8000u) ? -mag : mag);
    } else {
        const uint32_t e = (uint32_t)(d >> (15 * t)) & 0x7fffu;
        col = e & 0x3fffu;
        v = tmul<T>(x, (e & 0x4000u) ? -mag : mag);
    }
}
template <typename T>
__device__ __forceinline__ void r_product(const GenericR<T>& R, T, uint64_t d, uint32_t t, T x,
                                          uint32_t& col, T& v) {
    const uint32_t b0 = (uint32_t)d;
    col = R.Bj[b0 + t];
    v = tmul<T>(x, R.Bx[b0 + t]);
}

// ------------------------------------------------------------------------------------------
// block-level helpers (256 threads = 4 waves of 64)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// inclusive wave scan with DPP (row_shr 1/2/4/8 inside 16-lane rows, then row_bcast 15/31)
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}

// exclusive scan of one value per thread; *total = block sum. Contains two barriers.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_wsum, uint32_t* total) {
    const uint32_t inc = wave_incl_scan(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) s_wsum[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kBlock / 64; ++i) {
        uint32_t s = s_wsum[i];
        base += (i < w) ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// decoupled look-back, executed by wave 0 of the workgroup (all 64 lanes): publish this tile's
// aggregate, then read the states of 64 predecessors per poll (lane l reads tile - 1 - l - 64k),
// summing aggregates up to the nearest inclusive prefix; publish the inclusive prefix. Each state
// is one 8-byte granule {flag, value} written and read with relaxed agent-scope atomics (sc1), so
// no separate payload needs ordering (MI355X_MICROARCH.md, Workgroup dispatch: granule hand-off).
// Waits are bounded (kSpinLimit polls with s_sleep); a timeout sets ws->error.
__device__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// max_polls < 0: wait (bounded by kSpinLimit); otherwise give up after max_polls unsuccessful
// polls, return ~0ull and leave only the aggregate published. publish_agg = false: the aggregate
// is already there (defer_copy_kernel).
__device__ unsigned long long lookback_wave(unsigned long long* states, unsigned int tile,
                                            unsigned long long agg, Workspace* ws,
                                            long max_polls = -1, bool publish_agg = true,
                                            long max_ticks = 0) {
    const int lane = threadIdx.x & 63;
    if (tile == 0) {
        if (lane == 0)
            __hip_atomic_store(&states[0], kFlagP | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0ull;
    }
    if (lane == 0 && publish_agg)
        __hip_atomic_store(&states[tile], kFlagA | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long excl = 0;
    long base = (long)tile - 1;  // nearest predecessor not yet summed
    long spins = 0;
    const unsigned long long t0 = max_ticks > 0 ? __builtin_amdgcn_s_memrealtime() : 0ull;
    while (true) {
        const long idx = base - lane;
        unsigned long long st = idx >= 0 ? __hip_atomic_load(&states[idx], __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT)
                                         : kFlagP;  // before tile 0: prefix 0
        const unsigned long long ready = __ballot(st != 0);
        const unsigned long long pmask = __ballot((st & ~kValMask) == kFlagP);
        const int first_p = pmask ? __builtin_ctzll(pmask) : 64;
        const unsigned long long need = first_p >= 63 ? ~0ull : ((2ull << first_p) - 1);
        if ((ready & need) == need) {
            excl += wave_sum_u64(lane <= first_p ? (st & kValMask) : 0ull);
            if (first_p < 64) break;
            base -= 64;
            continue;
        }
        if (max_polls >= 0 && (max_ticks > 0 ? (long)(__builtin_amdgcn_s_memrealtime() - t0) >= max_ticks
                                             : spins >= max_polls))
            return ~0ull;  // defer: aggregate stays published
        if (++spins > kSpinLimit) {
            if (lane == 0) atomicOr(&ws->error, 1u);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0)
        __hip_atomic_store(&states[tile], kFlagP | (excl + agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// ------------------------------------------------------------------------------------------
// Exact slow path for tiles beyond the LDS caps: scipy's dense sums[p]/next[p] accumulator in LDS.
// Rows are done one after another; a row's entries stream in chunks of 256 (parallel gathers,
// products staged in LDS in (jj, kk) order), and one lane accumulates them in order. Pass 0 counts
// (row counts -> s_rowc), pass 1 writes at the tile offset from the look-back.
constexpr int kHeavyBuf = 32;   // staged products per chunk

__host__ __device__ inline size_t heavy_lds_bytes(int64_t p, size_t vs) {
    const size_t acc = (((size_t)p * (vs + 2)) + 15) & ~size_t(15);
    return acc + ((2 * kHeavyBuf + 15) & ~size_t(15)) + vs * kHeavyBuf + 4 * kBlock;  // + row counts
}

template <typename T, typename IP, typename OP, typename OI, typename RL>
__device__ void heavy_tile(const RL& R, T mag, const IP* __restrict__ Ap,
                           const int32_t* __restrict__ Aj, const T* __restrict__ Ax, int64_t row0,
                           int nrows, int p, unsigned char* lds, uint32_t* s_rowc, uint32_t* s_wsum,
                           int pass, unsigned long long tile_off, OP* __restrict__ Cp,
                           OI* __restrict__ Cj, T* __restrict__ Cx, bool write_entries, int order) {
    __shared__ int s_take, s_end;
    const size_t vs = sizeof(T);
    T* sums = reinterpret_cast<T*>(lds);
    int16_t* next = reinterpret_cast<int16_t*>(lds + vs * (size_t)p);
    unsigned char* buf = lds + ((((size_t)p * (vs + 2)) + 15) & ~size_t(15));
    uint16_t* s_hk = reinterpret_cast<uint16_t*>(buf);
    T* s_hv = reinterpret_cast<T*>(buf + ((2 * kHeavyBuf + 15) & ~size_t(15)));
    const int tid = threadIdx.x;
    for (int k = tid; k < p; k += kBlock) {
        sums[k] = T(0);
        next[k] = -1;
    }
    __syncthreads();
    unsigned long long off = tile_off;
    int head = -2, length = 0;  // meaningful on lane 0 only
    auto touch = [&](uint32_t k, T v) {
        sums[k] = tadd<T>(sums[k], v);
        if (next[k] == -1) {
            next[k] = (int16_t)head;
            head = (int)k;
            ++length;
        }
    };
    for (int r = 0; r < nrows; ++r) {
        const int64_t jb = (int64_t)Ap[row0 + r], je = (int64_t)Ap[row0 + r + 1];
        head = -2;
        length = 0;
        for (int64_t c = jb; c < je;) {
            const int64_t e = c + tid;
            uint32_t cnt = 0;
            uint64_t d = 0;
            T x = T(0);
            if (e < je) {
                x = Ax[e];
                d = r_describe<T>(R, Aj[e], cnt);
            }
            uint32_t tot;
            const uint32_t excl = block_excl_scan(cnt, s_wsum, &tot);
            const bool fits = e < je && excl + cnt <= (uint32_t)kHeavyBuf;
            const int take = __syncthreads_count(fits);
            if (take > 0) {
                if (fits) {
                    for (uint32_t t = 0; t < cnt; ++t) {
                        uint32_t col;
                        T v;
                        r_product<T>(R, mag, d, t, x, col, v);
                        s_hk[excl + t] = (uint16_t)col;
                        s_hv[excl + t] = v;
                    }
                    if (tid == take - 1) s_end = (int)(excl + cnt);
                }
                __syncthreads();
                if (tid == 0)
                    for (int q = 0; q < s_end; ++q) touch(s_hk[q], s_hv[q]);
                if (tid == 0) s_take = take;
            } else if (tid == 0) {  // one entry with more than kHeavyBuf products: straight from R
                for (uint32_t t = 0; t < cnt; ++t) {
                    uint32_t col;
                    T v;
                    r_product<T>(R, mag, d, t, x, col, v);
                    touch(col, v);
                }
                s_take = 1;
            }
            __syncthreads();
            c += s_take;
            __syncthreads();
        }
        if (tid == 0) {
            uint32_t cnt_r = 0;
            const unsigned long long row_off = off;
            for (int q = 0; q < length; ++q) {
                const T sv = sums[head];
                if (sv != T(0)) {
                    if (pass == 1 && write_entries) {
                        Cj[off] = (OI)head;
                        Cx[off] = sv;
                    }
                    ++off;
                    ++cnt_r;
                }
                const int tmp = head;
                head = next[head];
                next[tmp] = -1;
                sums[tmp] = T(0);
            }
            if (pass == 0) {
                s_rowc[r] = cnt_r;
            } else {
                Cp[row0 + r] = (OP)row_off;
                if (order == RP_ORDER_SORTED && write_entries && cnt_r > 1) {
                    const unsigned long long n = cnt_r;  // shell sort of the row segment (rare path)
                    for (unsigned long long gap = n / 2; gap > 0; gap /= 2)
                        for (unsigned long long a = gap; a < n; ++a) {
                            OI kc = Cj[row_off + a];
                            T kv = Cx[row_off + a];
                            unsigned long long b = a;
                            while (b >= gap && Cj[row_off + b - gap] > kc) {
                                Cj[row_off + b] = Cj[row_off + b - gap];
                                Cx[row_off + b] = Cx[row_off + b - gap];
                                b -= gap;
                            }
                            Cj[row_off + b] = kc;
                            Cx[row_off + b] = kv;
                        }
                }
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// the fused kernel
struct Caps {
    int cap_a;   // A entries per tile on the fast path (<= kCapAMax)
    int cap_p;   // products per tile on the fast path (<= 65535)
    int rpt;     // rows per tile (<= kBlock)
};

// Dynamic-LDS carve-up of a tile (host sizes it, device uses it; offsets 16-byte aligned):
//   X : eoff[cap_a + 1] (u16)                      product offset of every A entry (stage 1)
//   U : erow[cap_a] (u8, stage 1) | rank[cap_p + 1] (u16, stages 2-3)
//   P : pv[cap_p] (T), pkr[cap_p] (u32 = row << 16 | column)   products; leaders' sums in place
// The exact slow path reuses the whole region as scipy's dense sums[p]/next[p] accumulator.
struct TileLayout {
    size_t x, u, pv, pkr, total;
    __host__ __device__ TileLayout(const Caps& c, size_t vs) {
        auto al = [](size_t v) { return (v + 15) & ~size_t(15); };
        x = 0;
        u = al(2 * (size_t)(c.cap_a + 1));
        pv = u + al(std::max<size_t>((size_t)c.cap_a, 2 * (size_t)(c.cap_p + 1)));
        pkr = pv + al(vs * (size_t)c.cap_p);
        total = pkr + al(4 * (size_t)c.cap_p);
    }
};

// exclusive scan in place of n (<= 65535 total) u16 or u32 values in LDS by the whole block:
// each thread scans a contiguous chunk, chunk sums are block-scanned; a[n] = total (u32 return).
template <typename V>
__device__ __forceinline__ uint32_t lds_excl_scan(V* a, uint32_t n, uint32_t* s_wsum) {
    const uint32_t per = (n + kBlock - 1) / kBlock;
    const uint32_t c0 = std::min<uint32_t>(threadIdx.x * per, n), c1 = std::min<uint32_t>(c0 + per, n);
    uint32_t local = 0;
    for (uint32_t e = c0; e < c1; ++e) local += a[e];
    uint32_t total;
    uint32_t run = block_excl_scan(local, s_wsum, &total);
    for (uint32_t e = c0; e < c1; ++e) {
        const uint32_t v = a[e];
        a[e] = (V)run;
        run += v;
    }
    if (threadIdx.x == 0) a[n] = (V)total;
    __syncthreads();
    return total;
}

// WPE: minimum waves per SIMD the register allocation must allow (1 = unconstrained: 76 VGPRs,
// 6 waves). 7 is used when the tile's LDS leaves room for 7 tiles per CU (configs[3]: 29-row tiles,
// 19.6 KB; f32 packed, 71 VGPRs, no spills): 252 -> 235 ms. KDD2012 tiles (26.9 KB) are
// LDS-limited to 5 per CU, where the tighter allocation measured 3% slower.
template <typename T, typename IP, typename OP, typename OI, typename RL, int WPE = 1>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE)))
spgemm_lookback_kernel(RL R, T mag, int p, int64_t n_rows, const IP* __restrict__ Ap,
                       const int32_t* __restrict__ Aj, const T* __restrict__ Ax,
                       OP* __restrict__ Cp, OI* __restrict__ Cj, T* __restrict__ Cx,
                       unsigned long long capacity, Caps caps, int order, Workspace* ws,
                       unsigned int n_tiles, DeferSpace dfr) {
    extern __shared__ __align__(16) unsigned char lds[];
    __shared__ uint16_t s_rowptr[kBlock + 1];  // row -> first entry (tile-relative, <= cap_a)
    __shared__ uint16_t s_rowS[kBlock + 1];    // row -> first product
    __shared__ uint32_t s_wsum[kBlock / 64];
    __shared__ unsigned int s_tile;
    __shared__ int s_heavy;
    __shared__ unsigned long long s_off;
    __shared__ unsigned long long s_pool;

    unsigned long long* states = reinterpret_cast<unsigned long long*>(ws + 1);
    const int tid = threadIdx.x;
    if (tid == 0) {
        s_tile = atomicAdd(&ws->tile_counter, 1u);
        s_heavy = 0;
    }
    __syncthreads();
    const unsigned int tile = s_tile;
    if (tile >= n_tiles) return;  // uniform

    const int64_t row0 = (int64_t)tile * caps.rpt;
    const int nrows = (int)std::min<int64_t>(caps.rpt, n_rows - row0);
    const int64_t ea = (int64_t)Ap[row0];
    const int64_t eb = (int64_t)Ap[row0 + nrows];
    const int64_t nnz_t = eb - ea;

    const TileLayout L(caps, sizeof(T));
    uint16_t* s_eoff = reinterpret_cast<uint16_t*>(lds + L.x);
    uint8_t* s_erow = reinterpret_cast<uint8_t*>(lds + L.u);
    uint16_t* s_rank = reinterpret_cast<uint16_t*>(lds + L.u);
    T* s_pv = reinterpret_cast<T*>(lds + L.pv);
    uint32_t* s_pkr = reinterpret_cast<uint32_t*>(lds + L.pkr);

    if (nnz_t <= caps.cap_a) {  // uniform
        const uint32_t ne = (uint32_t)nnz_t;
        for (int r = tid; r <= nrows; r += kBlock) s_rowptr[r] = (uint16_t)((int64_t)Ap[row0 + r] - ea);
        // ---- stage 1a: coalesced A entries, one R-descriptor gather per entry, kept in registers
        // across the scan below (the 64-bit W word, or a generic R's row start)
        uint64_t d[kMaxE];
        T x[kMaxE];
        const int32_t* __restrict__ Ajt = Aj + ea;
        const T* __restrict__ Axt = Ax + ea;
        bool gated = false;
        if constexpr (std::is_same<RL, PackedR>::value) gated = R.BM != nullptr && ne > 0;
        if (gated) {
            // packed R with a nonempty-feature bitmap (m <= 2^26, L2-resident: 1.25 MB for
            // configs[3]): an entry whose R row is empty (73% on configs[3]) fetches no W line.
            // Loads in straight-line rounds (feature ids + values, bitmap words, W words), the W
            // load of a skipped entry an out-of-range buffer load (returns 0, no memory access)
            if constexpr (std::is_same<RL, PackedR>::value) {
                int32_t jv[kMaxE];
#pragma unroll
                for (int i = 0; i < kMaxE; ++i) {
                    const uint32_t ec = std::min<uint32_t>(tid + i * kBlock, ne - 1);
                    jv[i] = Ajt[ec];
                    x[i] = Axt[ec];
                }
                uint32_t bw[kMaxE];
#pragma unroll
                for (int i = 0; i < kMaxE; ++i) bw[i] = R.BM[(uint32_t)jv[i] >> 5];
                const __amdgpu_buffer_rsrc_t wr =
                    __builtin_amdgcn_make_buffer_rsrc((void*)R.W, (short)0, (int)R.w_bytes, 0x00020000);
#pragma unroll
                for (int i = 0; i < kMaxE; ++i) {
                    const uint32_t e = tid + i * kBlock;
                    const bool take = e < ne && ((bw[i] >> ((uint32_t)jv[i] & 31u)) & 1u);
                    const auto v = __builtin_amdgcn_raw_buffer_load_b64(wr, take ? (uint32_t)jv[i] << 3 : 0xfffffff8u,
                                                                        0, 0);
                    d[i] = ((uint64_t)v[1] << 32) | v[0];
                    if (e >= ne) x[i] = T(0);
                }
#pragma unroll
                for (int i = 0; i < kMaxE; ++i) {
                    const uint32_t e = tid + i * kBlock;
                    if (e < ne) {
                        uint32_t cnt = (uint32_t)(d[i] >> 61);
                        if (cnt == 7) {  // long R row (> 4 entries): its record in O
                            const uint64_t rec = d[i] & kLow61;
                            cnt = R.O[rec];
                            d[i] = kOvf | (rec + 1);
                        }
                        s_eoff[e] = (uint16_t)cnt;
                    }
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < kMaxE; ++i) {
                const uint32_t e = tid + i * kBlock;
                x[i] = T(0);
                d[i] = 0;
                if (e < ne) {
                    uint32_t cnt;
                    x[i] = Axt[e];
                    d[i] = r_describe<T>(R, Ajt[e], cnt);
                    s_eoff[e] = (uint16_t)std::min<uint32_t>(cnt, 0xffffu);
                }
            }
        }
        __syncthreads();
        // ---- stage 1b: product offsets per entry; entry -> row map; row product ranges
        if (tid < nrows)
            for (uint32_t e = s_rowptr[tid]; e < s_rowptr[tid + 1]; ++e) s_erow[e] = (uint8_t)tid;
        const uint32_t P_t = lds_excl_scan(s_eoff, ne, s_wsum);
        const bool fits = P_t <= (uint32_t)caps.cap_p;  // uniform; if not, offsets wrapped: slow path
        if (fits)
            for (int r = tid; r <= nrows; r += kBlock) {
                const uint32_t rs = s_eoff[s_rowptr[r]];
                s_rowS[r] = (uint16_t)rs;
                if (r < nrows && s_eoff[s_rowptr[r + 1]] - rs > (uint32_t)kRowProdMax) s_heavy = 1;
            }
        if (fits) {
            // ---- stage 1c: every product x*b (one rounding), grouped by row, in (jj, kk) order
#pragma unroll
            for (int i = 0; i < kMaxE; ++i) {
                if (tid + i * kBlock < ne) {
                    const uint32_t e = tid + i * kBlock;
                    const uint64_t de = d[i];
                    const uint32_t o0 = s_eoff[e], o1 = s_eoff[e + 1];
                    const uint32_t rtag = (uint32_t)s_erow[e] << 16;
                    for (uint32_t t = 0; t < o1 - o0; ++t) {
                        uint32_t col;
                        T v;
                        r_product<T>(R, mag, de, t, x[i], col, v);
                        s_pkr[o0 + t] = rtag | col;
                        s_pv[o0 + t] = v;
                    }
                }
            }
            // stage 2 reads keys in aligned groups of four: pad the last group with a key no product
            // has (rows < 256), so stale LDS from an earlier tile can never match
            if (tid < 4 && P_t + tid < (uint32_t)caps.cap_p && ((P_t + tid) >> 2) == (P_t >> 2))
                s_pkr[P_t + tid] = 0xffffffffu;
            __syncthreads();
            if (!s_heavy) {  // uniform
                // ---- stage 2: flat over products. A product leads its column group if no earlier
                // product of its row has that column (= scipy's first touch); the leader sums the
                // group in sequence order starting from +0 (scipy: sums[k] = 0, then +=).
                for (uint32_t q = tid; q < P_t; q += kBlock) {
                    const uint32_t kr = s_pkr[q];
                    const uint32_t r = kr >> 16;
                    const uint32_t rs = s_rowS[r], re = s_rowS[r + 1];
                    // keys are read four at a time (one ds_read_b128 per 16-byte aligned group).
                    // A key holds the row, so keys of other rows never match: before q only
                    // "earlier" matters for the leader test, after q only "later" for the sum.
                    const uint4* pk4 = reinterpret_cast<const uint4*>(s_pkr);
                    const uint32_t gq = q >> 2, oq = q & 3u;
                    bool leader = true;
                    for (uint32_t g = rs >> 2; g < gq; ++g) {
                        const uint4 k4 = pk4[g];
                        leader &= (k4.x != kr) & (k4.y != kr) & (k4.z != kr) & (k4.w != kr);
                    }
                    const uint4 kq = pk4[gq];
                    leader &= !(((oq > 0u) & (kq.x == kr)) | ((oq > 1u) & (kq.y == kr)) |
                                ((oq > 2u) & (kq.z == kr)));
                    uint16_t flag = 0;
                    if (leader) {
                        T sum = tadd<T>(T(0), s_pv[q]);
                        // the rest of q's group, then whole groups up to the row end, in order
                        if ((oq < 1u) & (kq.y == kr)) sum = tadd<T>(sum, s_pv[(gq << 2) + 1]);
                        if ((oq < 2u) & (kq.z == kr)) sum = tadd<T>(sum, s_pv[(gq << 2) + 2]);
                        if ((oq < 3u) & (kq.w == kr)) sum = tadd<T>(sum, s_pv[(gq << 2) + 3]);
                        for (uint32_t g = gq + 1; (g << 2) < re; ++g) {
                            const uint4 k4 = pk4[g];
                            if ((k4.x == kr) | (k4.y == kr) | (k4.z == kr) | (k4.w == kr)) {  // rare
                                const uint32_t b = g << 2;
                                if (k4.x == kr) sum = tadd<T>(sum, s_pv[b]);
                                if (k4.y == kr) sum = tadd<T>(sum, s_pv[b + 1]);
                                if (k4.z == kr) sum = tadd<T>(sum, s_pv[b + 2]);
                                if (k4.w == kr) sum = tadd<T>(sum, s_pv[b + 3]);
                            }
                        }
                        s_pv[q] = sum;  // position q is read by no other leader (column differs)
                        flag = sum != T(0) ? 1 : 0;
                    }
                    s_rank[q] = flag;
                }
                __syncthreads();
                // ---- stage 3: ranks of kept entries = tile-local output positions; the tile's slot
                // (or, without slots, its prefix from a blocking look-back)
                const uint32_t tile_c = lds_excl_scan(s_rank, P_t, s_wsum);
                const bool deferred = dfr.cols != nullptr;  // uniform: slots
                if (deferred) {
                    if (tid == 0) dfr.tcnt[tile] = tile_c;
                    s_pool = (unsigned long long)tile * dfr.slot;
                } else {
                    if (tid < 64) {
                        const unsigned long long g = lookback_wave(states, tile, tile_c, ws, -1, true, 0);
                        if (tid == 0) s_off = g;
                    }
                    __syncthreads();
                }
                const unsigned long long G = deferred ? 0ull : s_off;
                // slots: entries go to the tile's slot at their tile-local positions and the row
                // offsets to its header; slot_copy_kernel adds the offset after the scan
                if (deferred) {
                    uint16_t* ro = dfr.hdr + (size_t)tile * (caps.rpt + 1);
                    if (tid < nrows) ro[tid] = s_rank[s_rowS[tid]];
                    if (tid == 0) ro[nrows] = (uint16_t)tile_c;
                } else if (tid < nrows) {
                    Cp[row0 + tid] = (OP)(G + s_rank[s_rowS[tid]]);
                }
                uint16_t* __restrict__ pc = dfr.cols + (deferred ? s_pool : 0ull);
                T* __restrict__ pv = reinterpret_cast<T*>(dfr.vals) + (deferred ? s_pool : 0ull);
                if (deferred || G + tile_c <= capacity) {
                    // kept leaders write straight into the tile's contiguous output range
                    for (uint32_t q = tid; q < P_t; q += kBlock) {
                        const uint32_t rk = s_rank[q];
                        if (s_rank[q + 1] == rk) continue;  // not a kept leader
                        const uint32_t kr = s_pkr[q];
                        const uint32_t r = kr >> 16;
                        const uint32_t rs = s_rowS[r], re = s_rowS[r + 1];
                        uint32_t pos = s_rank[rs];
                        if (order == RP_ORDER_SORTED) {
                            for (uint32_t u = rs; u < re; ++u)
                                pos += (s_rank[u + 1] != s_rank[u] && s_pkr[u] < kr) ? 1u : 0u;
                        } else {
                            pos += s_rank[re] - 1 - rk;  // reverse first-touch order
                        }
                        if (deferred) {
                            pc[pos] = (uint16_t)(kr & 0xffffu);
                            pv[pos] = s_pv[q];
                        } else {
                            Cj[G + pos] = (OI)(kr & 0xffffu);
                            Cx[G + pos] = s_pv[q];
                        }
                    }
                }
                if (!deferred && tile == n_tiles - 1 && tid == 0) {
                    Cp[n_rows] = (OP)(G + tile_c);
                    ws->total = G + tile_c;
                }
                return;
            }
        }
        __syncthreads();
    }
    // ---- exact slow path (uniform branch)
    uint32_t* s_rowc = reinterpret_cast<uint32_t*>(lds + heavy_lds_bytes(p, sizeof(T)) - 4 * kBlock);
    heavy_tile<T, IP, OP, OI, RL>(R, mag, Ap, Aj, Ax, row0, nrows, p, lds, s_rowc, s_wsum, 0, 0,
                                  Cp, Cj, Cx, false, order);
    uint32_t tile_c;
    (void)block_excl_scan(tid < nrows ? s_rowc[tid] : 0u, s_wsum, &tile_c);
    if (dfr.cols) {  // slots: count only; tile_heavy_write_kernel writes it after the scan
        if (tid == 0) {
            dfr.tcnt[tile] = tile_c;
            dfr.hdr[(size_t)tile * (caps.rpt + 1) + nrows] = kHdrHeavy;
            dfr.list[atomicAdd(&ws->n_deferred, 1u)] = tile;
        }
        return;
    }
    if (tid < 64) {
        const unsigned long long g = lookback_wave(states, tile, tile_c, ws, -1, true, 0);
        if (tid == 0) s_off = g;
    }
    __syncthreads();
    const unsigned long long G = s_off;
    const bool write = G + tile_c <= capacity;
    heavy_tile<T, IP, OP, OI, RL>(R, mag, Ap, Aj, Ax, row0, nrows, p, lds, s_rowc, s_wsum, 1, G,
                                  Cp, Cj, Cx, write, order);
    if (tile == n_tiles - 1 && tid == 0) {
        Cp[n_rows] = (OP)(G + tile_c);
        ws->total = G + tile_c;
    }
}

// ------------------------------------------------------------------------------------------
// Staged gather of the row-lane pipeline. Uniform columns over a 437 MB W make
// every descriptor gather a random 128-B line fill, capped near 55 G lines/s on MI355X whatever the
// load flavour (profiles/r01_probe_gather_*.json). Staging turns them into L2 hits plus streams: the
// tile's entries are partitioned by column bucket (2^sb features = a W32 slice of 4 * 2^sb bytes),
// each bucket's words gathered on one XCD whose 4 MB L2 holds the slice, and the descriptors put
// back into entry order by the wave kernel. (The tile pipeline's own staged gather, measured slower
// than its direct gathers in every configuration, was removed in round 4.)
// W32 word of feature j (built from W): bits 30-31 = n if the R row has n <= 2 entries, the low
// 30 bits then hold W's slots 0-1 unchanged; n = 3 marks "more": the count and the feature's index
// in the side table SW, whose word the wave kernel fetches (4% of KDD2012 features).
constexpr int kStageMaxNB = 256;  // buckets (one per thread in the partition scan)

// bit j of BM = feature j has at least one R entry (57% of KDD2012 features have none)
__global__ void build_bitmap_kernel(const uint64_t* __restrict__ W, uint32_t* __restrict__ BM, int64_t m) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < (m + 31) / 32;
         k += (int64_t)gridDim.x * blockDim.x) {
        uint32_t b = 0;
        for (int i = 0; i < 32 && k * 32 + i < m; ++i) b |= (W[k * 32 + i] >> 61) ? (1u << i) : 0u;
        BM[k] = b;
    }
}

// Side table: the W words of the features with more than 2 R entries (4.1% of KDD2012's features,
// 1.9% of its A entries), packed in feature order (SW[k] = W[j] for the k-th such feature j). A W32
// code-3 word carries k instead of j, so the row-lane kernels fetch those words from an 8 MB table
// (MALL-resident, partly L2) instead of a random line of the 437 MB W. Built in two passes over
// 1024-feature blocks: counts, then (after an inclusive scan of the counts) the words.
constexpr int kSideBlock = 1024;
__global__ void __launch_bounds__(kSideBlock)
side_count_kernel(const uint64_t* __restrict__ W, int64_t m, int64_t* __restrict__ cnt) {
    __shared__ uint32_t s_n;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const int64_t j = (int64_t)blockIdx.x * kSideBlock + threadIdx.x;
    const bool side = j < m && (W[j] >> 61) > 2;
    const uint64_t b = __ballot(side);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&s_n, (uint32_t)__popcll(b));
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = s_n;
}

// W32 word of feature j: n <= 2 entries inline (the low 30 bits of W); more: code 3, the entry
// count (4 bits, 15 = "15 or more") and the side index k (26 bits: staging needs m <= 2^26), so
// the row-lane kernels know every entry's product count without the side gather. cnt_incl = the
// inclusive scan of side_count_kernel's counts.
__global__ void __launch_bounds__(kSideBlock)
build_w32_kernel(const uint64_t* __restrict__ W, const uint16_t* __restrict__ O, const int64_t* __restrict__ cnt_incl,
                 uint32_t* __restrict__ W32, uint64_t* __restrict__ SW, int64_t m) {
    __shared__ uint32_t s_wsum[kSideBlock / 64];
    const int64_t j = (int64_t)blockIdx.x * kSideBlock + threadIdx.x;
    const uint64_t w = j < m ? W[j] : 0ull;
    const uint32_t n = (uint32_t)(w >> 61);
    const bool side = n > 2;
    const uint64_t b = __ballot(side);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) s_wsum[wv] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t k = (uint32_t)(blockIdx.x ? cnt_incl[blockIdx.x - 1] : 0) +
                 (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
    for (int i = 0; i < wv; ++i) k += s_wsum[i];
    if (j >= m) return;
    if (side) SW[k] = w;
    const uint32_t cnt = n != 7 ? n : O[w & kLow61];
    W32[j] = n <= 2 ? ((n << 30) | (uint32_t)(w & 0x3fffffffu)) : (0xc0000000u | (std::min(cnt, 15u) << 26) | k);
}


// ---- staging for the row-lane pipeline: bucket-major runs inside groups of kRunGroup tiles.
// S holds, for tile group g and bucket b, the entries of all the group's tiles whose feature falls
// in b as ONE contiguous segment (one run per tile, runs in claim order); segments are laid out in
// (g, b) order, each with a reserve sized from the group's entries (lpr_reserve_kernel). Inside a
// tile's run the entries are grouped by 64-row unit (unit 0's first, any order inside a unit), so
// each wave of the wave kernel reads its own unit's part of every run. The gather streams whole
// segments (full 128-byte lines, nothing shared between workgroups). One pass over A (the
// partition claims the runs of a super-tile of kPartTiles tiles with one atomicAdd per bucket on
// its segment's fill); a segment past its reserve (columns far from uniform) sends the rest of the
// call to direct gathers. Index arrays (workspace, tile-major: a tile's table is contiguous):
//   OFF2[t][b] (u32)     start of tile t's run in segment (g, b), relative to the segment
//   CU[t][u - 1][b] (u16) entries of bucket b in units < u of tile t, u = 1..4 (u = 4: the run)
//   GB[g*nb + b] (i64)   segment start in S (exclusive prefix of the reserves), FILL[g*nb + b] its fill
// S word: the entry's index in its tile << 20 | its feature's bits inside the bucket. A tile past
// the entry cap stages nothing (its counts are 0): the heavy path reads A itself.
constexpr int kRunGroup = 4096;  // tiles per group (uniform KDD2012: ~110K entries per segment)

// XCD-aware tile order: workgroup i runs on XCD i % 8 (round-robin dispatch); XCD x takes tiles
// [x * t8, (x + 1) * t8) in order, so neighbouring tiles are in flight on one XCD together
__device__ __forceinline__ unsigned xcd_tile(unsigned i, unsigned t8) { return (i & 7u) * t8 + (i >> 3); }

// K0 (auto staging): staged or direct gathers, decided on the device per call. 8192 entries sampled
// evenly over the launch; the fraction of distinct features among them (an LDS hash set)
// estimates the share of gathers that miss L2 in direct mode: uniform KDD2012-shaped columns give
// ~100% (staging pays: configs[1] 21 ms vs 27 ms), Zipf(1.1) power-law columns ~40% (direct pays:
// 15 ms vs 21 ms). Staged iff at least kChooseDistinctPct percent are distinct.
constexpr int kChooseSamples = 8192, kChooseSlots = 16384, kChooseDistinctPct = 85;
template <typename IP>
__global__ void __launch_bounds__(1024)
lpr_choose_kernel(const IP* __restrict__ Ap, const int32_t* __restrict__ Aj, int64_t n_rows, uint32_t* __restrict__ gate) {
    __shared__ uint32_t s_tab[kChooseSlots];
    __shared__ uint32_t s_new;
    for (int i = threadIdx.x; i < kChooseSlots; i += 1024) s_tab[i] = 0u;
    if (threadIdx.x == 0) s_new = 0u;
    __syncthreads();
    const int64_t a0 = (int64_t)Ap[0], tot = (int64_t)Ap[n_rows] - a0;
    const int S = (int)std::min<int64_t>(kChooseSamples, std::max<int64_t>(tot, 0));
    for (int i = threadIdx.x; i < S; i += 1024) {
        const uint32_t key = (uint32_t)Aj[a0 + (int64_t)i * tot / S] + 1u;
        uint32_t h = (key * 0x9E3779B1u) >> 18;
        while (true) {  // S < slots: always terminates
            const uint32_t old = atomicCAS(&s_tab[h], 0u, key);
            if (old == 0u) {
                atomicAdd(&s_new, 1u);
                break;
            }
            if (old == key) break;
            h = (h + 1u) & (kChooseSlots - 1);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *gate = S > 0 && s_new * 100u >= (uint32_t)kChooseDistinctPct * (uint32_t)S ? 1u : 0u;
}

// K1: segment reserves. Segment (g, b) gets room for E + 8 sqrt(E) + 256 entries, E = the group's
// entries x bucket b's share of the features (the staged words of uniform columns are binomial
// around E: 8 sigma); GB[s] = exclusive prefix of the reserves, FILL[s] = 0. One workgroup.
constexpr int kResBlock = 1024;
template <typename IP>
__global__ void __launch_bounds__(kResBlock)
lpr_reserve_kernel(const IP* __restrict__ Ap, int64_t n_rows, int rpt, int64_t m, unsigned groups, int sb, int nb,
                   int cap_a, int64_t cap_words, int64_t* __restrict__ GB, uint32_t* __restrict__ FILL,
                   uint32_t* __restrict__ gate) {
    if (*gate == 0) return;  // the device chose direct gathers for this call
    __shared__ int64_t s[kResBlock];
    const unsigned S = groups * (unsigned)nb;
    const unsigned per = (S + kResBlock - 1) / kResBlock, lo = threadIdx.x * per, hi = std::min(S, lo + per);
    auto reserve = [&](unsigned sg) {
        const unsigned g = sg / (unsigned)nb, b = sg % (unsigned)nb;
        const int64_t r0 = std::min<int64_t>((int64_t)g * kRunGroup * rpt, n_rows);
        const int64_t r1 = std::min<int64_t>((int64_t)(g + 1) * kRunGroup * rpt, n_rows);
        // a tile past cap_a stages nothing, so a group stages at most cap_a entries per tile (the
        // workspace's S/D words are sized with the same bound for chunked launches)
        const double ents = (double)std::min<int64_t>((int64_t)Ap[r1] - (int64_t)Ap[r0],
                                                      (int64_t)cap_a * ((r1 - r0 + rpt - 1) / rpt));
        const double width = (double)std::min<int64_t>((int64_t)1 << sb, m - ((int64_t)b << sb));
        const double e = ents * width / (double)m;
        return (int64_t)(e + 8.0 * sqrt(e)) + 256;
    };
    int64_t sum = 0;
    for (unsigned i = lo; i < hi; ++i) sum += reserve(i);
    s[threadIdx.x] = sum;
    __syncthreads();
    for (unsigned o = 1; o < kResBlock; o <<= 1) {
        const int64_t v = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    int64_t run = s[threadIdx.x] - sum;
    for (unsigned i = lo; i < hi; ++i) {
        GB[i] = run;
        FILL[i] = 0u;
        run += reserve(i);
    }
    if (threadIdx.x == kResBlock - 1) {
        GB[S] = s[kResBlock - 1];
        if (s[kResBlock - 1] > cap_words) *gate = 0;  // cannot happen with the planned size: direct then
    }
}

// K2: partition, one workgroup per SUPER-TILE of kPartTiles consecutive tiles (one 256-thread
// part per tile). Each tile's entries are histogrammed by (unit, bucket) in LDS; the unit counts
// give CU and each entry's place inside its tile's run of a bucket (its unit's part's start + the
// rank the histogram's own LDS atomic returned: one atomic per entry), the bucket starts give the tile's bucket-ordered
// layout. ONE atomicAdd per bucket on FILL claims the segment room of the super-tile's runs at once:
// its tiles' runs of a bucket are adjacent in their segment, in tile order (OFF2 = each run's
// position), so the S stores of a bucket fill whole lines inside one workgroup and the wave kernel
// reads neighbouring units' parts of a run from lines its XCD's L2 already holds. The entries are
// ranked into bucket order in LDS and written to their runs (consecutive lanes -> consecutive S
// words). A run past its segment's reserve sets the gate to 0: the call's remaining kernels take
// direct gathers. A tile past the entry cap stages nothing (its counts are 0).
constexpr int kPartTiles = 2;
constexpr int kPBlock = kBlock * kPartTiles;
static_assert(kRunGroup % kPartTiles == 0, "a super-tile never straddles two groups");
// dynamic LDS: [the ranked S words [kPartTiles][cap_a], aliased by the unit histograms
// [kPartTiles][4][nb] (dead by then)] [cursors [kPartTiles][4][nb]] [run destinations
// [kPartTiles][nb] (i64)] [bucket starts [kPartTiles][nb + 1] (u16)] [each ranked word's bucket
// [kPartTiles][cap_a] (u8): the store loop finds its run without a search]
__host__ __device__ inline size_t lpr_partition_keys_bytes(int cap_a, int nb) {
    return (std::max<size_t>(4 * (size_t)kPartTiles * (size_t)cap_a, 16 * (size_t)kPartTiles * (size_t)nb) + 15) & ~size_t(15);
}
__host__ __device__ inline size_t lpr_partition_lds_bytes(int cap_a, int nb) {
    return lpr_partition_keys_bytes(cap_a, nb) + 16 * (size_t)kPartTiles * nb + 8 * (size_t)kPartTiles * nb +
           ((2 * (size_t)kPartTiles * (nb + 1) + 15) & ~size_t(15)) + (((size_t)kPartTiles * cap_a + 15) & ~size_t(15));
}
template <typename IP>
__global__ void __launch_bounds__(kPBlock)
lpr_partition_kernel(const IP* __restrict__ Ap, const int32_t* __restrict__ Aj, int64_t n_rows, int cap_a,
                     unsigned n_tiles, unsigned s8, int sb, int nb, uint32_t ostride, uint32_t* __restrict__ OFF2,
                     uint16_t* __restrict__ CU, const int64_t* __restrict__ GB, uint32_t* __restrict__ FILL,
                     uint32_t* __restrict__ S, uint32_t* __restrict__ gate) {
    extern __shared__ __align__(16) uint32_t s_key[];  // [kPartTiles][cap_a]; first the unit histograms
    __shared__ uint32_t s_wsum[kPBlock / 64];
    __shared__ int s_over;
    __shared__ uint32_t s_gate;
    const int tid = threadIdx.x, q = tid >> 8, qt = tid & (kBlock - 1), w = tid >> 6;
    const unsigned t0 = xcd_tile(blockIdx.x, s8) * kPartTiles;
    if (t0 >= n_tiles) return;  // uniform
    const unsigned t = t0 + q;
    const bool live = t < n_tiles;  // part-uniform
    // the tile's row pointers are requested with the gate (one memory round trip for both)
    int64_t ea = 0, ne = 0;
    uint32_t u1 = 0, u2 = 0, u3 = 0;  // first entries of units 1..3 (tile-relative)
    if (live) {
        const int64_t row0 = (int64_t)t * kBlock;
        ea = (int64_t)Ap[row0];
        ne = (int64_t)Ap[std::min<int64_t>(row0 + kBlock, n_rows)] - ea;
        u1 = (uint32_t)((int64_t)Ap[std::min<int64_t>(row0 + 64, n_rows)] - ea);
        u2 = (uint32_t)((int64_t)Ap[std::min<int64_t>(row0 + 128, n_rows)] - ea);
        u3 = (uint32_t)((int64_t)Ap[std::min<int64_t>(row0 + 192, n_rows)] - ea);
    }
    // Another workgroup of this launch may clear the gate (segment overflow below) at any time, so
    // the gate is read ONCE per workgroup and broadcast: every wave takes the same branch (a split
    // workgroup would run the scan and the S stores with LDS state its exited waves never wrote).
    if (tid == 0) s_gate = __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_gate == 0) return;  // uniform
    unsigned char* dyn = reinterpret_cast<unsigned char*>(s_key) + lpr_partition_keys_bytes(cap_a, nb);
    uint32_t* s_cur = reinterpret_cast<uint32_t*>(dyn);  // per (tile, unit, bucket): the part's start in the layout
    int64_t* s_dst = reinterpret_cast<int64_t*>(dyn + 16 * (size_t)kPartTiles * nb);  // per (tile, bucket)
    uint16_t* s_st = reinterpret_cast<uint16_t*>(dyn + 24 * (size_t)kPartTiles * nb);  // per tile: nb + 1
    uint8_t* s_bk = reinterpret_cast<uint8_t*>(dyn + 24 * (size_t)kPartTiles * nb +
                                               ((2 * (size_t)kPartTiles * (nb + 1) + 15) & ~size_t(15)));
    const uint32_t n = ne > cap_a ? 0u : (uint32_t)ne;  // a heavy tile stages nothing: all runs empty
    const int32_t* __restrict__ Ajt = Aj + ea;
    int32_t jj[kMaxE];  // feature | unit << 27 (staging needs m <= 2^26), -1 past the tile
#pragma unroll
    for (int i = 0; i < kMaxE; ++i) {
        const uint32_t e = qt + i * kBlock;
        jj[i] = e < n ? Ajt[e] : -1;
    }
    uint32_t* hu = s_key + (size_t)q * 4 * nb;  // unit histograms of this part's tile
    for (int i = qt; i < 4 * nb; i += kBlock) hu[i] = 0u;
    if (tid == 0) s_over = 0;
    __syncthreads();
    // the histogram's atomic returns each entry's rank inside its (unit, bucket) part (16 bits, two
    // per register): its place in the layout is then the part's start + rank, with no second
    // atomic (the order inside a part is the atomics' order either way; the wave kernel puts every
    // D word back at its entry index)
    uint32_t rk[kMaxE / 2] = {};
#pragma unroll
    for (int i = 0; i < kMaxE; ++i)
        if (jj[i] >= 0) {
            const uint32_t e = qt + i * kBlock;
            const uint32_t u = (e >= u1) + (e >= u2) + (e >= u3);
            jj[i] |= (int32_t)(u << 27);
            const uint32_t r = atomicAdd(&hu[u * nb + (((uint32_t)jj[i] & kW32J) >> sb)], 1u);
            rk[i >> 1] |= r << (16 * (i & 1));
        }
    __syncthreads();
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    if (qt < nb) {
        h0 = hu[qt];
        h1 = hu[nb + qt];
        h2 = hu[2 * nb + qt];
        h3 = hu[3 * nb + qt];
    }
    const uint32_t cnt = h0 + h1 + h2 + h3;
    // the super-tile's claim of bucket qt (part 0): issued now, consumed after the ranking
    uint32_t claim = 0, c4[kPartTiles] = {}, tot4 = 0;
    int64_t lo = 0, hi = 0;
    const unsigned sg = (t0 / kRunGroup) * (unsigned)nb + (unsigned)qt;
    if (q == 0 && qt < nb) {
#pragma unroll
        for (int k = 0; k < kPartTiles; ++k) {
            const uint32_t* hk = s_key + (size_t)k * 4 * nb;
            c4[k] = hk[qt] + hk[nb + qt] + hk[2 * nb + qt] + hk[3 * nb + qt];
            tot4 += c4[k];
        }
        if (tot4 > 0) {
            claim = atomicAdd(&FILL[sg], tot4);
            lo = GB[sg];
            hi = GB[sg + 1];
        }
    }
    // within-tile bucket starts: exclusive scan of cnt over the part's 256 threads
    const uint32_t inc = wave_incl_scan(cnt);
    if ((tid & 63) == 63) s_wsum[w] = inc;
    __syncthreads();  // also: every histogram read above is done (s_key is rewritten below)
    uint32_t st = inc - cnt;
    for (int i = 4 * q; i < w; ++i) st += s_wsum[i];
    uint32_t* cur = s_cur + (size_t)q * 4 * nb;
    if (qt < nb) {
        s_st[q * (nb + 1) + qt] = (uint16_t)st;
        cur[qt] = st;
        cur[nb + qt] = st + h0;
        cur[2 * nb + qt] = st + h0 + h1;
        cur[3 * nb + qt] = st + h0 + h1 + h2;
        if (live) {
            uint16_t* cu = CU + (size_t)t * 4 * ostride + qt;
            cu[0] = (uint16_t)h0;
            cu[ostride] = (uint16_t)(h0 + h1);
            cu[2 * ostride] = (uint16_t)(h0 + h1 + h2);
            cu[3 * ostride] = (uint16_t)cnt;
        }
    }
    if (qt == 0) s_st[q * (nb + 1) + nb] = (uint16_t)n;
    __syncthreads();
    const uint32_t mask = (1u << sb) - 1u;
    uint32_t* sk = s_key + (size_t)q * cap_a;
#pragma unroll
    for (int i = 0; i < kMaxE; ++i)
        if (jj[i] >= 0) {
            const uint32_t e = qt + i * kBlock;
            const uint32_t f = (uint32_t)jj[i] & kW32J;
            const uint32_t pos = cur[((uint32_t)jj[i] >> 27) * nb + (f >> sb)] + ((rk[i >> 1] >> (16 * (i & 1))) & 0xffffu);
            sk[pos] = (e << 20) | (f & mask);
            s_bk[(size_t)q * cap_a + pos] = (uint8_t)(f >> sb);
        }
    if (q == 0 && qt < nb) {  // the super-tile's runs of bucket qt, adjacent in tile order
        uint32_t run = claim;
        if (tot4 > 0 && lo + (int64_t)claim + tot4 > hi) s_over = 1;
#pragma unroll
        for (int k = 0; k < kPartTiles; ++k) {
            if (t0 + k < n_tiles) {
                s_dst[k * nb + qt] = lo + (int64_t)run - (int64_t)s_st[k * (nb + 1) + qt];
                OFF2[(size_t)(t0 + k) * ostride + qt] = run;
            }
            run += c4[k];
        }
    }
    __syncthreads();
    if (s_over) {  // uniform: a segment's reserve is exceeded
        if (tid == 0) *gate = 0;
        return;
    }
    const uint8_t* bkq = s_bk + (size_t)q * cap_a;
    for (uint32_t pos = qt; pos < n; pos += kBlock) S[s_dst[q * nb + bkq[pos]] + pos] = sk[pos];
}

// K3: gather, one workgroup per (bucket b, group g) segment, on XCD b % 8 (workgroup i
// runs on XCD i % 8, so one XCD's CUs work on one bucket at a time and its L2 holds that W32
// slice). The bucket's nonempty-feature bitmap (2^sb bits) is staged in LDS: an entry whose R row
// is empty (57% of KDD2012 entries) gets D = 0 without an L2 request, the others gather their
// W32 word. S in, D out: both streamed whole-line.
// 8 waves share one staged bitmap (64 KB at 2^19 features); 1024- or 256-thread workgroups and 4 or
// 16 entries per thread per round measured slower (§3d)
#ifndef RP_GATHER_BLOCK
#define RP_GATHER_BLOCK 512
#endif
constexpr int kGBlock = RP_GATHER_BLOCK;
#ifndef RP_GATHER_U
#define RP_GATHER_U 16
#endif
constexpr int kGatherU = RP_GATHER_U;  // words per thread per round
#ifndef RP_GATHER_MODE
#define RP_GATHER_MODE 0
#endif
__global__ void __launch_bounds__(kGBlock)
lpr_gather_kernel(const uint32_t* __restrict__ W32, const uint32_t* __restrict__ BM, const int64_t* __restrict__ GB,
                  const uint32_t* __restrict__ FILL, int sb, int nb, unsigned groups, const uint32_t* __restrict__ S,
                  uint32_t* __restrict__ D, const uint32_t* __restrict__ gate) {
    if (*gate == 0) return;
    extern __shared__ __align__(16) uint32_t s_bm[];  // 2^sb bits
    const unsigned xcd = blockIdx.x & 7u, k = blockIdx.x >> 3;
    const unsigned b = xcd + 8u * (k / groups);
    if (b >= (unsigned)nb) return;  // uniform
    const unsigned g = k % groups;
    const int64_t lo = GB[(size_t)g * nb + b], hi = lo + FILL[(size_t)g * nb + b];
    if (lo == hi) return;
    const uint32_t nwords = 1u << (sb - 5);
    const uint4* src = reinterpret_cast<const uint4*>(BM + ((size_t)b << (sb - 5)));
    for (uint32_t i = threadIdx.x; i < nwords / 4; i += kGBlock) reinterpret_cast<uint4*>(s_bm)[i] = src[i];
    __syncthreads();
    const uint32_t mask = (1u << sb) - 1u;
    // Straight-line rounds on raw buffers (no exec-mask branches: with a branch around every
    // conditional load the compiler drained vmcnt(0) before each lookup, 8 dependent L2 round
    // trips per round). The segment [lo, hi) as buffers from its line-aligned base: a word past hi
    // reads 0 / is not stored (out of range, no memory access), a word before lo (the previous
    // segment's tail in the first round) gets an out-of-range offset. Per round: the lookups of
    // round c (their S words arrived a round earlier), then the S loads of round c + 2, then the
    // D stores of round c: waiting for the lookups also drains only what round c - 1 issued, so
    // the stream loads and stores stay off the lookups' critical path. S and D non-temporal (keep
    // the W32 slice in L2).
    constexpr int kU = kGatherU;
    constexpr uint32_t kOob = 0x80000000u;
    const int64_t base = lo & ~int64_t(31);
    const uint32_t span = (uint32_t)((hi - base) * 4);
    const uint32_t skip = (uint32_t)((lo - base) * 4);  // bytes of the previous segment (< 128)
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)(S + base), (short)0, (int)span, 0x00020000);
    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc((void*)(D + base), (short)0, (int)span, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)(W32 + ((size_t)b << sb)), (short)0,
                                                                        (int)(4u << sb), 0x00020000);
    const uint32_t rounds = (span + 4u * kU * kGBlock - 1) / (4u * kU * kGBlock);
    auto off_of = [&](uint32_t c, int u) {  // byte offset of this lane's word u of round c
        const uint32_t o = 4u * ((c * kU + (uint32_t)u) * kGBlock + threadIdx.x);
        return o < skip ? kOob : o;
    };
    auto load_s = [&](uint32_t (&v)[kU], uint32_t c) {
#pragma unroll
        for (int u = 0; u < kU; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b32(sr, off_of(c, u), 0, 2);
    };
    // one round on the register set holding its S words; the set is then refilled with round c + 2
    // (two sets, the loop unrolled by two: no register copy of a pending load, which would make
    // the compiler wait for it)
    auto round = [&](uint32_t (&s)[kU], uint32_t c) {
        uint32_t w[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t col = s[u] & mask;
            const bool hit = (s_bm[col >> 5] >> (col & 31)) & 1u;  // a word past hi reads 0: any bit, not stored
#if RP_GATHER_MODE == 1
            uint32_t v = 0u;
            if (hit) v = __builtin_amdgcn_raw_buffer_load_b32(wr, col * 4u, 0, 0);
            w[u] = v;
#else
            w[u] = __builtin_amdgcn_raw_buffer_load_b32(wr, hit ? col * 4u : kOob, 0, 0);
#endif
        }
        load_s(s, c + 2);
#pragma unroll
        for (int u = 0; u < kU; ++u) __builtin_amdgcn_raw_buffer_store_b32(w[u], dr, off_of(c, u), 0, 2);
    };
    uint32_t s0[kU], s1[kU];
    load_s(s0, 0);
    load_s(s1, 1);
    for (uint32_t c = 0; c < rounds; c += 2) {  // a round past the end loads and stores nothing
        round(s0, c);
        round(s1, c + 1);
    }
}

// Tile slots to C after the scan of the tiles' counts (DeferSpace): grid-stride over the tiles;
// heavy tiles are written by tile_heavy_write_kernel.
template <typename T, typename OP, typename OI>
__global__ void __launch_bounds__(kBlock)
slot_copy_kernel(DeferSpace dfr, Caps caps, int64_t n_rows, unsigned n_tiles, OP* __restrict__ Cp,
                 OI* __restrict__ Cj, T* __restrict__ Cx, unsigned long long capacity) {
    const int tid = threadIdx.x;
    const T* vals = reinterpret_cast<const T*>(dfr.vals);
    for (unsigned tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const uint16_t* ro = dfr.hdr + (size_t)tile * (caps.rpt + 1);
        const int64_t row0 = (int64_t)tile * caps.rpt;
        const int nrows = (int)std::min<int64_t>(caps.rpt, n_rows - row0);
        const unsigned long long G = dfr.toff[tile];
        const uint32_t cnt = dfr.tcnt[tile];
        if (tile == n_tiles - 1 && tid == 0) Cp[n_rows] = (OP)(G + cnt);
        if (ro[nrows] == kHdrHeavy) continue;  // uniform
        for (int r = tid; r < nrows; r += kBlock) Cp[row0 + r] = (OP)(G + ro[r]);
        if (G + cnt <= capacity) {  // four entries per thread loaded before any is stored
            const uint16_t* __restrict__ sc = dfr.cols + (size_t)tile * dfr.slot;
            const T* __restrict__ sv = vals + (size_t)tile * dfr.slot;
            constexpr int kU = 4;
            for (uint32_t q0 = 0; q0 < cnt; q0 += kU * kBlock) {
                uint16_t cv[kU];
                T xv[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const uint32_t q = std::min(q0 + u * kBlock + tid, cnt - 1);
                    cv[u] = __builtin_nontemporal_load(sc + q);
                    xv[u] = __builtin_nontemporal_load(sv + q);
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const uint32_t q = q0 + u * kBlock + tid;
                    if (q < cnt) {
                        Cj[G + q] = (OI)cv[u];
                        Cx[G + q] = xv[u];
                    }
                }
            }
        }
    }
}

// Heavy tiles of the slot mode: the exact slow path counts again, then writes at the scanned offset.
template <typename T, typename IP, typename OP, typename OI, typename RL>
__global__ void __launch_bounds__(kBlock)
tile_heavy_write_kernel(RL R, T mag, int p, int64_t n_rows, const IP* __restrict__ Ap, const int32_t* __restrict__ Aj,
                        const T* __restrict__ Ax, OP* __restrict__ Cp, OI* __restrict__ Cj, T* __restrict__ Cx,
                        unsigned long long capacity, Caps caps, int order, Workspace* ws, DeferSpace dfr) {
    extern __shared__ __align__(16) unsigned char lds[];
    __shared__ uint32_t s_wsum[kBlock / 64];
    const unsigned nh = ws->n_deferred;
    uint32_t* s_rowc = reinterpret_cast<uint32_t*>(lds + heavy_lds_bytes(p, sizeof(T)) - 4 * kBlock);
    for (unsigned i = blockIdx.x; i < nh; i += gridDim.x) {
        const unsigned tile = dfr.list[i];
        const int64_t row0 = (int64_t)tile * caps.rpt;
        const int nrows = (int)std::min<int64_t>(caps.rpt, n_rows - row0);
        const unsigned long long G = dfr.toff[tile];
        heavy_tile<T, IP, OP, OI, RL>(R, mag, Ap, Aj, Ax, row0, nrows, p, lds, s_rowc, s_wsum, 0, 0, Cp, Cj, Cx,
                                      false, order);
        heavy_tile<T, IP, OP, OI, RL>(R, mag, Ap, Aj, Ax, row0, nrows, p, lds, s_rowc, s_wsum, 1, G, Cp, Cj, Cx,
                                      G + dfr.tcnt[tile] <= capacity, order);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Row-lane pipeline (packed R, short rows — KDD2012: 11 entries, 6 products/row).
// No look-back and no waiting: every wave's output goes to a fixed slot, then one scan and one copy.
//   lpr_main_kernel   one workgroup per tile of 256 rows, one wave per 64 rows. The tile's R
//                     descriptors (gathered from W directly, or the staged W32 words of
//                     lpr_partition/lpr_gather) land in LDS by entry; then each wave runs ONE
//                     flat pass over its entries (64 consecutive entries per step, no divergence):
//                     row of an entry from a row-start bitmap (popcount), its products, their kept
//                     prefix (wave scan) = their place in the wave's slot in first-touch order, and
//                     per row a product count and a 3 x 64-bit column signature (LDS atomics).
//                     A row whose signature cannot rule out a repeated column (~0.5% real repeats,
//                     ~1% false alarms) is recomputed by its lane exactly (LDS scratch: leaders sum
//                     their column group in sequence order) into the same slot range.
//   lpr_heavy_*       tiles beyond a cap (entries, side table, scratch, slot): the exact dense
//                     accumulator (heavy_tile) counts, then writes them in place.
//   lpr_scan_kernel   exclusive scan of the per-wave counts (decoupled look-back, 4096 per block)
//   lpr_copy_kernel   slots -> C: each row reversed (scipy's reverse first-touch order) or as is
//                     (ascending, sorted in the slot), indptr from the per-row counts.
// Per-row semantics are scipy's csr_matmat exactly: first touch = product order, sums start at +0
// and add in product order, sum != 0 kept.
constexpr int kLprRows = 256;      // rows per tile (4 waves x 64 rows)
constexpr int kLprSide = 96;       // features with > 2 R entries per tile (KDD2012: 56 +- 7.5; more -> heavy)
constexpr int kLprFlagWords = kCapAMax / 64 + 1;  // row-start bitmap words per wave

struct LprSpace {
    uint32_t* cnt;        // 4 x n_tiles: kept entries of each wave (slot fill)
    unsigned long long* off;  // 4 x n_tiles: exclusive prefix of cnt (+ base)
    uint32_t* hlist;      // heavy tiles, count in ws->n_deferred
    uint32_t* tflag;      // n_tiles: 1 = heavy (lpr_heavy_write places the tile)
    uint32_t* rowmeta;    // n_tiles x 256: the row's slot range, kst | kept << 16 (lpr_store_slot)
    uint16_t* cols;       // 4 x n_tiles x slot
    unsigned char* vals;  // 4 x n_tiles x slot x sizeof(T)
    unsigned long long* scan_state;  // one per 4096-wave scan block
    uint32_t slot;        // kept-entry capacity of one wave (a multiple of 32)
};

constexpr int kAuxNT = 2;  // buffer instruction cache policy: nt (gfx950)

__device__ __forceinline__ uint32_t lpr_h2(uint32_t col) { return (col * 0x9E3779B1u) >> 26; }

// Bloom check of one row's slot range [kst, kst + n): 3 x 64-bit filters in registers; true if a
// column finds its three bits already set by an earlier one (every real repeat does; false alarms
// ~ (i/64)^3 for the i-th product). Columns are read four at a time (four LDS loads in flight per
// round trip instead of one); a row without slot entries (n = 0) checks nothing.
__device__ __forceinline__ bool lpr_bloom(const uint16_t* cb, uint32_t kst, uint32_t n) {
    uint64_t b0 = 0, b1 = 0, b2 = 0;
    bool hit = false;
    for (uint32_t q0 = 0; q0 < n; q0 += 4) {
        uint32_t c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = q0 + u < n ? (uint32_t)cb[kst + q0 + u] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (q0 + u < n) {
                const uint32_t col = c[u];
                const uint64_t m0 = 1ull << (col & 63), m1 = 1ull << ((col >> 6) & 63), m2 = 1ull << lpr_h2(col);
                hit |= (b0 & m0) && (b1 & m1) && (b2 & m2);
                b0 |= m0;
                b1 |= m1;
                b2 |= m2;
            }
    }
    return hit;
}

// Exact repeat check of one row's slot range [kst, kst + n) (the staged wave kernel): every pair of
// its first 16 columns compared in registers (120 compares, straight-line, no false alarms: ~1/3
// of the round-5 3 x 64-bit Bloom check's VALU, which also flagged ~1% of the rows for nothing); a row of more than 16
// products is flagged (the exact path handles it). Columns past n are distinct sentinels.
__device__ __forceinline__ bool lpr_repeat16(const uint16_t* cb, uint32_t kst, uint32_t n, uint32_t lim) {
    uint32_t c[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t v = cb[std::min(kst + (uint32_t)i, lim)];
        c[i] = (uint32_t)i < n ? v : 0x10000u + (uint32_t)i;
    }
    bool rep = n > 16;
#pragma unroll
    for (int i = 1; i < 16; ++i)
#pragma unroll
        for (int j = 0; j < i; ++j) rep |= c[i] == c[j];
    return rep;
}

// A wave's slot to HBM (row r's kept entries at [kst, kst + kept), in first-touch order, or
// ascending for RP_ORDER_SORTED): `extent` entries copied coalesced, each row's (kst, kept) in
// rowmeta, the run's entry count in *cnt. A slot without gaps (every row with entries starts at
// the kept count of the rows before it: the usual case) is stored in its final order, each row
// reversed here for scipy's reverse first-touch order, and the copy kernel moves it as one run;
// a slot with gaps (entries the exact path merged or dropped) is stored as built, and the copy
// kernel finds each output's row and reverses it there. Both kernels apply the same test
// (lpr_slot_final).
// unit slots hold a multiple of 64 entries (whole 128-B lines of columns and of values) and are
// stored as whole lines (the padding past the kept entries included): no line of a slot is written
// partially (14.25-14.31 -> 14.14-14.22 ms per configs[1] pass, same box)
constexpr uint32_t kSlotRound = 64u;
__device__ __forceinline__ bool lpr_slot_final(uint32_t c, uint32_t kst, uint32_t pre) {
    return __ballot(c > 0 && kst != pre) == 0;
}
template <typename T>
__device__ __forceinline__ uint32_t lpr_store_slot(uint16_t* cb, T* vb, uint32_t kst, uint32_t kept,
                                                   bool valid, int lane, uint32_t extent, int order,
                                                   uint32_t* __restrict__ rowmeta, uint32_t* __restrict__ cnt,
                                                   uint16_t* __restrict__ oc, T* __restrict__ ov) {
    const uint32_t c = valid ? kept : 0u;
    const uint32_t incl = wave_scan_dpp(c);
    const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
    if (order != RP_ORDER_SORTED && lpr_slot_final(c, kst, incl - c)) {
        const uint32_t half = c >> 1;
        for (uint32_t i = 0; __ballot(i < half); ++i)
            if (i < half) {
                const uint32_t a = kst + i, b = kst + c - 1 - i;
                const uint16_t ca = cb[a], cz = cb[b];
                const T va = vb[a], vz = vb[b];
                cb[a] = cz;
                cb[b] = ca;
                vb[a] = vz;
                vb[b] = va;
            }
        __builtin_amdgcn_wave_barrier();
    }
    // 16 bytes per lane and store (8 columns, 16 / sizeof(T) values), non-temporal. A wave's slot
    // regions start 128-B aligned and hold slot (a multiple of 64) entries: the tail rounded up to
    // whole lines stays inside them (extent <= slot: a fuller unit went heavy before its store).
    if (valid) rowmeta[lane] = kst | (c << 16);
    if (lane == 0) *cnt = tot;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)oc, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)ov, (short)0, 0x7fffffff, 0x00020000);
    const uint32_t ext_c = (extent + 63) & ~63u;  // whole 128-B lines (the slot holds a multiple of 64 entries)
    const uint32_t ext_v = (extent + 128u / (uint32_t)sizeof(T) - 1u) & ~(128u / (uint32_t)sizeof(T) - 1u);
    for (uint32_t o = 8 * lane; o < ext_c; o += 512)
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u*>(cb + o), rc, 2 * o, 0, kAuxNT);
    constexpr uint32_t kPer = 16 / sizeof(T);
    for (uint32_t o = kPer * lane; o < ext_v; o += 64 * kPer)
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u*>(vb + o), rv, (uint32_t)sizeof(T) * o, 0,
                                               kAuxNT);
    return tot;
}

// products of an entry with LDS descriptor d: bits 30-31 = n <= 2 inline 15-bit slots (sign << 14 |
// col) in R's storage order; n = 3: the W word in side[d & mask] (<= 4 inline, or an O record).
// t-th product's (sign << 14 | col)
__device__ __forceinline__ uint32_t lpr_slot(uint32_t d, uint32_t t, const uint64_t* side, const uint16_t* O) {
    if ((d >> 30) < 3) return (d >> (15 * t)) & 0x7fffu;
    const uint64_t w = side[d & kW32J];
    if ((w >> 61) != 7) return (uint32_t)(w >> (15 * t)) & 0x7fffu;
    const uint32_t e = O[(w & kLow61) + 1 + t];
    return ((e & 0x8000u) >> 1) | (e & 0x3fffu);
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan_t(T v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}


// staged runs of the row-lane pipeline (see lpr_partition_kernel)
struct LprStage {
    const uint32_t* gate;  // staged iff *gate (a segment overflow in the partition clears it)
    const uint32_t* w32;   // W32 table: direct gathers (NULL: the 8-byte W words)
    const uint32_t* off2;
    const uint16_t* cu;
    const int64_t* gb;
    const uint32_t* s;
    const uint32_t* d;
    uint32_t ostride;
    int nb;
};

// One workgroup per tile, no persistence (direct gathers: the two dependent rounds, feature ids
// then W words, are cheaper to hide with more resident tiles than with cross-tile pipelining;
// measured: power-law direct main kernel 12.4 ms here vs 15.3 ms persistent). Launched when the
// call takes direct gathers (the host read lpr_choose_kernel's verdict, or staging is off).
template <typename T, typename IP>
__global__ void __launch_bounds__(kLprRows)
lpr_main_flat_kernel(PackedR R, T mag, int64_t n_rows, const IP* __restrict__ Ap, const int32_t* __restrict__ Aj,
                const T* __restrict__ Ax, const uint32_t* __restrict__ w32, int cap_a, unsigned n_tiles, unsigned t8,
                int order, LprSpace sp, Workspace* ws) {
    extern __shared__ __align__(16) unsigned char lds[];          // s_desc[cap_a] u32
    __shared__ uint16_t s_rowptr[kLprRows + 1];
    __shared__ uint64_t s_side[kLprSide];
    __shared__ uint32_t s_sidej[kLprSide];                          // side entry's SW index (W32 gathers)
    __shared__ uint16_t s_sfk[kLprSide];                            // side entry's slot position
    __shared__ uint8_t s_sfw[kLprSide];                             // ... in the slot of this wave
    __shared__ T s_sfx[kLprSide];                                   // ... and its value
    __shared__ uint64_t s_flag[4][kLprFlagWords];                  // row-start bitmap per wave
    __shared__ uint64_t s_susp[4];                                  // rows flagged for the exact path
    __shared__ uint16_t s_kst[4][64];
    __shared__ uint8_t s_nz2row[4][64];
    __shared__ uint32_t s_nside, s_scr[4];
    __shared__ int s_bad;
    uint32_t* s_desc = reinterpret_cast<uint32_t*>(lds);
    uint16_t* s_colbuf = reinterpret_cast<uint16_t*>(lds + ((4 * (size_t)cap_a + 15) & ~size_t(15)));  // 4 x slot
    T* s_valbuf = reinterpret_cast<T*>(lds + ((4 * (size_t)cap_a + 15) & ~size_t(15)) +
                                       ((8 * (size_t)sp.slot + 15) & ~size_t(15)));                // 4 x slot

    const unsigned tile = xcd_tile(blockIdx.x, t8);
    if (tile >= n_tiles) return;  // uniform
    const int tid = threadIdx.x;
    const int64_t row0 = (int64_t)tile * kLprRows;
    const int nrows = (int)std::min<int64_t>(kLprRows, n_rows - row0);
    const int64_t ea = (int64_t)Ap[row0];
    const int64_t ne64 = (int64_t)Ap[row0 + nrows] - ea;
    // this wave's entry range [E0, E1) (wave-uniform) and the row pointers, all in the first round
    const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t E0 = (uint32_t)((int64_t)Ap[row0 + std::min(64 * wu, nrows)] - ea);
    const uint32_t E1 = (uint32_t)((int64_t)Ap[row0 + std::min(64 * wu + 64, nrows)] - ea);
    const int64_t rp0 = tid <= nrows ? (int64_t)Ap[row0 + tid] : 0;
    const int64_t rp1 = tid == 0 && nrows == kLprRows ? (int64_t)Ap[row0 + kLprRows] : 0;
    if (tid == 0) {
        s_nside = 0;
        s_bad = ne64 > cap_a;
    }
    if (tid < 4) s_scr[tid] = 0;
    __syncthreads();
    auto go_heavy = [&]() {  // one lane of the tile: the heavy path takes the whole tile
        if (atomicOr(&sp.tflag[tile], 1u) == 0u) sp.hlist[atomicAdd(&ws->n_deferred, 1u)] = tile;
    };
    if (s_bad) {  // uniform: too many entries for the tile's LDS
        if (tid == 0) go_heavy();
        return;
    }
    const uint32_t ne = (uint32_t)ne64;
    // the flat pass's first values (entry order, coalesced) in flight together with step A's loads;
    // unconditional loads (index clamped, value masked): straight-line vmcnt accounting
    const T* __restrict__ Axw = Ax + ea;
    const uint32_t elast = E1 > E0 ? E1 - 1 : E0;
    auto ldx = [&](uint32_t j) {
        const uint32_t e = E0 + 64 * j + (tid & 63);
        const T v = Axw[std::min(e, elast)];
        return e < E1 ? v : T(0);
    };
    T x0 = ldx(0), x1 = ldx(1), x2 = ldx(2), x3 = ldx(3);
    // ---- step A: R descriptors of the tile's entries into LDS, by entry
    // LDS descriptor of an entry: n <= 2 -> the W32 form (count, two inline 15-bit slots);
    // more entries -> code 3 | count (4 bits) << 26 | side index: the feature's W word lands in
    // s_side[k] (8-byte W gathers: now; W32 gathers: from SW after step A, needed only after the
    // flat pass)
    auto put_side = [&](uint32_t e, uint32_t c4, uint32_t j_or_0, uint64_t w, bool have_w) {
        const uint32_t k = atomicAdd(&s_nside, 1u);
        if (k < (uint32_t)kLprSide) {
            if (have_w) s_side[k] = w;
            s_sidej[k] = j_or_0;
        } else {
            s_bad = 1;
        }
        s_desc[e] = 0xc0000000u | (c4 << 26) | k;
    };
    auto put_desc = [&](uint32_t e, uint64_t w) {  // direct mode: the W word itself
        const uint32_t n = (uint32_t)(w >> 61);
        if (n <= 2) s_desc[e] = (n << 30) | (uint32_t)(w & 0x3fffffffu);
        else put_side(e, std::min(n != 7 ? n : (uint32_t)R.O[w & kLow61], 15u), 0u, w, true);
    };
    constexpr int kU = 12;  // loads of a round issued before any is used
    {
        const int32_t* __restrict__ Ajt = Aj + ea;
        for (uint32_t q0 = tid; q0 < ne; q0 += kU * kLprRows) {
            int32_t jv[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint32_t e = q0 + u * kLprRows;
                jv[u] = e < ne ? Ajt[e] : -1;
            }
            if (w32) {  // the 4-byte W32 words: twice the features per line; > 2 entries -> side
                uint32_t w[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) w[u] = jv[u] >= 0 ? w32[jv[u]] : 0u;
#pragma unroll
                for (int u = 0; u < kU; ++u)
                    if (q0 + u * kLprRows < ne) {
                        if ((w[u] >> 30) == 3) put_side(q0 + u * kLprRows, (w[u] >> 26) & 15u, w[u] & kW32J, 0ull, false);
                        else s_desc[q0 + u * kLprRows] = w[u];
                    }
            } else {
                uint64_t w[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) w[u] = jv[u] >= 0 ? R.W[jv[u]] : 0ull;
#pragma unroll
                for (int u = 0; u < kU; ++u)
                    if (q0 + u * kLprRows < ne) put_desc(q0 + u * kLprRows, w[u]);
            }
        }
    }
    if (tid <= nrows) s_rowptr[tid] = (uint16_t)(rp0 - ea);
    if (tid == 0 && nrows == kLprRows) s_rowptr[kLprRows] = (uint16_t)(rp1 - ea);
    __syncthreads();
    if (s_bad) {  // uniform: side table full
        if (tid == 0) go_heavy();
        return;
    }
    // W32 gathers: the W words of the side entries are gathered now (from the side table) and
    // only needed after the flat pass (their counts came with the W32 words)
    const uint32_t nside = s_nside;
    uint64_t sidew = 0;
    const bool side_later = w32 != nullptr;  // side W words not in LDS yet
    if (side_later && (uint32_t)tid < nside) sidew = R.SW[s_sidej[tid]];
    // ---- step B: one wave per 64 rows, one flat pass over the wave's entries
    const int w = tid >> 6, lane = tid & 63;
    const int r = tid;  // this lane's row (for per-row work)
    const bool valid = r < nrows;
    const uint32_t rs = valid ? s_rowptr[r] : 0u, re = valid ? s_rowptr[r + 1] : 0u;
    const uint32_t nsteps = (E1 - E0 + 63) >> 6;
    for (uint32_t k = lane; k < nsteps; k += 64) s_flag[w][k] = 0ull;
    if (lane == 0) s_susp[w] = 0ull;
    __builtin_amdgcn_wave_barrier();
    const bool nonempty = re > rs;
    const uint64_t ne_mask = __ballot(nonempty);
    if (nonempty) {
        const uint32_t b = rs - E0;
        atomicOr(reinterpret_cast<unsigned long long*>(&s_flag[w][b >> 6]), 1ull << (b & 63));
        s_nz2row[w][__builtin_popcountll(ne_mask & ((1ull << lane) - 1))] = (uint8_t)lane;
    }
    __builtin_amdgcn_wave_barrier();
    // the wave's slot is built in LDS (columns cb, values vb, first-touch order) and stored to
    // HBM with coalesced stores at the end: no global store inside the pass, so the compiler's
    // vmcnt accounting keeps the value prefetch in flight
    uint16_t* cb = s_colbuf + (size_t)w * sp.slot;
    T* vb = s_valbuf + (size_t)w * sp.slot;
    uint32_t carry_r = 0, carry_k = 0;
    auto step = [&](uint32_t j, T x) {
        const uint32_t e = E0 + 64 * j + lane;
        const bool ve = e < E1;
        const uint64_t fw = s_flag[w][j];
        const uint32_t nr = carry_r + (uint32_t)__builtin_popcountll(fw & ((2ull << lane) - 1)) - 1u;
        const uint32_t row = s_nz2row[w][nr & 63];
        const uint32_t d = ve ? s_desc[e] : 0u;
        const uint32_t n = d >> 30;
        const uint32_t np = n < 3 ? n : (d >> 26) & 15u;  // n == 3: a side entry (count in the word)
        // all products of an entry are +-(x * mag) (x * -mag is -(x * mag) exactly; a kept product
        // is nonzero, so scipy's 0 + it is itself)
        const T xm = tmul<T>(x, mag);
        const bool nzx = xm != T(0);
        const uint32_t kc = nzx ? np : 0u;
        const uint32_t kinc = wave_scan_dpp(kc);
        const uint32_t K = carry_k + kinc - kc;
        if (ve && ((fw >> lane) & 1ull)) s_kst[w][row] = (uint16_t)K;  // the row's first entry
        const uint32_t sl0 = d & 0x7fffu, sl1 = (d >> 15) & 0x7fffu;
        if (n < 3 && kc >= 1 && K < sp.slot) {
            cb[K] = (uint16_t)(sl0 & 0x3fffu);
            vb[K] = (sl0 & 0x4000u) ? -xm : xm;
        }
        if (n < 3 && kc >= 2 && K + 1 < sp.slot) {
            cb[K + 1] = (uint16_t)(sl1 & 0x3fffu);
            vb[K + 1] = (sl1 & 0x4000u) ? -xm : xm;
        }
        // side entries keep a gap [K, K + np) in the slot, filled after the pass (their W words
        // may still be in flight); a zero product is not in the slot: its row takes the exact path
        if (n == 3) {
            const uint32_t k = d & kW32J;
            s_sfk[k] = kc ? (uint16_t)K : (uint16_t)0xffffu;
            s_sfw[k] = (uint8_t)w;
            s_sfx[k] = x;
            if (np == 15) s_bad = 1;  // 15 or more entries: the count is not exact -> heavy tile
        }
        if (ve && np > 0 && !nzx) atomicOr(reinterpret_cast<unsigned long long*>(&s_susp[w]), 1ull << row);
        carry_k += __builtin_amdgcn_readlane(kinc, 63);
        carry_r += (uint32_t)__builtin_popcountll(fw);
    };
    // values straight from HBM in entry order (coalesced), four steps in flight ahead of use, in
    // two alternating register sets (no copy at the loop edge: see lpr_main_kernel)
    for (uint32_t j = 0; j < nsteps; j += 8) {
        const T y0 = ldx(j + 4), y1 = ldx(j + 5), y2 = ldx(j + 6), y3 = ldx(j + 7);
        step(j, x0);
        if (j + 1 < nsteps) step(j + 1, x1);
        if (j + 2 < nsteps) step(j + 2, x2);
        if (j + 3 < nsteps) step(j + 3, x3);
        if (j + 4 >= nsteps) break;  // uniform
        x0 = ldx(j + 8);
        x1 = ldx(j + 9);
        x2 = ldx(j + 10);
        x3 = ldx(j + 11);
        step(j + 4, y0);
        if (j + 5 < nsteps) step(j + 5, y1);
        if (j + 6 < nsteps) step(j + 6, y2);
        if (j + 7 < nsteps) step(j + 7, y3);
    }
    bool overflow = carry_k > sp.slot;
    __syncthreads();
    // side fill: every side entry's products into its gap, in R's storage order
    if ((uint32_t)tid < nside) {
        const uint64_t sw = side_later ? sidew : s_side[tid];
        if (side_later) s_side[tid] = sw;
        const uint32_t k0 = s_sfk[tid];
        if (k0 != 0xffffu) {
            uint16_t* cbw = s_colbuf + (size_t)s_sfw[tid] * sp.slot;
            T* vbw = s_valbuf + (size_t)s_sfw[tid] * sp.slot;
            const T x = s_sfx[tid];
            const bool rec = (sw >> 61) == 7;
            const uint32_t np = rec ? R.O[sw & kLow61] : (uint32_t)(sw >> 61);
            for (uint32_t t = 0; t < np && k0 + t < sp.slot; ++t) {
                uint32_t sl;
                if (rec) {
                    const uint32_t e = R.O[(sw & kLow61) + 1 + t];
                    sl = ((e & 0x8000u) >> 1) | (e & 0x3fffu);
                } else {
                    sl = (uint32_t)(sw >> (15 * t)) & 0x7fffu;
                }
                cbw[k0 + t] = (uint16_t)(sl & 0x3fffu);
                vbw[k0 + t] = tadd<T>(T(0), tmul<T>(x, (sl & 0x4000u) ? -mag : mag));
            }
        }
    }
    __syncthreads();
    if (s_bad) {  // uniform: a side entry with 15 or more products
        if (tid == 0) go_heavy();
        return;
    }
    // ---- per row: kept count and a Bloom check of its columns (3 x 64-bit filters in registers):
    // a column whose 3 bits are all set already flags the row for the exact path (every real
    // repeat does; false alarms ~ (i/64)^3 for the i-th product)
    const uint32_t kst = nonempty ? s_kst[w][lane] : 0u;
    const uint64_t after = ne_mask & ~((2ull << lane) - 1);  // the next non-empty row ends this one
    const int nxt = after ? __builtin_ctzll(after) : 64;
    const uint32_t kst_next = __shfl(kst, nxt & 63, 64);
    const uint32_t kend = nxt < 64 ? kst_next : carry_k;
    uint32_t kept = nonempty ? kend - kst : 0u;
    bool hit = false;
    if (!overflow) hit = lpr_bloom(cb, kst, kept);
    const uint64_t susp = s_susp[w];
    uint64_t todo = susp | __ballot(hit);  // lane == row within the wave
    __builtin_amdgcn_wave_barrier();  // the row-start bitmap is dead from here: the scratch reuses it
    constexpr int kScr = (int)((kLprFlagWords * 8 - 16) / (2 + sizeof(T)));
    uint16_t* scol = reinterpret_cast<uint16_t*>(&s_flag[w][0]);
    T* sval = reinterpret_cast<T*>(reinterpret_cast<unsigned char*>(&s_flag[w][0]) + ((2 * kScr + 15) & ~15));
    if (__ballot(overflow)) todo = 0;
    // exact path, one flagged row at a time, the whole wave on it: its products in sequence order,
    // then every product checks for an earlier one of its column (first touch); a leader sums its
    // group in order; kept leaders land in the row's slot range in that order. A Bloom-flagged row
    // is read from its slot range (64 products or fewer: one round, reads before writes); a row
    // with a zero value rebuilds its products into the scratch (as lpr_wave_kernel)
    while (todo) {
        const int R0 = __builtin_ctzll(todo);
        todo &= todo - 1;
        const uint32_t a0 = __shfl(rs, R0, 64), a1 = __shfl(re, R0, 64), kR = __shfl(kst, R0, 64);
        const uint32_t kE = __shfl(kend, R0, 64);
        const bool from_slot = !((susp >> R0) & 1ull) && kE - kR <= 64u;  // uniform
        const uint16_t* pc = from_slot ? cb + kR : scol;
        const T* pv = from_slot ? vb + kR : sval;
        uint32_t nprod = from_slot ? kE - kR : 0u;
        for (uint32_t e0 = a0; !from_slot && e0 < a1; e0 += 64) {
            const uint32_t e = e0 + lane;
            const bool in = e < a1;
            const uint32_t d = in ? s_desc[e] : 0u;
            const T x = in ? Axw[e] : T(0);
            const uint32_t np = in ? ((d >> 30) < 3 ? (d >> 30) : (d >> 26) & 15u) : 0u;
            const uint32_t inc = wave_scan_dpp(np);
            const uint32_t q0 = nprod + inc - np;
            for (uint32_t t = 0; t < np; ++t)
                if (q0 + t < (uint32_t)kScr) {
                    const uint32_t sl = lpr_slot(d, t, s_side, R.O);
                    scol[q0 + t] = (uint16_t)(sl & 0x3fffu);
                    sval[q0 + t] = tmul<T>(x, (sl & 0x4000u) ? -mag : mag);
                }
            nprod += __builtin_amdgcn_readlane(inc, 63);
        }
        if (nprod > (uint32_t)kScr) {
            overflow = true;
            break;
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t nk = 0;
        for (uint32_t q0 = 0; q0 < nprod; q0 += 64) {
            const uint32_t q = q0 + lane;
            bool lead = q < nprod;
            T sum = T(0);
            uint16_t cq = 0;
            if (lead) {
                cq = pc[q];
                for (uint32_t b = 0; b < q && lead; ++b) lead = pc[b] != cq;
                if (lead) {
                    sum = tadd<T>(T(0), pv[q]);
                    for (uint32_t b = q + 1; b < nprod; ++b)
                        if (pc[b] == cq) sum = tadd<T>(sum, pv[b]);
                }
            }
            const bool keep = lead && sum != T(0);
            const uint32_t ki = wave_scan_dpp(keep ? 1u : 0u);
            if (keep) {
                if (kR + nk + ki - 1 >= sp.slot) overflow = true;
                else {
                    cb[kR + nk + ki - 1] = cq;
                    vb[kR + nk + ki - 1] = sum;
                }
            }
            nk += __builtin_amdgcn_readlane(ki, 63);
        }
        if (lane == R0) kept = nk;
        __builtin_amdgcn_wave_barrier();
    }
    // a row that gained entries in the exact path (its side entries were not in the slot) must
    // still end before the next row's range
    if (kst + kept > kend && nonempty) overflow = true;
    if (__ballot(overflow)) {  // this wave cannot finish on the fast path: the whole tile goes heavy
        if (lane == 0) go_heavy();
        return;
    }
    if (order == RP_ORDER_SORTED && kept > 1) {  // ascending columns inside the row's slot range
        for (uint32_t a = kst + 1; a < kst + kept; ++a) {
            const uint16_t kc = cb[a];
            const T kv = vb[a];
            uint32_t b = a;
            while (b > kst && cb[b - 1] > kc) {
                cb[b] = cb[b - 1];
                vb[b] = vb[b - 1];
                --b;
            }
            cb[b] = kc;
            vb[b] = kv;
        }
    }
    __builtin_amdgcn_wave_barrier();
    const size_t wt = (size_t)tile * 4 + w;
    lpr_store_slot<T>(cb, vb, kst, kept, valid, lane, carry_k, order, sp.rowmeta + (size_t)tile * kLprRows + 64 * w,
                      sp.cnt + wt, sp.cols + wt * sp.slot, reinterpret_cast<T*>(sp.vals) + wt * sp.slot);
}


// ------------------------------------------------------------------------------------------
// Staged row-lane wave kernel, the uniform-column default: one 64-thread
// workgroup = one wave = one 64-row unit, independent of every other wave (no block barrier, full
// occupancy). Round 1: the unit's row pointers and its part of the tile's run table (per bucket:
// OFF2 + the unit's cumulative counts CU). Round 2: the S and D words of its parts of the runs
// (bucket order; a super-tile's units read neighbouring parts of the same lines on one XCD) and
// its values, all in flight together; each D word is put back in entry order by its S word's entry
// index (LDS), then every lane holds its entries' descriptors in registers. The flat pass then
// runs from registers: per step, an entry's row from the row-start bitmap, its products' kept
// prefix (DPP scan) = their place in the slot, in first-touch order. Side entries (> 2 R entries)
// keep a gap, filled after the pass from their side-table words. Row phase: Bloom check, exact
// path for flagged rows, optional sort, row metadata, the slot stored coalesced.
// A call whose partition overflowed a segment's reserve (gate 0) runs this kernel with direct
// gathers: the unit's feature ids, then their W32 words.
// (Round 4 ran an unsort kernel between the gather and this kernel: every descriptor written back
// to HBM in entry order and read again, 10.6 GB per configs[1] pass)
constexpr int kWaveSteps = 16;                 // entries per unit on the fast path: 16 x 64 (KDD2012: 704)
// side entries (features with > 2 R entries, 1.9% of KDD2012's) per unit beyond this -> heavy tile.
// Poisson tails: a 704-entry unit has 13.3 on average; 32 was exceeded by ~7 of 1.87M units per
// configs[1] pass (4e-6 each), and 6 heavy tiles cost 1.6 ms; past 64: ~1e-24.
constexpr int kWaveSide = 64;
constexpr int kWaveScr = 128;                  // exact-path scratch (products of one row)
// dynamic LDS: region A = the unit's descriptors (ucap words, entry order), later the slot's
// columns + values (every descriptor is in registers before the first slot store); region B = the
// run lookup (start bitmap, run offsets), later the exact-path scratch
__host__ __device__ inline size_t lpr_wave_region_a(uint32_t slot, size_t vs, uint32_t ucap) {
    // (+2: the flat pass's clamped product stores past a full slot)
    const size_t s = ((2 * ((size_t)slot + 2) + 15) & ~size_t(15)) + ((vs * ((size_t)slot + 2) + 15) & ~size_t(15));
    return std::max(s, 4 * (size_t)ucap);
}
__host__ __device__ inline size_t lpr_wave_lds_bytes(uint32_t slot, size_t vs, uint32_t ucap, int nb) {
    const size_t scr = std::max(((2 * (size_t)kWaveScr + 15) & ~size_t(15)) + vs * kWaveScr,
                                (2 + vs + 4) * (size_t)kWaveSide);  // exact scratch / side list
    const size_t tab = (8 * (size_t)kWaveSteps + 4 * (size_t)std::max(nb, 1) + 15) & ~size_t(15);
    // a multiple of 16 bytes: the next wave's regions (8-byte bitmap words, f64 values) stay aligned
    return lpr_wave_region_a(slot, vs, ucap) + std::max(scr, tab);
}
// t-th product's (sign << 14 | col) of an entry with descriptor d (code 3: side-table word)
__device__ __forceinline__ uint32_t lpr_slot_sw(uint32_t d, uint32_t t, const uint64_t* SW, const uint16_t* O) {
    if ((d >> 30) < 3) return (d >> (15 * t)) & 0x7fffu;
    const uint64_t w = SW[d & kW32J];
    if ((w >> 61) != 7) return (uint32_t)(w >> (15 * t)) & 0x7fffu;
    const uint32_t e = O[(w & kLow61) + 1 + t];
    return ((e & 0x8000u) >> 1) | (e & 0x3fffu);
}
// v[x] for a runtime x (unrolled selects: no dynamic register indexing, no scratch; the empty asm
// keeps the compiler from folding the selects back into an indexed load of a stack copy)
template <int N>
__device__ __forceinline__ uint32_t reg_pick(const uint32_t (&v)[N], uint32_t x) {
    uint32_t r = v[0];
#pragma unroll
    for (int i = 1; i < N; ++i) {
        uint32_t t = v[i];
        __asm__("" : "+v"(t));
        r = (uint32_t)i == x ? t : r;
    }
    return r;
}
// f32: built for 7 waves per SIMD (72 VGPRs: the S/D words and the values in flight together; LDS
// allows ~29 one-wave workgroups per CU anyway; 8 waves in 64 VGPRs measured slower, §3d); f64
// unconstrained. One wave per workgroup, each its own unit, no block barrier (a super-tile's 8 units
// in one workgroup measured slower too: 25.6 vs 18.3 ms, §3d).
#ifndef RP_WAVE_WPE
#define RP_WAVE_WPE 7
#endif
template <typename T, typename IP, int WPE = std::is_same<T, float>::value ? RP_WAVE_WPE : 1>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
lpr_wave_kernel(PackedR R, T mag, int64_t n_rows, const IP* __restrict__ Ap, const int32_t* __restrict__ Aj,
                const T* __restrict__ Ax, LprStage stg, int cap_a, uint32_t ucap, unsigned n_tiles, unsigned s8,
                int order, LprSpace sp, Workspace* ws) {
    extern __shared__ __align__(16) unsigned char lds[];  // region A (descriptors, then slot), region B
    __shared__ uint64_t s_flag[kWaveSteps];               // row-start bitmap over the unit's entries
    __shared__ uint64_t s_susp;                           // rows flagged for the exact path
    __shared__ uint16_t s_kst[64];
    __shared__ uint8_t s_nz2row[64];
    const int lane = threadIdx.x & 63;
    // unit order follows the partition's XCD ranges: XCD x takes the units of super-tiles
    // [x * s8, (x + 1) * s8) in order (workgroup i runs on XCD i % 8)
    const unsigned rb = (blockIdx.x & 7u) * (4u * kPartTiles * s8) + (blockIdx.x >> 3);
    if (rb >= 4 * n_tiles) return;
    const unsigned tile = rb >> 2, u = rb & 3;
    const int64_t row0 = (int64_t)rb * 64;
    if (row0 >= n_rows) {  // the last tile's empty units
        if (lane == 0) sp.cnt[rb] = 0u;
        return;
    }
    const int nrows = (int)std::min<int64_t>(64, n_rows - row0);
    const int64_t trow0 = (int64_t)tile * kLprRows;
    const int64_t ta = (int64_t)Ap[trow0];
    const int64_t tn = (int64_t)Ap[std::min<int64_t>(trow0 + kLprRows, n_rows)] - ta;
    const uint32_t E0 = (uint32_t)((int64_t)Ap[row0] - ta), E1 = (uint32_t)((int64_t)Ap[row0 + nrows] - ta);
    const uint32_t rs0 = (uint32_t)((int64_t)Ap[row0 + std::min(lane, nrows)] - ta);  // straight-line load
    const uint32_t rs = lane < nrows ? rs0 : E1;
    auto go_heavy = [&]() {  // the heavy path takes the whole tile (idempotent over its four units)
        if (lane == 0 && atomicOr(&sp.tflag[tile], 1u) == 0u) sp.hlist[atomicAdd(&ws->n_deferred, 1u)] = tile;
    };
    // staged: this unit's part of tile run b is [c0, c1) of the run at GB[g, b] + OFF2[tile, b];
    // the table loads need only the unit index, so they go out with the row pointers
    const size_t gq = (size_t)(tile / kRunGroup) * stg.nb;
    int64_t g0 = 0;
    constexpr int kNBL = kStageMaxNB / 64;
    uint32_t cnt[kNBL], src[kNBL];
    // Loads below are straight-line (clamped addresses, results masked afterwards): a load guarded
    // by its own branch made the compiler wait for it inside the branch (vmcnt(0) after every load).
    // The run table is read whatever the gate says (its words are only used when staged)
    {
        g0 = stg.gb[gq];
        const uint16_t* __restrict__ cu1 = stg.cu + ((size_t)tile * 4 + u) * stg.ostride;
        const uint16_t* __restrict__ cu0 = u ? cu1 - stg.ostride : cu1;
        const uint32_t* __restrict__ o2 = stg.off2 + (size_t)tile * stg.ostride;
        const int64_t* __restrict__ gbq = stg.gb + gq;
        // unit 0 has no row before it: its c0 is masked to 0 after an unconditional load (an opaque
        // mask: a select of a load becomes a branch around it, and the branch a wait)
        uint32_t m0 = u ? 0xffffffffu : 0u;
        __asm__("" : "+v"(m0));
#pragma unroll
        for (int h = 0; h < kNBL; ++h) {
            const int b = std::min(64 * h + lane, stg.nb - 1);
            const uint32_t c1 = cu1[b], c0 = (uint32_t)cu0[b] & m0;
            const bool ok = 64 * h + lane < stg.nb;
            cnt[h] = ok ? c1 - c0 : 0u;
            src[h] = (uint32_t)(gbq[b] - g0) + o2[b] + c0;
        }
    }
    const uint32_t staged = *stg.gate;  // uniform: 0 after a segment overflow (direct gathers)
    // keep the table and gate loads here, in the row pointers' round trip: the compiler sank them
    // below the early returns (they are only used on the staged path), which cost the unit one or
    // two more dependent round trips before its S/D loads (wave kernel 6.59 -> 6.34 ms)
    __asm__ volatile("" ::: "memory");
    const uint32_t nu = E1 - E0, nsteps = (nu + 63) >> 6;
    if (tn > cap_a || nu > ucap) {  // uniform: the partition staged nothing / too many for the registers
        go_heavy();
        return;
    }
    if (nu == 0) {  // uniform: 64 empty rows (or fewer at the end): nothing to gather or store
        if (lane < nrows) sp.rowmeta[row0 + lane] = 0u;
        if (lane == 0) sp.cnt[rb] = 0u;
        return;
    }
    const T* __restrict__ Axt = Ax + ta;
    const uint32_t elast = E1 - 1;
    uint32_t dv[kWaveSteps];
    T xv[kWaveSteps];  // lanes past the unit hold any value: their descriptors are 0 (no products)
    uint32_t* desc = reinterpret_cast<uint32_t*>(lds);
    const size_t ra = lpr_wave_region_a(sp.slot, sizeof(T), ucap);
    // the side list (written from the side pre-pass to the side fill) in region B: the run lookup
    // there is dead once the S/D loads are issued, the exact-path scratch is used only after it
    uint16_t* s_sfk = reinterpret_cast<uint16_t*>(lds + ra);                      // slot position (0xffff: zero x)
    T* s_sfx = reinterpret_cast<T*>(lds + ra + 2 * kWaveSide);                     // ... its value
    uint32_t* s_sfj = reinterpret_cast<uint32_t*>(lds + ra + (2 + sizeof(T)) * kWaveSide);  // side-table index
    constexpr int kW0 = 12;  // steps loaded unconditionally (KDD2012 units: 11-12); the rest if present
    if (staged) {
        // the unit's layout: runs in bucket order; run k (k-th nonempty bucket) starts at layout
        // position pos (bit pos of the start bitmap), its words at S/D index ksrc[k] + position
        uint64_t* sbm = reinterpret_cast<uint64_t*>(lds + ra);
        uint32_t* ksrc = reinterpret_cast<uint32_t*>(lds + ra + 8 * kWaveSteps);
        if (lane < kWaveSteps) sbm[lane] = 0ull;
        __builtin_amdgcn_wave_barrier();
        uint32_t pos0 = 0, nrun = 0;
        const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
        for (int h = 0; h < kNBL; ++h) {
            if (64 * h >= stg.nb) continue;  // uniform
            const uint32_t inc = wave_scan_dpp(cnt[h]);
            const uint32_t pos = pos0 + inc - cnt[h];
            const uint64_t nz = __ballot(cnt[h] > 0);
            if (cnt[h] > 0) {
                ksrc[nrun + (uint32_t)__popcll(nz & lt)] = src[h] - pos;
                atomicOr(reinterpret_cast<unsigned long long*>(&sbm[pos >> 6]), 1ull << (pos & 63));
            }
            pos0 += __builtin_amdgcn_readlane(inc, 63);
            nrun += (uint32_t)__popcll(nz);
        }
        if (pos0 != nu) {  // uniform; cannot happen (the partition counted this tile): exact path
            go_heavy();
            return;
        }
        __builtin_amdgcn_wave_barrier();
        // lane x < kWaveSteps: bitmap word x and the start bits below it (read back per step as
        // wave-uniform values: position 64 x + lane's run is then two mbcnt instructions away)
        const uint64_t bw = lane < kWaveSteps ? sbm[lane] : 0ull;
        const uint32_t bc = (uint32_t)__popcll(bw);
        const uint32_t bpre = wave_scan_dpp(bc) - bc;
        const uint32_t bw_lo = (uint32_t)bw, bw_hi = (uint32_t)(bw >> 32);
        const uint32_t* __restrict__ St = stg.s + g0;
        const uint32_t* __restrict__ Dt = stg.d + g0;
        uint32_t sv[kWaveSteps];
        // plain loads (the neighbouring units of the super-tile read the same lines), 32-bit byte
        // offsets from the group base (a group's words stay far below 2^30)
        auto sd_load = [&](int x) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)bw_lo, x);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)bw_hi, x);
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bpre, x);
            // start bits at positions [0, lane] of word x: bit 0, then bits 1..lane (mbcnt of w >> 1)
            const uint32_t lo1 = (lo >> 1) | (hi << 31), hi1 = hi >> 1;
            const uint32_t k = b0 + (lo & 1u) + __builtin_amdgcn_mbcnt_hi(hi1, __builtin_amdgcn_mbcnt_lo(lo1, 0u)) - 1u;
            const bool in = 64u * x + lane < nu;  // lanes past the unit load the unit's first word
            const uint32_t i = ksrc[in ? k : 0u] + (in ? 64u * x + lane : 0u);
            sv[x] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(St) + (i << 2));
            dv[x] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(Dt) + (i << 2));
        };
#pragma unroll
        for (int x = 0; x < kW0; ++x) sd_load(x);
        if (nsteps > kW0) {  // uniform
#pragma unroll
            for (int x = kW0; x < kWaveSteps; ++x) sd_load(x);
        }
        // the values, in flight with the S/D words (one memory round trip for all three)
        // the unit's values as a buffer of nu entries: no clamp (a lane past the unit reads 0, no
        // memory access), the step offset folds into the instruction
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(Axt + E0), (short)0, (int)(nu * sizeof(T)), 0x00020000);
        auto ldx = [&](int x) { return buf_load_t<T>(xr, (uint32_t)((64 * x + lane) * sizeof(T))); };
#pragma unroll
        for (int x = 0; x < kW0; ++x) xv[x] = ldx(x);
        if (nsteps > kW0) {  // uniform
#pragma unroll
            for (int x = kW0; x < kWaveSteps; ++x) xv[x] = ldx(x);
        }
        // each D word to its entry's place (lanes past the unit loaded the first word: skipped)
#pragma unroll
        for (int x = 0; x < kW0; ++x)
            if (64u * x + lane < nu) desc[(sv[x] >> 20) - E0] = dv[x];
        if (nsteps > kW0) {  // uniform
#pragma unroll
            for (int x = kW0; x < kWaveSteps; ++x)
                if (64u * x + lane < nu) desc[(sv[x] >> 20) - E0] = dv[x];
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int x = 0; x < kWaveSteps; ++x) {
            const uint32_t v = desc[64u * x + lane];  // (past the unit: any LDS word, masked below)
            dv[x] = 64u * x + lane < nu ? v : 0u;
        }
        // every descriptor is in registers before the slot (region A) is written below
        __builtin_amdgcn_wave_barrier();
        __asm__ volatile("" ::: "memory");
    } else {
        const int32_t* __restrict__ Ajt = Aj + ta;
        int32_t jv[kWaveSteps];
#pragma unroll
        for (int x = 0; x < kWaveSteps; ++x) {
            const uint32_t e = std::min(E0 + 64 * x + lane, elast);
            jv[x] = Ajt[e];
            xv[x] = Axt[e];
        }
#pragma unroll
        for (int x = 0; x < kWaveSteps; ++x) {
            const uint32_t w = stg.w32[jv[x]];
            dv[x] = 64u * x + lane < nu ? w : 0u;
        }
    }
    // side entries (code 3) in entry order: their side-table words are requested now and used after
    // the flat pass (which lists the same entries in the same order), so the gather's latency hides
    // behind the pass
    uint32_t nside_pre = 0;
#pragma unroll
    for (int x = 0; x < kWaveSteps; ++x) {
        if ((uint32_t)x < nsteps) {  // uniform
            const bool side = (dv[x] >> 30) == 3u && 64u * x + lane < nu;
            const uint64_t sm = __ballot(side);
            if (side) {
                const uint32_t k = nside_pre + __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                if (k < (uint32_t)kWaveSide) s_sfj[k] = dv[x] & kW32J;
            }
            nside_pre += (uint32_t)__popcll(sm);
        }
    }
    __builtin_amdgcn_wave_barrier();
    const uint64_t side_w = (uint32_t)lane < std::min(nside_pre, (uint32_t)kWaveSide) ? R.SW[s_sfj[lane]] : 0ull;
    const uint32_t re = __shfl_down(rs, 1, 64);
    const uint32_t rend = lane == nrows - 1 ? E1 : (lane < nrows ? re : E1);
    const bool valid = lane < nrows;
    const bool nonempty = valid && rend > rs;
    uint16_t* cb = reinterpret_cast<uint16_t*>(lds);
    T* vb = reinterpret_cast<T*>(lds + ((2 * ((size_t)sp.slot + 2) + 15) & ~size_t(15)));
    uint16_t* scol = reinterpret_cast<uint16_t*>(lds + ra);
    T* sval = reinterpret_cast<T*>(lds + ra + ((2 * (size_t)kWaveScr + 15) & ~size_t(15)));
    if ((uint32_t)lane < nsteps) s_flag[lane] = 0ull;
    if (lane == 0) s_susp = 0ull;
    __builtin_amdgcn_wave_barrier();
    const uint64_t ne_mask = __ballot(nonempty);
    if (nonempty) {
        const uint32_t b = rs - E0;
        atomicOr(reinterpret_cast<unsigned long long*>(&s_flag[b >> 6]), 1ull << (b & 63));
        s_nz2row[__builtin_popcountll(ne_mask & ((1ull << lane) - 1))] = (uint8_t)lane;
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t carry_r = 0, carry_k = 0, nside = 0;
    bool bad = false;
    auto step = [&](uint32_t j, uint32_t d, T x) {
        const uint32_t e = E0 + 64 * j + lane;
        const bool ve = e < E1;
        const uint64_t fw = s_flag[j];
        const uint32_t nr = carry_r + (uint32_t)__builtin_popcountll(fw & ((2ull << lane) - 1)) - 1u;
        const uint32_t row = s_nz2row[nr & 63];
        const uint32_t n = d >> 30;
        const uint32_t np = n < 3 ? n : (d >> 26) & 15u;  // code 3: a side entry (count in the word)
        // all products of an entry are +-(x * mag): x * -mag is -(x * mag) exactly, and a kept
        // product is nonzero, so 0 + it (scipy's first add) is itself
        const T xm = tmul<T>(x, mag);
        const bool nzx = xm != T(0);
        const uint32_t kc = nzx ? np : 0u;
        const uint32_t kinc = wave_scan_dpp(kc);
        const uint32_t K = carry_k + kinc - kc;
        if (ve && ((fw >> lane) & 1ull)) s_kst[row] = (uint16_t)K;  // the row's first entry
        // products at K, K + 1 (K clamped: past the slot, both land in its two spare entries; the
        // unit then goes heavy)
        const uint32_t Kc = std::min(K, sp.slot);
        uint16_t* cK = cb + Kc;
        T* vK = vb + Kc;
        if (n < 3 && kc >= 1) {
            cK[0] = (uint16_t)(d & 0x3fffu);
            vK[0] = (d & 0x4000u) ? -xm : xm;
            if (kc >= 2) {
                cK[1] = (uint16_t)((d >> 15) & 0x3fffu);
                vK[1] = (d & 0x20000000u) ? -xm : xm;
            }
        }
        // side entries keep a gap [K, K + np) in the slot, filled after the pass; a zero product
        // is not in the slot: its row takes the exact path
        const bool side = ve && n == 3;
        const uint64_t sm = __ballot(side);
        if (side) {
            const uint32_t k = nside + __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
            if (k < (uint32_t)kWaveSide) {  // (its side-table index: listed before the pass)
                s_sfk[k] = kc ? (uint16_t)K : (uint16_t)0xffffu;
                s_sfx[k] = x;
            }
            if (np == 15) bad = true;  // 15 or more entries: the count is not exact -> heavy tile
        }
        nside += (uint32_t)__builtin_popcountll(sm);
        if (ve && np > 0 && !nzx) atomicOr(reinterpret_cast<unsigned long long*>(&s_susp), 1ull << row);
        carry_k += __builtin_amdgcn_readlane(kinc, 63);
        carry_r += (uint32_t)__builtin_popcountll(fw);
    };
#pragma unroll
    for (int x = 0; x < kWaveSteps; ++x)
        if ((uint32_t)x < nsteps) step(x, dv[x], xv[x]);
    bad = __ballot(bad) != 0 || nside > (uint32_t)kWaveSide;
    bool overflow = carry_k > sp.slot;
    // side fill: every side entry's products into its gap, in R's storage order
    if (!bad && (uint32_t)lane < nside) {
        const uint64_t sw = side_w;
        const uint32_t k0 = s_sfk[lane];
        if (k0 != 0xffffu) {
            const T x = s_sfx[lane];
            const bool rec = (sw >> 61) == 7;
            const uint32_t np = rec ? R.O[sw & kLow61] : (uint32_t)(sw >> 61);
            for (uint32_t t = 0; t < np && k0 + t < sp.slot; ++t) {
                uint32_t sl;
                if (rec) {
                    const uint32_t e = R.O[(sw & kLow61) + 1 + t];
                    sl = ((e & 0x8000u) >> 1) | (e & 0x3fffu);
                } else {
                    sl = (uint32_t)(sw >> (15 * t)) & 0x7fffu;
                }
                cb[k0 + t] = (uint16_t)(sl & 0x3fffu);
                vb[k0 + t] = tadd<T>(T(0), tmul<T>(x, (sl & 0x4000u) ? -mag : mag));
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (bad) {  // uniform
        go_heavy();
        return;
    }
    // ---- per row: kept count and a Bloom check of its columns (3 x 64-bit filters in registers)
    const uint32_t kst = nonempty ? s_kst[lane] : 0u;
    const uint64_t after = ne_mask & ~((2ull << lane) - 1);  // the next non-empty row ends this one
    const int nx = after ? __builtin_ctzll(after) : 64;
    const uint32_t kst_next = __shfl(kst, nx & 63, 64);
    const uint32_t kend_r = nx < 64 ? kst_next : carry_k;
    uint32_t kept = nonempty ? kend_r - kst : 0u;
    bool hit = false;
    if (!overflow) hit = lpr_repeat16(cb, kst, kept, sp.slot + 1);
    const uint64_t susp = s_susp;
    uint64_t todo = susp | __ballot(hit);  // lane == row within the unit
    if (__ballot(overflow)) todo = 0;
    // exact path, one flagged row at a time, the whole wave on it: its products in sequence order,
    // then every product checks for an earlier one of its column (first touch); a leader sums its
    // group in order; kept leaders land in the row's slot range in that order. A row the Bloom check
    // flagged already has all its products in sequence order in its slot range: read there (64 or
    // fewer: one round, every read before the first write). A row with a zero value (its zero
    // products are not in the slot) rebuilds them into the scratch from the descriptors in the
    // registers (entry e - E0 = step x, lane l: dv[x] of lane l).
    while (todo) {
        const int R0 = __builtin_ctzll(todo);
        todo &= todo - 1;
        const uint32_t a0 = __shfl(rs, R0, 64), a1 = __shfl(rend, R0, 64), kR = __shfl(kst, R0, 64);
        const uint32_t kE = __shfl(kend_r, R0, 64);
        const bool from_slot = !((susp >> R0) & 1ull) && kE - kR <= 64u;  // uniform
        const uint16_t* pc = from_slot ? cb + kR : scol;
        const T* pv = from_slot ? vb + kR : sval;
        uint32_t nprod = from_slot ? kE - kR : 0u;
        for (uint32_t e0 = a0; !from_slot && e0 < a1; e0 += 64) {
            const uint32_t e = e0 + lane;
            const bool in = e < a1;
            // the entry's W32 word gathered again (rows with a zero value are rare; the unit's
            // descriptors are not kept in registers past the flat pass)
            const uint32_t d = in ? stg.w32[Aj[ta + e]] : 0u;
            const T x = in ? Axt[e] : T(0);
            const uint32_t np = in ? ((d >> 30) < 3 ? (d >> 30) : (d >> 26) & 15u) : 0u;
            const uint32_t inc = wave_scan_dpp(np);
            const uint32_t q0 = nprod + inc - np;
            for (uint32_t t = 0; t < np; ++t)
                if (q0 + t < (uint32_t)kWaveScr) {
                    const uint32_t sl = lpr_slot_sw(d, t, R.SW, R.O);
                    scol[q0 + t] = (uint16_t)(sl & 0x3fffu);
                    sval[q0 + t] = tmul<T>(x, (sl & 0x4000u) ? -mag : mag);
                }
            nprod += __builtin_amdgcn_readlane(inc, 63);
        }
        if (nprod > (uint32_t)kWaveScr) {
            overflow = true;
            break;
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t nk = 0;
        for (uint32_t q0 = 0; q0 < nprod; q0 += 64) {
            const uint32_t q = q0 + lane;
            bool lead = q < nprod;
            T sum = T(0);
            uint16_t cq = 0;
            if (lead) {
                cq = pc[q];
                for (uint32_t b = 0; b < q && lead; ++b) lead = pc[b] != cq;
                if (lead) {
                    sum = tadd<T>(T(0), pv[q]);
                    for (uint32_t b = q + 1; b < nprod; ++b)
                        if (pc[b] == cq) sum = tadd<T>(sum, pv[b]);
                }
            }
            const bool keep = lead && sum != T(0);
            const uint32_t ki = wave_scan_dpp(keep ? 1u : 0u);
            if (keep) {
                if (kR + nk + ki - 1 >= sp.slot) overflow = true;
                else {
                    cb[kR + nk + ki - 1] = cq;
                    vb[kR + nk + ki - 1] = sum;
                }
            }
            nk += __builtin_amdgcn_readlane(ki, 63);
        }
        if (lane == R0) kept = nk;
        __builtin_amdgcn_wave_barrier();
    }
    // a row that gained entries in the exact path (side products not in the slot) must still end
    // before the next row's range
    if (kst + kept > kend_r && nonempty) overflow = true;
    if (__ballot(overflow)) {  // this unit cannot finish on the fast path: the whole tile goes heavy
        go_heavy();
        return;
    }
    if (order == RP_ORDER_SORTED && kept > 1) {  // ascending columns inside the row's slot range
        for (uint32_t a = kst + 1; a < kst + kept; ++a) {
            const uint16_t kc = cb[a];
            const T kv = vb[a];
            uint32_t b = a;
            while (b > kst && cb[b - 1] > kc) {
                cb[b] = cb[b - 1];
                vb[b] = vb[b - 1];
                --b;
            }
            cb[b] = kc;
            vb[b] = kv;
        }
    }
    __builtin_amdgcn_wave_barrier();
    lpr_store_slot<T>(cb, vb, kst, kept, valid, lane, carry_k, order, sp.rowmeta + row0, sp.cnt + rb,
                      sp.cols + (size_t)rb * sp.slot, reinterpret_cast<T*>(sp.vals) + (size_t)rb * sp.slot);
}

// heavy tiles, pass 0: the exact dense accumulator counts their rows (grid-stride over the list);
// the count goes to the tile's first wave slot, the other three are zeroed
template <typename T, typename IP>
__global__ void __launch_bounds__(kBlock)
lpr_heavy_count_kernel(PackedR R, T mag, int64_t n_rows, const IP* __restrict__ Ap, const int32_t* __restrict__ Aj,
                       const T* __restrict__ Ax, int p, LprSpace sp, Workspace* ws) {
    extern __shared__ __align__(16) unsigned char lds[];
    __shared__ uint32_t s_wsum[kBlock / 64];
    const unsigned nh = ws->n_deferred;
    uint32_t* s_rowc = reinterpret_cast<uint32_t*>(lds + heavy_lds_bytes(p, sizeof(T)) - 4 * kBlock);
    for (unsigned i = blockIdx.x; i < nh; i += gridDim.x) {
        const unsigned tile = sp.hlist[i];
        const int64_t row0 = (int64_t)tile * kLprRows;
        const int nrows = (int)std::min<int64_t>(kLprRows, n_rows - row0);
        heavy_tile<T, IP, int64_t, int32_t, PackedR>(R, mag, Ap, Aj, Ax, row0, nrows, p, lds, s_rowc, s_wsum, 0, 0,
                                                     nullptr, nullptr, nullptr, false, RP_ORDER_SCIPY);
        uint32_t tot;
        (void)block_excl_scan(threadIdx.x < (unsigned)nrows ? s_rowc[threadIdx.x] : 0u, s_wsum, &tot);
        if (threadIdx.x < 4) sp.cnt[(size_t)tile * 4 + threadIdx.x] = threadIdx.x == 0 ? tot : 0u;
        __syncthreads();
    }
}

// heavy tiles, pass 1: write at the tile's offset (after the scan)
template <typename T, typename IP, typename OP, typename OI>
__global__ void __launch_bounds__(kBlock)
lpr_heavy_write_kernel(PackedR R, T mag, int64_t n_rows, const IP* __restrict__ Ap, const int32_t* __restrict__ Aj,
                       const T* __restrict__ Ax, int p, LprSpace sp, Workspace* ws, OP* __restrict__ Cp,
                       OI* __restrict__ Cj, T* __restrict__ Cx, unsigned long long capacity, int order) {
    extern __shared__ __align__(16) unsigned char lds[];
    __shared__ uint32_t s_wsum[kBlock / 64];
    const unsigned nh = ws->n_deferred;
    const unsigned n_tiles = (unsigned)((n_rows + kLprRows - 1) / kLprRows);
    uint32_t* s_rowc = reinterpret_cast<uint32_t*>(lds + heavy_lds_bytes(p, sizeof(T)) - 4 * kBlock);
    for (unsigned i = blockIdx.x; i < nh; i += gridDim.x) {
        const unsigned tile = sp.hlist[i];
        const int64_t row0 = (int64_t)tile * kLprRows;
        const int nrows = (int)std::min<int64_t>(kLprRows, n_rows - row0);
        const unsigned long long G = sp.off[(size_t)tile * 4];
        const uint32_t cnt = sp.cnt[(size_t)tile * 4];
        heavy_tile<T, IP, OP, OI, PackedR>(R, mag, Ap, Aj, Ax, row0, nrows, p, lds, s_rowc, s_wsum, 1, G, Cp, Cj, Cx,
                                           G + cnt <= capacity, order);
        if (tile == n_tiles - 1 && threadIdx.x == 0) Cp[n_rows] = (OP)(G + cnt);
        __syncthreads();
    }
}

// exclusive scan of the wave counts: 4096 per block (16 per thread), decoupled look-back over
// blocks (taken in order from a ticket so every predecessor is running or done). Offsets start at
// *base_in (the entries of earlier row chunks); the running total goes to *base_out and ws->total.
constexpr int kScanPer = 16;
__global__ void __launch_bounds__(kBlock)
lpr_scan_kernel(LprSpace sp, size_t n, const unsigned long long* __restrict__ base_in,
                unsigned long long* __restrict__ base_out, Workspace* ws, unsigned* ticket) {
    __shared__ uint32_t s_wsum[kBlock / 64];
    __shared__ unsigned s_blk;
    __shared__ unsigned long long s_off;
    if (threadIdx.x == 0) s_blk = atomicAdd(ticket, 1u);
    __syncthreads();
    const unsigned blk = s_blk;
    const size_t t0 = (size_t)blk * (kBlock * kScanPer) + (size_t)threadIdx.x * kScanPer;
    uint32_t v[kScanPer];
    uint32_t local = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        v[i] = t0 + i < n ? sp.cnt[t0 + i] : 0u;
        local += v[i];
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan(local, s_wsum, &tot);
    if (threadIdx.x < 64) {
        const unsigned long long g = lookback_wave(sp.scan_state, blk, tot, ws);
        if (threadIdx.x == 0) s_off = g + *base_in;
    }
    __syncthreads();
    unsigned long long o = s_off + ex;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        if (t0 + i < n) sp.off[t0 + i] = o;
        o += v[i];
    }
    if (t0 < n && t0 + kScanPer >= n) {  // the thread holding the last count: the running total
        ws->total = o;
        *base_out = o;
    }
}

// slots -> C: one workgroup per tile (grid-stride), one wave per 64-row unit. The unit's rows (slot
// ranges kst | kept << 16 in rowmeta) get their output offsets from a wave scan of the kept counts
// (indptr); each output o finds its row (the last lane whose offset is <= o: empty rows share the
// next row's offset) and reads its entry from the slot, the row reversed for scipy's reverse
// first-touch order or as built (ascending) for RP_ORDER_SORTED. kCopyU steps of 64 outputs are
// loaded before any is stored. Heavy tiles are placed by lpr_heavy_write_kernel.
template <typename T, typename OP, typename OI>
__global__ void __launch_bounds__(kBlock)
lpr_copy_kernel(LprSpace sp, int64_t n_rows, unsigned n_tiles, OP* __restrict__ Cp, OI* __restrict__ Cj,
                T* __restrict__ Cx, unsigned long long capacity, int order) {
    const T* vals = reinterpret_cast<const T*>(sp.vals);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (unsigned tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        if (sp.tflag[tile]) continue;  // lpr_heavy_write_kernel places it
        const size_t wt = (size_t)tile * 4 + w;
        const unsigned long long G = sp.off[wt];
        const uint32_t cnt = sp.cnt[wt];
        const int64_t row0 = (int64_t)tile * kLprRows;
        const int nrows = (int)std::min<int64_t>(kLprRows, n_rows - row0);
        const int r = 64 * w + lane;
        const uint32_t meta = r < nrows ? sp.rowmeta[row0 + r] : 0u;
        const uint32_t kst = meta & 0xffffu, kept = meta >> 16;
        const uint32_t pre = wave_scan_dpp(kept) - kept;
        if (r < nrows) Cp[row0 + r] = (OP)(G + pre);
        if (tile == n_tiles - 1 && threadIdx.x == kBlock - 1) Cp[n_rows] = (OP)(G + cnt);
        if (G + cnt > capacity) continue;
        const uint16_t* __restrict__ sc = sp.cols + wt * sp.slot;
        const T* __restrict__ sv = vals + wt * sp.slot;
        constexpr int kCopyU = 8;
        if (lpr_slot_final(kept, kst, pre)) {  // stored in final order (lpr_store_slot): one run
            for (uint32_t q0 = 0; q0 < cnt; q0 += 64 * kCopyU) {
                uint16_t cv[kCopyU];
                T xv[kCopyU];
#pragma unroll
                for (int u = 0; u < kCopyU; ++u) {
                    const uint32_t o = std::min(q0 + 64 * u + lane, cnt - 1);
                    cv[u] = __builtin_nontemporal_load(sc + o);
                    xv[u] = __builtin_nontemporal_load(sv + o);
                }
#pragma unroll
                for (int u = 0; u < kCopyU; ++u) {
                    const uint32_t o = q0 + 64 * u + lane;
                    if (o < cnt) {
                        Cj[G + o] = (OI)cv[u];
                        Cx[G + o] = xv[u];
                    }
                }
            }
            continue;
        }
        // the row's first slot entry and the step to the next output: reversed (scipy) or forward
        const bool rev = order != RP_ORDER_SORTED;
        const uint32_t base = rev ? kst + kept - 1 : kst;
        for (uint32_t q0 = 0; q0 < cnt; q0 += 64 * kCopyU) {  // wave-uniform trip count
            uint16_t cv[kCopyU];
            T xv[kCopyU];
#pragma unroll
            for (int u = 0; u < kCopyU; ++u) {
                const uint32_t o = q0 + 64 * u + lane;
                int lo = 0;
#pragma unroll
                for (int step = 32; step > 0; step >>= 1) {
                    const uint32_t pv = (uint32_t)__shfl((int)pre, lo + step, 64);
                    if (lo + step < 64 && pv <= o) lo += step;
                }
                const uint32_t i = o - (uint32_t)__shfl((int)pre, lo, 64);
                const uint32_t b = (uint32_t)__shfl((int)base, lo, 64);
                const uint32_t src = std::min(rev ? b - i : b + i, sp.slot - 1);
                cv[u] = o < cnt ? __builtin_nontemporal_load(sc + src) : (uint16_t)0;
                xv[u] = o < cnt ? __builtin_nontemporal_load(sv + src) : T(0);
            }
#pragma unroll
            for (int u = 0; u < kCopyU; ++u) {
                const uint32_t o = q0 + 64 * u + lane;
                if (o < cnt) {
                    Cj[G + o] = (OI)cv[u];
                    Cx[G + o] = xv[u];
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// small helper kernels
template <typename S, typename D>
__global__ void convert_kernel(const S* __restrict__ s, D* __restrict__ d, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        d[i] = (D)s[i];
}

// first position (atomicMin) of a column index outside [0, m): host-path input validation
__global__ void check_columns_kernel(const int32_t* __restrict__ Aj, int64_t n, int64_t m,
                                     unsigned long long* first_bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t j = Aj[i];
        if (j < 0 || (int64_t)j >= m) atomicMin(first_bad, (unsigned long long)i);
    }
}

template <typename S, typename D>
__global__ void rebase_kernel(const S* __restrict__ s, D* __restrict__ d, int64_t n, int64_t add) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        d[i] = (D)((int64_t)s[i] + add);
}

// ---- synthetic rows: counter-based RNG (splitmix64 of seed, row, draw)
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double u01(uint64_t h) { return ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

__device__ int synth_count(uint64_t seed, int64_t row, double lam, int cap) {
    if (lam < 0) return std::min((int)(-lam + 0.5), cap);  // fixed count (configs[3]: 100 per row)
    // 1 + Poisson(lam) by inversion
    const double u = u01(mix64(seed ^ mix64((uint64_t)row * 2 + 1)));
    double pk = exp(-lam), cdf = pk;
    int k = 0;
    while (u > cdf && k < 4096) {
        ++k;
        pk *= lam / k;
        cdf += pk;
    }
    return std::min(1 + k, cap);
}

template <typename IP>
__global__ void synth_count_kernel(int64_t n_rows, uint64_t seed, double lam, int cap, int64_t m,
                                   IP* __restrict__ counts) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows;
         i += (int64_t)gridDim.x * blockDim.x)
        counts[i + 1] = (IP)std::min<int64_t>(synth_count(seed, i, lam, cap), m);
}

constexpr int kSynthMaxK = 256;

__global__ void synth_fill_kernel(int64_t n_rows, int64_t m, uint64_t seed, int dist,
                                  double zipf_s, uint64_t perm_a, uint64_t perm_b,
                                  const int64_t* __restrict__ indptr, int32_t* __restrict__ Aj,
                                  float* __restrict__ Ax) {
    int32_t cols[kSynthMaxK];
    const double one_minus_s = 1.0 - zipf_s;
    const double top = pow((double)m + 1.0, one_minus_s);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = indptr[i];
        const int k = (int)(indptr[i + 1] - b);
        uint64_t ctr = 0;
        for (int t = 0; t < k; ++t) {
            int32_t c;
            bool dup;
            do {
                const uint64_t h = mix64(seed ^ mix64(((uint64_t)i << 20) ^ (ctr++) ^ 0xA5A5000000000000ull));
                if (dist == 0) {
                    c = (int32_t)(((h >> 32) * (uint64_t)m) >> 32);
                } else {
                    // bounded Zipf(s) rank by continuous inversion, then a fixed affine permutation
                    const double u = u01(h);
                    double xr = pow(1.0 - u * (1.0 - top), 1.0 / one_minus_s);
                    int64_t rank = (int64_t)xr - 1;
                    rank = rank < 0 ? 0 : (rank >= m ? m - 1 : rank);
                    c = (int32_t)((perm_a * (uint64_t)rank + perm_b) % (uint64_t)m);
                }
                dup = false;
                for (int q = 0; q < t; ++q) dup |= (cols[q] == c);
            } while (dup);
            // insertion into sorted position
            int q = t;
            while (q > 0 && cols[q - 1] > c) {
                cols[q] = cols[q - 1];
                --q;
            }
            cols[q] = c;
        }
        for (int t = 0; t < k; ++t) {
            Aj[b + t] = cols[t];
            Ax[b + t] = 1.0f;
        }
    }
}

// three-phase device scan (block sums, scan of block sums, add back) for int64 counts
constexpr int kScanBlock = 1024;
__global__ void scan_blocks_kernel(int64_t* a, int64_t n, int64_t* bsum) {
    __shared__ int64_t s[kScanBlock];
    const int64_t i = blockIdx.x * (int64_t)kScanBlock + threadIdx.x;
    s[threadIdx.x] = i < n ? a[i] : 0;
    __syncthreads();
    for (int o = 1; o < kScanBlock; o <<= 1) {
        int64_t t = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
        __syncthreads();
        s[threadIdx.x] += t;
        __syncthreads();
    }
    if (i < n) a[i] = s[threadIdx.x];
    if (threadIdx.x == kScanBlock - 1) bsum[blockIdx.x] = s[threadIdx.x];
}
__global__ void scan_add_kernel(int64_t* a, int64_t n, const int64_t* bsum_scanned) {
    const int64_t i = blockIdx.x * (int64_t)kScanBlock + threadIdx.x;
    if (blockIdx.x > 0 && i < n) a[i] += bsum_scanned[blockIdx.x - 1];
}

// ------------------------------------------------------------------------------------------
// host-side structures
}  // namespace

namespace rpd {
// block sums of every level in one scratch buffer (grown, never freed here: a hipFree per scan
// synchronised the whole device and serialised the libsvm stream's uploads with its kernels)
static int scan_level(int64_t* a, int64_t n, hipStream_t st, int64_t* scratch) {
    const int64_t nb = (n + kScanBlock - 1) / kScanBlock;
    hipLaunchKernelGGL(scan_blocks_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, a, n, scratch);
    if (nb > 1) {
        scan_level(scratch, nb, st, scratch + nb + 1);
        hipLaunchKernelGGL(scan_add_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, a, n, scratch);
    }
    return RP_OK;
}

int inclusive_scan_i64(int64_t* a, int64_t n, hipStream_t st, DevBuf& tmp, int device) {
    if (n <= 0) return RP_OK;
    size_t words = 0;
    for (int64_t m = n; m > 1;) {
        m = (m + kScanBlock - 1) / kScanBlock;
        words += (size_t)m + 1;
    }
    int rc = tmp.grow(sizeof(int64_t) * std::max<size_t>(words, 1), device);
    if (rc) return rc;
    scan_level(a, n, st, (int64_t*)tmp.p);
    HIP_TRY(hipGetLastError());
    return RP_OK;
}

}  // namespace rpd

struct rp_projector {
    int device = 0;
    int64_t m = 0, p = 0, nnz = 0;
    int layout = RP_LAYOUT_GENERIC;
    int value_type = RP_F32;
    double mag = 0.0;
    int bs = 0;
    // packed
    DevBuf W, O, spare;  // packed image: W (u64 per feature), O (long-row records); spare unused
    DevBuf W32;          // staged-gather table derived from W (u32 per feature), m <= 2^26 only
    DevBuf SW;           // side table: W words of the features with > 2 entries (W32 code 3)
    DevBuf BM;           // nonempty-feature bitmap (1 bit per feature) for the staged gather
    int stage_mode = -1; // -1 auto, 0 off, 1 on (rp_projector_set_staging)
    int stage_sb = 0;    // bucket = 2^sb features; 0 = auto
    // rp_projector_set_option (tuning and tests; the library reads no environment variables)
    int opt_pipeline = 0;       // 0 auto, 1 tile, 2 row-lane where it can run
    int opt_defer_polls = -2;   // tile pipeline: -1 no slots (every tile waits, then writes C); else slots
    int opt_defer_ticks = -1;   // ignored since round 6 (kept for the ABI)
    int64_t opt_chunk_rows = 0; // 0 default
    int opt_host_threads = -1;  // -1 default
    // the last stream call (rp_project_stream / rp_libsvm_project_stream): chunks, chunks recomputed
    // after the pipeline (their output outgrew the device slot), slot regrowths in the pipeline
    int64_t st_chunks = 0, st_redo = 0, st_regrow = 0;
    // generic
    DevBuf Bp, Bj, Bx32, Bx64;
    // internal workspace and host-path staging
    DevBuf ws, ws_check;
    DevBuf a_ptr, a_idx, a_val;
    std::mutex mu;
};

struct rp_result {
    rp_projector* h = nullptr;
    int64_t n_rows = 0, nnz = 0;
    int value_type = RP_F32;
    DevBuf cp, cj, cx;  // int64 indptr, int32 indices, T data
};

namespace {

Caps choose_caps(int64_t n_rows, int64_t nnz_a, double prod_per_entry) {
    // rows per tile: 256 when rows are short (KDD: 11 entries), fewer for long rows or dense R so
    // a tile's entries fit the register-held stage-1 window (kMaxE per thread) and its products a
    // ~40 KB LDS tile; caps leave ~6 sigma headroom (a tile beyond them takes the exact slow path)
    constexpr double kProdBudget = 2816.0;
    Caps c;
    const double avg = n_rows > 0 ? std::max((double)nnz_a / (double)n_rows, 1e-9) : 1.0;
    const double ppe = std::max(prod_per_entry, 1e-9);
    const double want = std::min(0.72 * kCapAMax / avg, 0.72 * kProdBudget / (avg * ppe));
    c.rpt = (int)std::max(1.0, std::min((double)kBlock, want));
    const double ents = avg * c.rpt;
    // 6 sigma of a sum of rpt Poisson-like row lengths (sd ~ sqrt(ents)); the products' sd is
    // ~1.25 sqrt(products) for single-magnitude SRP matrices (compound of R-row counts)
    c.cap_a = (int)std::min<double>(kCapAMax, ((int)(ents + 6.0 * std::sqrt(ents) + 40.0) + 63) & ~63);
    const double prods = std::max(1.0, ents * prod_per_entry);
    c.cap_p = (int)std::min<double>(8192.0, ((int)(prods + 7.5 * std::sqrt(prods) + 40.0) + 63) & ~63);
    return c;
}

size_t lds_bytes_for(const Caps& c, int value_size, int64_t p) {
    const TileLayout L(c, (size_t)value_size);
    return std::max(L.total, heavy_lds_bytes(p, (size_t)value_size));
}

// Launch plan and workspace carve-up (offsets in bytes from the workspace start). Tile pipeline:
//   [Workspace header + look-back states] [deferred list, pool offsets, headers, pool]. Row-lane:
//   [header + scan states + heavy flags] [carry slots + gate] [wave counts, offsets, heavy list,
//   row metadata, slots] [staged: OFF2, CU, GB, FILL, S, D]   (value size vs: 8 when sizing)
struct Plan {
    Caps caps;
    int64_t n_tiles = 0;
    bool staged = false;
    bool defer = false;
    int sb = 0, nb = 0;
    uint32_t ostride = 0;
    size_t head = 0, dlist = 0, pofs = 0, dhdr = 0, pcols = 0, pvals = 0, tcnt = 0, cu = 0, s = 0, d = 0;
    unsigned long long pool_cap = 0;  // tile pipeline: entries per tile slot
    size_t total = 0;
    // row-lane pipeline (lpr_*): tiles of kLprRows rows, every tile's output in a fixed slot
    bool lpr = false;
    uint32_t lpr_slot = 0;
    int64_t lpr_chunk = 0;    // rows per launch sequence (a multiple of kLprRows; n_rows if one)
    size_t carry = 0;         // two u64 running-total slots (chunk k reads k & 1, writes the other),
                              // then the u32 staging gate (lpr_choose_kernel) at carry + 16
    bool gated = false;       // staging decided on the device per call (auto mode)
    size_t zero = 0;          // bytes zeroed once per call (header + states [+ carry])
    int64_t scan_blocks = 0;
    size_t lcnt = 0, loff = 0, lhl = 0, ltf = 0, lrow = 0, lcols = 0, lvals = 0;
    size_t off2 = 0, gb = 0, fill = 0;  // staged runs (lpr_reserve_kernel, lpr_partition_kernel)
    int64_t sd_words = 0;               // S / D capacity (words)
    unsigned groups = 0;
    uint32_t ucap = 0;                  // staged: entries per 64-row unit on the fast path (<= 16 steps)
};

// slot copy workgroups: one per tile up to 2^23 tiles (grid-stride beyond); 2^20 workgroups each
// looping over ~7 configs[3] tiles measured 18.1 ms against 16.3 for one tile per workgroup
constexpr unsigned kSlotCopyGrid = 1u << 23;
constexpr int64_t kStageMinNnz = 1 << 22;      // auto: stage only launches this large
// rp_project_stream's default chunk: configs[1] host CSR in/out measured 475 M rows/s with 4M-row
// chunks, 544 M with 2M (shorter fill and drain of the upload/compute/download pipeline)
constexpr int64_t kStreamChunkRows = (int64_t)2 << 20;
constexpr int64_t kStageMinTable = 64ll << 20;  // ... and only a W past L2/MALL-friendly sizes

// Row-lane pipeline choice: packed R, short rows (one lane walks a row), few products per row.
// RP_PIPE=tile|lpr forces a pipeline where it can run (tests, measurements).
constexpr double kLprMaxRowEntries = 24.0, kLprMaxRowProducts = 24.0;
constexpr bool kLprAuto = true;        // auto picks the row-lane pipeline (configs[1]: 22 ms vs 28 tile)
constexpr bool kLprStageAuto = true;   // ... and staging inside it (large launches over a large R)
// rows per launch sequence of the row-lane pipeline: the workspace (~150 B per KDD2012 row) is sized
// for one chunk, so a launch of 1.08B rows (configs[2] on one GPU) needs ~20 GB, not ~190 GB
constexpr int64_t kLprChunkRows = (int64_t)1 << 27;
int64_t lpr_chunk_rows(const rp_projector* h) {  // RP_OPT_CHUNK_ROWS: rounded up to whole tiles
    if (h->opt_chunk_rows > 0)
        return std::max<int64_t>(kLprRows, (h->opt_chunk_rows + kLprRows - 1) / kLprRows * kLprRows);
    return kLprChunkRows;
}
bool lpr_wanted(const rp_projector* h, int64_t n_rows, int64_t nnz_a) {
    if (h->layout != RP_LAYOUT_PACKED || n_rows <= 0 || nnz_a < 0) return false;
    const double ppe = h->m > 0 ? (double)h->nnz / (double)h->m : 0.0;
    const double avg = (double)nnz_a / (double)n_rows;
    const bool fits = avg <= kLprMaxRowEntries && avg * ppe <= kLprMaxRowProducts &&
                      avg * kLprRows + 6.0 * std::sqrt(avg * kLprRows) + 40.0 <= kCapAMax;
    if (h->opt_pipeline == 1) return false;  // RP_OPT_PIPELINE: tile forced
    if (h->opt_pipeline == 2) return fits;   // row-lane forced where it can run
    return kLprAuto && fits;
}

Plan make_plan(const rp_projector* h, int64_t n_rows, int64_t nnz_a, bool allow_stage = true,
               int vs = 8, bool allow_defer = true) {
    Plan pl;
    const double ppe = h->m > 0 ? (double)h->nnz / (double)h->m : 0.0;
    auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
    if (lpr_wanted(h, n_rows, nnz_a) && allow_defer) {
        // one lane per row: 256-row tiles, entries capped for LDS (6 sigma), the output slot for the
        // expected products + 7.5 sigma (a tile beyond either takes the exact heavy path)
        pl.lpr = true;
        const double avg = (double)nnz_a / (double)n_rows;
        const double ents = avg * kLprRows, prods = std::max(1.0, ents * ppe);
        pl.caps.rpt = kLprRows;
        pl.caps.cap_a = (int)std::min<double>(kCapAMax, ((int)(ents + 6.0 * std::sqrt(ents) + 40.0) + 63) & ~63);
        pl.caps.cap_p = (int)std::min<double>(65535.0, ((int)(prods + 9.5 * std::sqrt(prods) + 64.0) + 63) & ~63);
        const double prods_w = std::max(1.0, avg * 64 * ppe);  // one wave's slot: 64 rows
        // mean + 7 sigma (sigma ~ 1.25 sqrt(mean) for single-magnitude SRP rows) + 32: KDD2012 608,
        // which keeps a tile's LDS (descriptors + the 4 slots) at 32 KB: 5 tiles per CU
        pl.lpr_slot = (uint32_t)std::min<double>(65472.0, ((int)(prods_w + 8.75 * std::sqrt(prods_w) + 32.0) + kSlotRound - 1) & ~(kSlotRound - 1));
        pl.lpr_chunk = std::min<int64_t>(n_rows, lpr_chunk_rows(h));
        pl.n_tiles = (pl.lpr_chunk + kLprRows - 1) / kLprRows;
        const size_t nw = 4 * (size_t)pl.n_tiles;
        pl.scan_blocks = ((int64_t)nw + kBlock * kScanPer - 1) / (kBlock * kScanPer);
        // header, scan states and the per-tile heavy flags are zeroed by one memset per call
        pl.ltf = al(sizeof(Workspace) + 8u * (size_t)std::max<int64_t>(pl.scan_blocks, 1));
        pl.head = pl.ltf + al(4 * (size_t)pl.n_tiles);
        pl.carry = pl.head;
        pl.zero = pl.carry + 16;
        pl.lcnt = pl.carry + 256;
        pl.loff = pl.lcnt + al(4 * nw);
        pl.lhl = pl.loff + al(8 * nw);
        pl.lrow = pl.lhl + al(4 * (size_t)pl.n_tiles);
        pl.lcols = pl.lrow + al(4 * (size_t)kLprRows * (size_t)pl.n_tiles);
        pl.lvals = pl.lcols + al(2 * (size_t)pl.lpr_slot * nw);
        pl.total = pl.lvals + al((size_t)vs * (size_t)pl.lpr_slot * nw);
        const bool want_stage = h->stage_mode == 1 || (h->stage_mode == -1 && kLprStageAuto &&
                                                       nnz_a >= kStageMinNnz && 8 * h->m >= kStageMinTable);
        // the wave kernel holds a unit's descriptors in registers, at most kWaveSteps x 64: a unit
        // of 64 average rows plus 8 sigma must fit (KDD2012: 704 + 212 -> cap 1024, 12 sigma); a
        // unit past the cap takes the exact heavy path with its tile. Rows of more than ~12.5
        // entries on average take direct gathers instead.
        const double ents_u = avg * 64, need_u = ents_u + 8.0 * std::sqrt(ents_u);
        pl.ucap = (uint32_t)std::min<double>(64.0 * kWaveSteps, ((int)need_u + 63) & ~63);
        const bool fits_u = need_u <= 64.0 * kWaveSteps;
        if (allow_stage && want_stage && fits_u && h->W32.p) {
            int sb = h->stage_sb > 0 ? h->stage_sb : 19;
            auto nbk = [&](int b) { return (int)((h->m + ((int64_t)1 << b) - 1) >> b); };
            while (h->stage_sb <= 0 && nbk(sb) > kStageMaxNB && sb < 20) ++sb;
            if (sb >= 1 && sb <= 20 && nbk(sb) <= kStageMaxNB) {
                pl.staged = true;
                pl.gated = h->stage_mode == -1;
                pl.sb = sb;
                pl.nb = std::max(nbk(sb), 1);
                // run tables tile-major: a tile's (nb + 1) bucket starts and nb run positions are
                // contiguous (one or two lines per tile for the partition's stores and the main
                // kernel's loads, instead of one line per bucket)
                pl.ostride = (uint32_t)((pl.nb + 1 + 7) & ~7);
                pl.groups = (unsigned)((pl.n_tiles + kRunGroup - 1) / kRunGroup);
                pl.off2 = pl.total;
                pl.cu = pl.off2 + al(4 * (size_t)pl.ostride * (size_t)pl.n_tiles);
                pl.gb = pl.cu + al(2 * 4 * (size_t)pl.ostride * (size_t)pl.n_tiles);
                const size_t nseg = (size_t)pl.groups * pl.nb;
                pl.fill = pl.gb + al(8 * (nseg + 1));
                // staged entries of one chunk: all of them, or (several chunks) at most cap_a per
                // tile (a tile past the cap stages nothing); plus the segments' reserves
                // (lpr_reserve_kernel: sum of 8 sqrt(E_s) <= 8 sqrt(segments x entries), 256 each)
                const double se = pl.lpr_chunk < n_rows ? (double)pl.n_tiles * (double)pl.caps.cap_a : (double)nnz_a;
                const size_t sd = (size_t)(se + 8.0 * std::sqrt((double)nseg * se)) + 256 * nseg + 1024;
                pl.sd_words = (int64_t)sd;
                pl.s = pl.fill + al(4 * nseg);
                pl.d = pl.s + al(4 * sd);
                pl.total = pl.d + al(4 * sd);
            }
        }
        return pl;
    }
    pl.caps = choose_caps(n_rows, nnz_a >= 0 ? nnz_a : n_rows * 11, ppe);
    pl.n_tiles = n_rows > 0 ? (n_rows + pl.caps.rpt - 1) / pl.caps.rpt : 0;
    pl.head = al(sizeof(Workspace) + 8u * (size_t)std::max<int64_t>(pl.n_tiles, 1));
    pl.zero = pl.head;
    pl.total = pl.head;
    if (pl.n_tiles > 0 && allow_defer && nnz_a >= 0) {  // tile slots (DeferSpace): list, offsets, headers, slots
        pl.defer = true;
        pl.pool_cap = (unsigned long long)pl.caps.cap_p;  // a tile's outputs <= its products <= cap_p
        const size_t nt = (size_t)pl.n_tiles;
        pl.dlist = pl.total;
        pl.pofs = pl.dlist + al(4 * nt);
        pl.tcnt = pl.pofs + al(8 * nt);
        pl.dhdr = pl.tcnt + al(4 * nt);
        pl.pcols = pl.dhdr + al(2 * (size_t)(pl.caps.rpt + 1) * nt);
        pl.pvals = pl.pcols + al(2 * (size_t)pl.pool_cap * nt);
        pl.total = pl.pvals + al((size_t)vs * (size_t)pl.pool_cap * nt);
    }
    return pl;  // the tile pipeline gathers R's descriptors directly (its staged gather was removed)
}

template <typename T, typename IP, typename OP, typename OI, typename RL, int WPE = 1>
int launch_main(const RL& R, T mag, rp_projector* h, const rp_csr_in* a, const rp_csr_out* c,
                int order, Workspace* ws, unsigned n_tiles, const Plan& pl, size_t lds,
                hipStream_t st) {
    if constexpr (WPE == 1 && std::is_same<T, float>::value && std::is_same<RL, PackedR>::value) {
        // 7 tiles per CU fit the LDS (static arrays ~1.6 KB per tile): take the 7-wave build
        if (lds + 2048 <= 160 * 1024 / 7)
            return launch_main<T, IP, OP, OI, RL, 7>(R, mag, h, a, c, order, ws, n_tiles, pl, lds, st);
    }
    HIP_TRY(hipFuncSetAttribute((const void*)spgemm_lookback_kernel<T, IP, OP, OI, RL, WPE>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    char* base = reinterpret_cast<char*>(ws);
    // slots unless the workspace is small or RP_OPT_DEFER_POLLS = -1 (every tile waits, then writes C)
    const bool slots = pl.defer && h->opt_defer_polls != -1;
    DeferSpace dfr{reinterpret_cast<unsigned int*>(base + pl.dlist),
                   reinterpret_cast<unsigned long long*>(base + pl.pofs),
                   reinterpret_cast<uint16_t*>(base + pl.dhdr),
                   slots ? reinterpret_cast<uint16_t*>(base + pl.pcols) : nullptr,
                   reinterpret_cast<unsigned char*>(base + pl.pvals), reinterpret_cast<uint32_t*>(base + pl.tcnt),
                   pl.pool_cap};
    hipLaunchKernelGGL((spgemm_lookback_kernel<T, IP, OP, OI, RL, WPE>), dim3(n_tiles), dim3(kBlock), lds, st,
                       R, mag, (int)h->p, a->n_rows,
                       (const IP*)a->indptr, a->indices, (const T*)a->data, (OP*)c->indptr,
                       (OI*)c->indices, (T*)c->data, (unsigned long long)c->capacity, pl.caps, order,
                       ws, n_tiles, dfr);
    HIP_TRY(hipGetLastError());
    if (slots) {
        // the tiles' offsets: scan of tcnt (4096 per block, look-back over blocks; its states in
        // the tile-state region, its ticket / zero base / total in the header's pad words)
        LprSpace scan{dfr.tcnt, dfr.toff, nullptr, nullptr, nullptr, nullptr, nullptr,
                      reinterpret_cast<unsigned long long*>(ws + 1), 0u};
        const unsigned scan_blocks = (unsigned)(((size_t)n_tiles + kBlock * kScanPer - 1) / (kBlock * kScanPer));
        hipLaunchKernelGGL(lpr_scan_kernel, dim3(scan_blocks), dim3(kBlock), 0, st, scan, (size_t)n_tiles,
                           (const unsigned long long*)&ws->pad[1], &ws->pad[2], ws,
                           reinterpret_cast<unsigned*>(&ws->pad[0]));
        HIP_TRY(hipGetLastError());
        const size_t hl = heavy_lds_bytes(h->p, sizeof(T));
        HIP_TRY(hipFuncSetAttribute((const void*)tile_heavy_write_kernel<T, IP, OP, OI, RL>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)hl));
        hipLaunchKernelGGL((tile_heavy_write_kernel<T, IP, OP, OI, RL>), dim3(256), dim3(kBlock), hl, st, R, mag,
                           (int)h->p, a->n_rows, (const IP*)a->indptr, a->indices, (const T*)a->data, (OP*)c->indptr,
                           (OI*)c->indices, (T*)c->data, (unsigned long long)c->capacity, pl.caps, order, ws, dfr);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL((slot_copy_kernel<T, OP, OI>), dim3(std::min(n_tiles, kSlotCopyGrid)), dim3(kBlock), 0,
                           st, dfr, pl.caps, a->n_rows, n_tiles, (OP*)c->indptr, (OI*)c->indices,
                           (T*)c->data, (unsigned long long)c->capacity);
        HIP_TRY(hipGetLastError());
    }
    return RP_OK;
}

size_t lpr_lds_bytes(int cap_a, size_t vs, uint32_t slot) {  // lpr_main_flat_kernel: descriptors + 4 slots
    return ((4 * (size_t)cap_a + 15) & ~size_t(15)) + ((8 * (size_t)slot + 15) & ~size_t(15)) + 4 * vs * (size_t)slot;
}

// One row chunk of the row-lane pipeline. staged: reserve, partition, gather, wave kernel (which
// takes direct gathers itself if a segment overflowed: the gate); direct: lpr_main_flat_kernel.
// Then the heavy tiles' count, the scan of the wave counts, the copy and the heavy tiles' write.
template <typename T, typename IP, typename OP, typename OI>
int launch_lpr_chunk(const PackedR& R, T mag, rp_projector* h, const rp_csr_in* a, const rp_csr_out* c, int order,
                     Workspace* ws, const Plan& pl, bool staged, hipStream_t st, int64_t chunk) {
    char* base = reinterpret_cast<char*>(ws);
    unsigned long long* carry = reinterpret_cast<unsigned long long*>(base + pl.carry);
    LprSpace sp{reinterpret_cast<uint32_t*>(base + pl.lcnt), reinterpret_cast<unsigned long long*>(base + pl.loff),
                reinterpret_cast<uint32_t*>(base + pl.lhl), reinterpret_cast<uint32_t*>(base + pl.ltf),
                reinterpret_cast<uint32_t*>(base + pl.lrow), reinterpret_cast<uint16_t*>(base + pl.lcols),
                reinterpret_cast<unsigned char*>(base + pl.lvals), reinterpret_cast<unsigned long long*>(ws + 1),
                pl.lpr_slot};
    const unsigned n_tiles = (unsigned)((a->n_rows + kLprRows - 1) / kLprRows);
    const IP* Ap = (const IP*)a->indptr;
    const T* Ax = (const T*)a->data;
    const unsigned t8 = (n_tiles + 7) / 8;
    if (staged) {
        // the gate word: 1 unless a segment overflow in a partition (this chunk's or an earlier
        // one's) cleared it; the wave kernel then gathers directly
        uint32_t* gate = reinterpret_cast<uint32_t*>(base + pl.carry + 16);
        uint32_t* OFF2 = reinterpret_cast<uint32_t*>(base + pl.off2);
        uint16_t* CU = reinterpret_cast<uint16_t*>(base + pl.cu);
        int64_t* GB = reinterpret_cast<int64_t*>(base + pl.gb);
        uint32_t* FILL = reinterpret_cast<uint32_t*>(base + pl.fill);
        uint32_t* Sw = reinterpret_cast<uint32_t*>(base + pl.s);
        uint32_t* Dw = reinterpret_cast<uint32_t*>(base + pl.d);
        hipLaunchKernelGGL((lpr_reserve_kernel<IP>), dim3(1), dim3(kResBlock), 0, st, Ap, a->n_rows, (int)kLprRows,
                           (int64_t)h->m, pl.groups, pl.sb, pl.nb, pl.caps.cap_a, pl.sd_words, GB, FILL, gate);
        HIP_TRY(hipGetLastError());
        const size_t plds = lpr_partition_lds_bytes(pl.caps.cap_a, pl.nb);
        HIP_TRY(hipFuncSetAttribute((const void*)lpr_partition_kernel<IP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)plds));
        const unsigned n_st = (n_tiles + kPartTiles - 1) / kPartTiles, s8 = (n_st + 7) / 8;
        hipLaunchKernelGGL((lpr_partition_kernel<IP>), dim3(8 * s8), dim3(kPBlock), plds, st, Ap, a->indices,
                           a->n_rows, pl.caps.cap_a, n_tiles, s8, pl.sb, pl.nb, pl.ostride, OFF2, CU,
                           (const int64_t*)GB, FILL, Sw, gate);
        HIP_TRY(hipGetLastError());
        const unsigned grid = 8u * (unsigned)((pl.nb + 7) / 8) * pl.groups;
        const size_t glds = (size_t)4 << (pl.sb - 5);
        HIP_TRY(hipFuncSetAttribute((const void*)lpr_gather_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)glds));
        hipLaunchKernelGGL(lpr_gather_kernel, dim3(grid), dim3(kGBlock), glds, st, (const uint32_t*)h->W32.p,
                           (const uint32_t*)h->BM.p, (const int64_t*)GB, (const uint32_t*)FILL, pl.sb, pl.nb,
                           pl.groups, (const uint32_t*)Sw, Dw, gate);
        HIP_TRY(hipGetLastError());
        const LprStage stg{gate, (const uint32_t*)h->W32.p, OFF2, CU, GB, Sw, Dw, pl.ostride, pl.nb};
        const size_t wlds = lpr_wave_lds_bytes(pl.lpr_slot, sizeof(T), pl.ucap, pl.nb);
        HIP_TRY(hipFuncSetAttribute((const void*)lpr_wave_kernel<T, IP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)wlds));
        hipLaunchKernelGGL((lpr_wave_kernel<T, IP>), dim3(8u * 4u * kPartTiles * s8), dim3(64), wlds,
                           st, R, mag, a->n_rows, Ap, a->indices, Ax, stg, pl.caps.cap_a, pl.ucap, n_tiles, s8, order,
                           sp, ws);
    } else {
        const size_t lds = lpr_lds_bytes(pl.caps.cap_a, sizeof(T), pl.lpr_slot);
        const void* fn = (const void*)lpr_main_flat_kernel<T, IP>;
        HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((lpr_main_flat_kernel<T, IP>), dim3(8 * t8), dim3(kLprRows), lds, st, R, mag,
                           a->n_rows, Ap, a->indices, Ax, (const uint32_t*)h->W32.p, pl.caps.cap_a, n_tiles, t8, order,
                           sp, ws);
    }
    HIP_TRY(hipGetLastError());
    const size_t hl = heavy_lds_bytes(h->p, sizeof(T));
    HIP_TRY(hipFuncSetAttribute((const void*)lpr_heavy_count_kernel<T, IP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)hl));
    hipLaunchKernelGGL((lpr_heavy_count_kernel<T, IP>), dim3(256), dim3(kBlock), hl, st, R, mag, a->n_rows, Ap,
                       a->indices, Ax, (int)h->p, sp, ws);
    HIP_TRY(hipGetLastError());
    const unsigned scan_blocks = (unsigned)((4 * (size_t)n_tiles + kBlock * kScanPer - 1) / (kBlock * kScanPer));
    hipLaunchKernelGGL(lpr_scan_kernel, dim3(scan_blocks), dim3(kBlock), 0, st, sp, 4 * (size_t)n_tiles,
                       (const unsigned long long*)(carry + (chunk & 1)), carry + ((chunk + 1) & 1), ws,
                       &ws->tile_counter);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL((lpr_copy_kernel<T, OP, OI>), dim3(std::min<unsigned>(n_tiles, 1u << 20)), dim3(kBlock), 0, st,
                       sp, a->n_rows, n_tiles, (OP*)c->indptr, (OI*)c->indices, (T*)c->data,
                       (unsigned long long)c->capacity, order);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipFuncSetAttribute((const void*)lpr_heavy_write_kernel<T, IP, OP, OI>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)hl));
    hipLaunchKernelGGL((lpr_heavy_write_kernel<T, IP, OP, OI>), dim3(256), dim3(kBlock), hl, st, R, mag, a->n_rows, Ap,
                       a->indices, Ax, (int)h->p, sp, ws, (OP*)c->indptr, (OI*)c->indices, (T*)c->data,
                       (unsigned long long)c->capacity, order);
    HIP_TRY(hipGetLastError());
    return RP_OK;
}

// The row-lane pipeline over chunks of pl.lpr_chunk rows (one chunk unless the launch is huge):
// chunk k sees the rows [k * chunk, ...) as its own CSR (indptr offset, entries indexed through it),
// writes its indptr slice and its entries at the running total of the chunks before it (a device
// carry slot), and re-zeroes the per-chunk header and states first. All on one stream. In auto
// staging mode lpr_choose_kernel samples the call's feature ids first and the host reads its
// verdict (4 bytes: the call's one wait, which lets only the chosen branch's kernels launch); a
// caller may pass the choice instead (*choice >= 0: 1 staged, 0 direct; the stream pipelines reuse
// their first chunk's), and gets back what was chosen. *choice == kChoiceOnDevice: the call must not
// wait on the host (rp_project_device without total_nnz: timing loops, graph capture), so the
// verdict stays on the device as the gate word and the staged branch is launched whatever it says:
// with gate 0 the reserve, partition and gather kernels return at once and the wave kernel gathers
// R's words directly (correct for any columns; on far-from-uniform columns slower than the direct
// branch the host-read verdict launches).
constexpr int kChoiceOnDevice = -2;
template <typename T, typename IP, typename OP, typename OI>
int launch_lpr(const PackedR& R, T mag, rp_projector* h, const rp_csr_in* a, const rp_csr_out* c, int order,
               Workspace* ws, const Plan& pl, hipStream_t st, int* choice) {
    const int64_t n = a->n_rows, step = std::max<int64_t>(pl.lpr_chunk, 1);
    uint32_t* gate = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws) + pl.carry + 16);
    bool staged = pl.staged, on_device = false;
    if (pl.gated && n > 0) {  // staged or direct for this call: sampled on the device
        if (choice && *choice >= 0) {
            staged = *choice != 0;
        } else {
            hipLaunchKernelGGL((lpr_choose_kernel<IP>), dim3(1), dim3(1024), 0, st, (const IP*)a->indptr, a->indices, n,
                               gate);
            HIP_TRY(hipGetLastError());
            if (choice && *choice == kChoiceOnDevice) {
                on_device = true;  // the gate word carries the verdict to the staged kernels
            } else {
                uint32_t g = 0;
                HIP_TRY(hipMemcpyAsync(&g, gate, 4, hipMemcpyDeviceToHost, st));
                HIP_TRY(poll_stream(st));
                staged = g != 0;
            }
        }
    }
    if (choice && !on_device) *choice = staged ? 1 : 0;
    // the gate: staged until a segment overflows; 0 records a direct call (rp_project_choice)
    if (pl.staged && !on_device) HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)gate, staged ? 1u : 0u, 1, st));
    int64_t k = 0;
    for (int64_t r0 = 0; r0 < n; r0 += step, ++k) {
        rp_csr_in sa = *a;
        sa.n_rows = std::min(step, n - r0);
        sa.indptr = (const IP*)a->indptr + r0;
        sa.nnz = -1;
        rp_csr_out sc = *c;
        sc.indptr = (OP*)c->indptr + r0;
        if (k > 0) HIP_TRY(hipMemsetAsync(ws, 0, pl.head, st));  // the carry slots follow the header
        const int rc = launch_lpr_chunk<T, IP, OP, OI>(R, mag, h, &sa, &sc, order, ws, pl, staged, st, k);
        if (rc) return rc;
    }
    return RP_OK;
}

template <typename T, typename IP, typename OP, typename OI, typename RL>
int launch_typed(const RL& R, T mag, rp_projector* h, const rp_csr_in* a, const rp_csr_out* c,
                 int order, Workspace* ws, unsigned n_tiles, const Plan& pl, size_t lds,
                 hipStream_t st, int* choice) {
    if constexpr (std::is_same<RL, PackedR>::value) {
        if (pl.lpr) return launch_lpr<T, IP, OP, OI>(R, mag, h, a, c, order, ws, pl, st, choice);
    }
    return launch_main<T, IP, OP, OI, RL>(R, mag, h, a, c, order, ws, n_tiles, pl, lds, st);
}

template <typename T, typename RL>
int dispatch_idx(const RL& R, T mag, rp_projector* h, const rp_csr_in* a, const rp_csr_out* c,
                 int order, Workspace* ws, unsigned n_tiles, const Plan& caps, size_t lds,
                 hipStream_t st, int* choice) {
    const bool ip64 = a->indptr_type == RP_I64, op64 = c->indptr_type == RP_I64,
               oi64 = c->indices_type == RP_I64;
#define RP_L(IP, OP, OI) return launch_typed<T, IP, OP, OI, RL>(R, mag, h, a, c, order, ws, n_tiles, caps, lds, st, choice)
    if (!ip64 && !op64 && !oi64) RP_L(int32_t, int32_t, int32_t);
    if (!ip64 && op64 && !oi64) RP_L(int32_t, int64_t, int32_t);
    if (!ip64 && op64 && oi64) RP_L(int32_t, int64_t, int64_t);
    if (ip64 && !op64 && !oi64) RP_L(int64_t, int32_t, int32_t);
    if (ip64 && op64 && !oi64) RP_L(int64_t, int64_t, int32_t);
    if (ip64 && op64 && oi64) RP_L(int64_t, int64_t, int64_t);
    if (!ip64 && !op64 && oi64) RP_L(int32_t, int32_t, int64_t);
    RP_L(int64_t, int32_t, int64_t);
#undef RP_L
}

int ensure_generic_values(rp_projector* h, int T) {
    if (h->layout != RP_LAYOUT_GENERIC) return RP_OK;
    if (T == RP_F32) {
        if (!h->Bx32.p) return fail(RP_ERR_INVALID, "R was given as float64; compute type float32 would round R (use float64)");
        return RP_OK;
    }
    if (h->Bx64.p) return RP_OK;
    int rc = h->Bx64.ensure(sizeof(double) * (size_t)std::max<int64_t>(h->nnz, 1), h->device);
    if (rc) return rc;
    if (h->nnz > 0) {
        hipLaunchKernelGGL((convert_kernel<float, double>), dim3(1024), dim3(256), 0, nullptr,
                           (const float*)h->Bx32.p, (double*)h->Bx64.p, h->nnz);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipDeviceSynchronize());
    }
    return RP_OK;
}

// choice: the staging verdict of a row-lane call in auto mode (see launch_lpr); NULL or -1 = sample it
int project_device_impl(rp_projector* h, const rp_csr_in* a, const rp_csr_out* c, int order,
                        void* workspace, int64_t workspace_bytes, hipStream_t st,
                        int64_t* total_nnz, int64_t nnz_a_hint, int* choice = nullptr) {
    if (!a || !c) return fail(RP_ERR_INVALID, "NULL operand");
    if (a->n_rows < 0) return fail(RP_ERR_INVALID, "n_rows < 0");
    if (a->data_type != RP_F32 && a->data_type != RP_F64)
        return fail(RP_ERR_INVALID, "A data type must be RP_F32 or RP_F64");
    if ((a->indptr_type != RP_I32 && a->indptr_type != RP_I64) ||
        (c->indptr_type != RP_I32 && c->indptr_type != RP_I64) ||
        (c->indices_type != RP_I32 && c->indices_type != RP_I64))
        return fail(RP_ERR_INVALID, "index types must be RP_I32 or RP_I64");
    if (a->data_type == RP_F32 && h->value_type == RP_F64)
        return fail(RP_ERR_INVALID, "compute type must be upcast(A, R) = float64 for a float64 R");
    if (a->n_rows >= (int64_t)1 << 40) return fail(RP_ERR_UNSUPPORTED, "too many rows");
    int rc = ensure_generic_values(h, a->data_type);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(h->device));

    const int vs = dtype_size(a->data_type);
    Plan plan = make_plan(h, a->n_rows, nnz_a_hint, true, vs);
    if (workspace) {  // a smaller caller workspace: no staging, then no deferred output either
        if (workspace_bytes < (int64_t)plan.head)
            return fail(RP_ERR_INVALID, "workspace of %lld bytes < %zu needed", (long long)workspace_bytes,
                        plan.head);
        if (workspace_bytes < (int64_t)plan.total) plan = make_plan(h, a->n_rows, nnz_a_hint, false, vs);
        if (workspace_bytes < (int64_t)plan.total)
            plan = make_plan(h, a->n_rows, nnz_a_hint, false, vs, false);
    }
    const Caps& caps = plan.caps;
    const size_t lds = plan.lpr ? std::max({lpr_lds_bytes(caps.cap_a, (size_t)vs, plan.lpr_slot), heavy_lds_bytes(h->p, (size_t)vs),
                                            plan.staged ? lpr_partition_lds_bytes(caps.cap_a, plan.nb) : (size_t)0})
                                : lds_bytes_for(caps, dtype_size(a->data_type), h->p);
    if (lds > 160 * 1024 - 4096)
        return fail(RP_ERR_UNSUPPORTED, "p=%lld too large for the LDS accumulator (%zu bytes)",
                    (long long)h->p, lds);
    const int64_t n_tiles64 = plan.n_tiles;
    if (n_tiles64 >= (int64_t)1 << 31) return fail(RP_ERR_UNSUPPORTED, "too many tiles");
    const unsigned n_tiles = (unsigned)n_tiles64;
    Workspace* ws = (Workspace*)workspace;  // caller's: rp_project_workspace_bytes(h, n, nnz) bytes
    if (!ws) {
        rc = h->ws.ensure(plan.total, h->device);
        if (rc) return rc;
        ws = (Workspace*)h->ws.p;
    }
    HIP_TRY(hipMemsetAsync(ws, 0, plan.zero, st));  // header + look-back states only
    if (n_tiles == 0) {
        // empty A: indptr = [0] (a memset: no host source, so nothing to wait for unless asked)
        HIP_TRY(hipMemsetAsync(c->indptr, 0, (size_t)dtype_size(c->indptr_type), st));
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)&ws->staged_used, 0, 1, st));
        if (total_nnz) {
            HIP_TRY(hipStreamSynchronize(st));
            *total_nnz = 0;
        }
        return RP_OK;
    }
    if (h->layout == RP_LAYOUT_PACKED) {
        PackedR R{(const uint64_t*)h->W.p, (const uint16_t*)h->O.p, (const uint64_t*)h->SW.p,
                  (const uint32_t*)h->BM.p, h->BM.p ? (uint32_t)(8 * h->m) : 0u};
        rc = a->data_type == RP_F64
                 ? dispatch_idx<double, PackedR>(R, h->mag, h, a, c, order, ws, n_tiles, plan, lds, st, choice)
                 : dispatch_idx<float, PackedR>(R, (float)h->mag, h, a, c, order, ws, n_tiles, plan, lds, st, choice);
    } else if (a->data_type == RP_F64) {
        GenericR<double> R{(const int32_t*)h->Bp.p, (const uint16_t*)h->Bj.p, (const double*)h->Bx64.p};
        rc = dispatch_idx<double, GenericR<double>>(R, 0.0, h, a, c, order, ws, n_tiles, plan, lds, st, choice);
    } else {
        GenericR<float> R{(const int32_t*)h->Bp.p, (const uint16_t*)h->Bj.p, (const float*)h->Bx32.p};
        rc = dispatch_idx<float, GenericR<float>>(R, 0.0f, h, a, c, order, ws, n_tiles, plan, lds, st, choice);
    }
    if (rc) return rc;
    // what ran, for rp_project_choice: the row-lane gate when staged (the device's choice, or a
    // segment overflow that sent the call to the direct kernel), else the plan's staging
    if (plan.lpr && plan.staged)
        HIP_TRY(hipMemcpyAsync(&ws->staged_used, reinterpret_cast<char*>(ws) + plan.carry + 16, 4,
                               hipMemcpyDeviceToDevice, st));
    else
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)&ws->staged_used, plan.staged ? 1 : 0, 1, st));
    if (total_nnz) {
        Workspace hw;
        HIP_TRY(hipMemcpyAsync(&hw, ws, sizeof hw, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (hw.error) return fail(RP_ERR_TIMEOUT, "device look-back wait expired");
        *total_nnz = (int64_t)hw.total;
        if ((int64_t)hw.total > c->capacity)
            return fail(RP_ERR_CAPACITY, "output capacity %lld < nnz %lld", (long long)c->capacity,
                        (long long)hw.total);
    }
    return RP_OK;
}

// ---- host-side R image (packed single-magnitude layout, or generic CSR)
struct HostImage {
    int layout = RP_LAYOUT_GENERIC;
    double mag = 0.0;
    int bs = 0;
    int64_t nnz = 0, b0 = 0;
    std::vector<uint64_t> W;
    std::vector<uint16_t> O;
    std::vector<int32_t> Bp;
    std::vector<uint16_t> Bj;
};

int build_image(int64_t m, int64_t p, const void* indptr, int32_t indptr_type, const void* indices,
                int32_t indices_type, const void* data, int32_t data_type, int32_t layout,
                HostImage& img) {
    if (m < 0 || p <= 0) return fail(RP_ERR_INVALID, "bad shape (%lld, %lld)", (long long)m, (long long)p);
    if (!indptr || (indptr_type != RP_I32 && indptr_type != RP_I64) ||
        (indices_type != RP_I32 && indices_type != RP_I64) ||
        (data_type != RP_F32 && data_type != RP_F64))
        return fail(RP_ERR_INVALID, "bad R arrays");
    if (layout != RP_LAYOUT_AUTO && layout != RP_LAYOUT_GENERIC && layout != RP_LAYOUT_PACKED)
        return fail(RP_ERR_INVALID, "bad layout %d", layout);
    if (p > 32767) return fail(RP_ERR_UNSUPPORTED, "p=%lld > 32767 not supported by the GPU path", (long long)p);
    if (m >= ((int64_t)1 << 31)) return fail(RP_ERR_UNSUPPORTED, "m >= 2^31");
    const int64_t b0 = ptr_at(indptr, indptr_type, 0);
    const int64_t nnz = ptr_at(indptr, indptr_type, m) - b0;
    if (nnz < 0 || nnz >= ((int64_t)1 << 31) - 1) return fail(RP_ERR_UNSUPPORTED, "R nnz out of range");
    if (nnz > 0 && (!indices || !data)) return fail(RP_ERR_INVALID, "NULL R indices/data");
    for (int64_t j = 0; j < m; ++j)
        if (ptr_at(indptr, indptr_type, j + 1) < ptr_at(indptr, indptr_type, j))
            return fail(RP_ERR_INVALID, "R indptr not monotone");
    // validate columns and detect the single-magnitude layout
    double mag = 0.0;
    bool single = p <= 16384 && nnz > 0;
    for (int64_t q = 0; q < nnz; ++q) {
        const int64_t col = ptr_at(indices, indices_type, b0 + q);
        if (col < 0 || col >= p) return fail(RP_ERR_INVALID, "R column index %lld out of range", (long long)col);
        if (single) {
            const double v = val_at(data, data_type, b0 + q);
            const double av = std::fabs(v);
            if (q == 0) mag = av;
            if (!(av == mag) || av == 0.0 || std::isnan(v)) single = false;
        }
    }
    if (layout == RP_LAYOUT_PACKED && !single)
        return fail(RP_ERR_UNSUPPORTED, "R does not qualify for the packed layout");
    img.nnz = nnz;
    img.b0 = b0;
    if (!(single && layout != RP_LAYOUT_GENERIC)) {
        img.layout = RP_LAYOUT_GENERIC;
        img.Bp.resize((size_t)m + 1);
        img.Bj.resize((size_t)nnz);
        for (int64_t j = 0; j <= m; ++j) img.Bp[(size_t)j] = (int32_t)(ptr_at(indptr, indptr_type, j) - b0);
        for (int64_t q = 0; q < nnz; ++q) img.Bj[(size_t)q] = (uint16_t)ptr_at(indices, indices_type, b0 + q);
        return RP_OK;
    }
    img.layout = RP_LAYOUT_PACKED;
    img.mag = mag;
    img.bs = 0;
    img.W.assign((size_t)m, 0);
    img.O.clear();
    for (int64_t j = 0; j < m; ++j) {
        const int64_t s0 = ptr_at(indptr, indptr_type, j), t0 = ptr_at(indptr, indptr_type, j + 1);
        const int64_t cnt = t0 - s0;
        if (cnt <= 4) {
            uint64_t w = (uint64_t)cnt << 61;
            for (int64_t q = 0; q < cnt; ++q) {
                const uint64_t col = (uint64_t)ptr_at(indices, indices_type, s0 + q);
                const bool neg = val_at(data, data_type, s0 + q) < 0;
                w |= ((neg ? 0x4000ull : 0ull) | col) << (15 * q);
            }
            img.W[(size_t)j] = w;
        } else {
            img.W[(size_t)j] = kOvf | (uint64_t)img.O.size();
            img.O.push_back((uint16_t)cnt);
            for (int64_t q = 0; q < cnt; ++q) {
                const uint32_t col = (uint32_t)ptr_at(indices, indices_type, s0 + q);
                const bool neg = val_at(data, data_type, s0 + q) < 0;
                img.O.push_back((uint16_t)((neg ? 0x8000u : 0u) | col));
            }
        }
    }
    return RP_OK;
}

// the three buffers of an image: packed W/O/-, or generic Bp/Bj/values (values from the caller)
void image_parts(const HostImage& img, const void* data, int32_t data_type, const void* src[3],
                 int64_t bytes[3]) {
    if (img.layout == RP_LAYOUT_PACKED) {
        src[0] = img.W.data(); bytes[0] = 8 * (int64_t)img.W.size();
        src[1] = img.O.data(); bytes[1] = 2 * (int64_t)img.O.size();
        src[2] = nullptr; bytes[2] = 0;
    } else {
        const int vs = dtype_size(data_type);
        src[0] = img.Bp.data(); bytes[0] = 4 * (int64_t)img.Bp.size();
        src[1] = img.Bj.data(); bytes[1] = 2 * (int64_t)img.Bj.size();
        src[2] = data ? (const char*)data + (size_t)vs * (size_t)img.b0 : nullptr;
        bytes[2] = (int64_t)vs * img.nnz;
    }
}

}  // namespace

// ==========================================================================================
// C-ABI
extern "C" {


const char* rp_last_error(void) { return g_err.c_str(); }
const char* rp_version(void) { return "rp-mi355x 0.1 (gfx950)"; }

int rp_abi_version(void) { return RP_ABI_VERSION; }

// The sha256 prefix of every source this library was compiled from (build.py passes it as
// RP_SRC_SHA16 and also finds it in the binary through the marker), so a benched or tested number
// names the binary that produced it and a stale build is refused (build.py / _native.load).
#ifndef RP_SRC_SHA16
#define RP_SRC_SHA16 "unknown"
#endif
__attribute__((used)) static const char kBuildMarker[] = "rp-src-sha16:" RP_SRC_SHA16;
// the compiler identity hash (build.py compiler_hash) the source id above includes: the loader
// recomputes the id with it instead of running the compiler
#ifndef RP_CC_SHA16
#define RP_CC_SHA16 "unknown"
#endif
__attribute__((used)) static const char kCcMarker[] = "rp-cc-sha16:" RP_CC_SHA16;
const char* rp_build_id(void) { return kBuildMarker + 13; }

int rp_device_count(int* count) {
    if (!count) return fail(RP_ERR_INVALID, "NULL count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(RP_ERR_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *count = n;
    return RP_OK;
}

namespace {
// the staged-gather table (u32 per feature) derived from the uploaded W
int build_w32(rp_projector* h) {
    if (h->layout != RP_LAYOUT_PACKED || h->m <= 0 || h->m > ((int64_t)1 << 26)) return RP_OK;
    int rc = h->W32.ensure(4 * (size_t)h->m, h->device);
    if (rc) return rc;
    // side table: count the features with > 2 entries per 1024-feature block, scan, then write
    const int64_t nblk = (h->m + kSideBlock - 1) / kSideBlock;
    DevBuf cnt, tmp;
    if ((rc = cnt.ensure(8 * (size_t)nblk, h->device))) return rc;
    hipLaunchKernelGGL(side_count_kernel, dim3((unsigned)nblk), dim3(kSideBlock), 0, nullptr,
                       (const uint64_t*)h->W.p, h->m, (int64_t*)cnt.p);
    HIP_TRY(hipGetLastError());
    if ((rc = rpd::inclusive_scan_i64((int64_t*)cnt.p, nblk, nullptr, tmp, h->device))) return rc;
    int64_t nside = 0;
    HIP_TRY(hipMemcpy(&nside, (int64_t*)cnt.p + nblk - 1, 8, hipMemcpyDeviceToHost));
    if ((rc = h->SW.ensure(8 * (size_t)std::max<int64_t>(nside, 1), h->device))) return rc;
    hipLaunchKernelGGL(build_w32_kernel, dim3((unsigned)nblk), dim3(kSideBlock), 0, nullptr, (const uint64_t*)h->W.p,
                       (const uint16_t*)h->O.p, (const int64_t*)cnt.p, (uint32_t*)h->W32.p, (uint64_t*)h->SW.p, h->m);
    HIP_TRY(hipGetLastError());
    // bitmap padded to whole 2^20-feature slices so a gather workgroup can stage any slice
    const size_t bm_words = (size_t)((h->m + (1 << 20) - 1) >> 20) << 15;
    rc = h->BM.ensure(4 * bm_words, h->device);
    if (rc) return rc;
    HIP_TRY(hipMemset(h->BM.p, 0, 4 * bm_words));
    hipLaunchKernelGGL(build_bitmap_kernel, dim3(2048), dim3(256), 0, nullptr, (const uint64_t*)h->W.p,
                       (uint32_t*)h->BM.p, h->m);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());  // cnt / tmp are released on return
    return RP_OK;
}
}  // namespace

int rp_projector_create(int device, int64_t m, int64_t p, const void* indptr, int32_t indptr_type,
                        const void* indices, int32_t indices_type, const void* data,
                        int32_t data_type, int32_t layout, rp_projector** out) {
    if (!out) return fail(RP_ERR_INVALID, "NULL out");
    *out = nullptr;
    HostImage img;
    int rc = build_image(m, p, indptr, indptr_type, indices, indices_type, data, data_type, layout, img);
    if (rc) return rc;
    rp_projector* h = new (std::nothrow) rp_projector();
    if (!h) return fail(RP_ERR_NOMEM, "out of host memory");
    h->device = device;
    h->m = m;
    h->p = p;
    h->nnz = img.nnz;
    h->value_type = data_type;
    h->layout = img.layout;
    h->mag = img.mag;
    h->bs = img.bs;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete h;
        return fail(RP_ERR_HIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
    }
    const void* src[3];
    int64_t bytes[3];
    image_parts(img, data, data_type, src, bytes);
    DevBuf* dst[3];
    if (img.layout == RP_LAYOUT_PACKED) {
        dst[0] = &h->W; dst[1] = &h->O; dst[2] = &h->spare;
    } else {
        dst[0] = &h->Bp; dst[1] = &h->Bj; dst[2] = data_type == RP_F64 ? &h->Bx64 : &h->Bx32;
    }
    for (int i = 0; i < 3; ++i) {
        if ((rc = dst[i]->ensure((size_t)std::max<int64_t>(bytes[i], 2), device))) {
            delete h;
            return rc;
        }
        dst[i]->bytes = (size_t)bytes[i];
        if (bytes[i] > 0) e = hipMemcpy(dst[i]->p, src[i], (size_t)bytes[i], hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            delete h;
            return fail(RP_ERR_HIP, "R upload failed: %s", hipGetErrorString(e));
        }
    }
    if ((rc = build_w32(h))) {
        delete h;
        return rc;
    }
    *out = h;
    return RP_OK;
}

int rp_pack_r_host(int64_t m, int64_t p, const void* indptr, int32_t indptr_type, const void* indices,
                   int32_t indices_type, const void* data, int32_t data_type, int32_t layout,
                   rp_projector_info* info, void* buf0, void* buf1, void* buf2) {
    if (!info) return fail(RP_ERR_INVALID, "NULL info");
    HostImage img;
    int rc = build_image(m, p, indptr, indptr_type, indices, indices_type, data, data_type, layout, img);
    if (rc) return rc;
    std::memset(info, 0, sizeof *info);
    info->m = m;
    info->p = p;
    info->nnz = img.nnz;
    info->layout = img.layout;
    info->value_type = data_type;
    info->magnitude = img.mag;
    info->block_shift = img.bs;
    info->n_buffers = 3;
    const void* src[3];
    int64_t bytes[3];
    image_parts(img, data, data_type, src, bytes);
    void* dst[3] = {buf0, buf1, buf2};
    for (int i = 0; i < 3; ++i) {
        info->buffer_bytes[i] = bytes[i];
        if (dst[i] && bytes[i] > 0) std::memcpy(dst[i], src[i], (size_t)bytes[i]);
    }
    return RP_OK;
}

int rp_projector_info_get(const rp_projector* h, rp_projector_info* out) {
    if (!h || !out) return fail(RP_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    out->m = h->m;
    out->p = h->p;
    out->nnz = h->nnz;
    out->layout = h->layout;
    out->value_type = h->value_type;
    out->magnitude = h->mag;
    out->block_shift = h->bs;
    if (h->layout == RP_LAYOUT_PACKED) {
        out->n_buffers = 3;
        out->buffer_bytes[0] = (int64_t)h->W.bytes;
        out->buffer_bytes[1] = (int64_t)h->O.bytes;
        out->buffer_bytes[2] = 0;
    } else {
        out->n_buffers = 3;
        out->buffer_bytes[0] = (int64_t)h->Bp.bytes;
        out->buffer_bytes[1] = (int64_t)h->Bj.bytes;
        const DevBuf& bx = h->value_type == RP_F64 ? h->Bx64 : h->Bx32;
        out->buffer_bytes[2] = (int64_t)bx.bytes;
    }
    return RP_OK;
}

static const DevBuf* image_buffer(const rp_projector* h, int which) {
    if (h->layout == RP_LAYOUT_PACKED) {
        const DevBuf* b[3] = {&h->W, &h->O, &h->spare};
        return (which >= 0 && which < 3) ? b[which] : nullptr;
    }
    const DevBuf* b[3] = {&h->Bp, &h->Bj, h->value_type == RP_F64 ? &h->Bx64 : &h->Bx32};
    return (which >= 0 && which < 3) ? b[which] : nullptr;
}

int rp_projector_export(const rp_projector* h, int32_t which, void* dst_device, void* stream) {
    if (!h || !dst_device) return fail(RP_ERR_INVALID, "NULL argument");
    const DevBuf* b = image_buffer(h, which);
    if (!b) return fail(RP_ERR_INVALID, "buffer index %d out of range", which);
    HIP_TRY(hipSetDevice(h->device));
    if (b->bytes)
        HIP_TRY(hipMemcpyAsync(dst_device, b->p, b->bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return RP_OK;
}

int rp_projector_create_from_device(int device, const rp_projector_info* info,
                                    const void* const* buffers, rp_projector** out) {
    if (!info || !buffers || !out) return fail(RP_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (info->layout != RP_LAYOUT_PACKED && info->layout != RP_LAYOUT_GENERIC)
        return fail(RP_ERR_INVALID, "bad layout");
    rp_projector* h = new (std::nothrow) rp_projector();
    if (!h) return fail(RP_ERR_NOMEM, "out of host memory");
    h->device = device;
    h->m = info->m;
    h->p = info->p;
    h->nnz = info->nnz;
    h->layout = info->layout;
    h->value_type = info->value_type;
    h->mag = info->magnitude;
    h->bs = info->block_shift;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete h;
        return fail(RP_ERR_HIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
    }
    DevBuf* dst[3];
    if (h->layout == RP_LAYOUT_PACKED) {
        dst[0] = &h->W; dst[1] = &h->O; dst[2] = &h->spare;
    } else {
        dst[0] = &h->Bp; dst[1] = &h->Bj; dst[2] = h->value_type == RP_F64 ? &h->Bx64 : &h->Bx32;
    }
    for (int i = 0; i < 3; ++i) {
        int rc = dst[i]->ensure((size_t)std::max<int64_t>(info->buffer_bytes[i], 2), device);
        if (rc) { delete h; return rc; }
        dst[i]->bytes = (size_t)info->buffer_bytes[i];
        if (info->buffer_bytes[i] > 0) {
            e = hipMemcpy(dst[i]->p, buffers[i], (size_t)info->buffer_bytes[i], hipMemcpyDeviceToDevice);
            if (e != hipSuccess) { delete h; return fail(RP_ERR_HIP, "image copy: %s", hipGetErrorString(e)); }
        }
    }
    if (int rc = build_w32(h)) {
        delete h;
        return rc;
    }
    *out = h;
    return RP_OK;
}

int rp_projector_destroy(rp_projector* h) {
    delete h;
    return RP_OK;
}

int64_t rp_project_workspace_bytes(const rp_projector* h, int64_t n_rows, int64_t nnz_a) {
    if (!h || n_rows < 0) return -1;
    if (nnz_a < 0) {  // unknown nnz: look-back states for the worst case (one row per tile) only
        const int64_t tiles = n_rows > 0 ? n_rows : 1;
        return (int64_t)((sizeof(Workspace) + 8 * (size_t)tiles + 255) & ~size_t(255));
    }
    return (int64_t)make_plan(h, n_rows, nnz_a).total;
}

int64_t rp_project_workspace_bytes_for(const rp_projector* h, int64_t n_rows, int64_t nnz_a, int32_t data_type) {
    if (data_type != RP_F32 && data_type != RP_F64) return -1;
    if (!h || n_rows < 0 || nnz_a < 0) return rp_project_workspace_bytes(h, n_rows, nnz_a);
    return (int64_t)make_plan(h, n_rows, nnz_a, true, dtype_size(data_type)).total;
}

int rp_project_plan(const rp_projector* h, int64_t n_rows, int64_t nnz_a, int32_t* pipeline, int32_t* staged,
                    int32_t* bucket_shift) {
    if (!h || n_rows < 0) return fail(RP_ERR_INVALID, "NULL projector or n_rows < 0");
    const Plan pl = make_plan(h, n_rows, nnz_a);
    if (pipeline) *pipeline = pl.lpr ? RP_PIPE_ROWLANE : RP_PIPE_TILE;
    if (staged) *staged = pl.gated ? 2 : pl.staged ? 1 : 0;
    if (bucket_shift) *bucket_shift = pl.staged ? pl.sb : 0;
    return RP_OK;
}

int rp_project_choice(const rp_projector* h, int64_t n_rows, int64_t nnz_a, const void* workspace,
                      int32_t* staged) {
    if (!h || !staged) return fail(RP_ERR_INVALID, "NULL argument");
    (void)n_rows;
    (void)nnz_a;
    if (!workspace) return fail(RP_ERR_INVALID, "the choice lives in the caller's workspace");
    // every call records what ran in its workspace header (after all its kernels, on its stream);
    // the caller has synchronised that stream (documented in rp.h)
    uint32_t g = 0;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipMemcpy(&g, &reinterpret_cast<const Workspace*>(workspace)->staged_used, 4, hipMemcpyDeviceToHost));
    *staged = g ? 1 : 0;
    return RP_OK;
}

int rp_projector_set_staging(rp_projector* h, int32_t mode, int32_t bucket_shift) {
    if (!h) return fail(RP_ERR_INVALID, "NULL projector");
    if (mode < -1 || mode > 1) return fail(RP_ERR_INVALID, "mode must be -1 (auto), 0 (off) or 1 (on)");
    if (bucket_shift != 0 && (bucket_shift < 1 || bucket_shift > 20))
        return fail(RP_ERR_INVALID, "bucket_shift must be 0 (auto) or in [1, 20]");
    if (mode == 1 && !h->W32.p)
        return fail(RP_ERR_UNSUPPORTED, "staged gather needs the packed layout and m <= 2^26");
    const int sb = bucket_shift > 0 ? bucket_shift : 20;
    if (mode == 1 && ((h->m + ((int64_t)1 << sb) - 1) >> sb) > kStageMaxNB)
        return fail(RP_ERR_INVALID, "m=%lld needs more than %d buckets of 2^%d features", (long long)h->m,
                    kStageMaxNB, sb);
    h->stage_mode = mode;
    h->stage_sb = bucket_shift;
    return RP_OK;
}

int rp_projector_set_option(rp_projector* h, int32_t option, int64_t value) {
    if (!h) return fail(RP_ERR_INVALID, "NULL projector");
    switch (option) {
        case RP_OPT_PIPELINE:
            if (value < 0 || value > 2) return fail(RP_ERR_INVALID, "pipeline must be 0 (auto), 1 (tile) or 2 (row-lane)");
            h->opt_pipeline = (int)value;
            return RP_OK;
        case RP_OPT_DEFER_POLLS:
            h->opt_defer_polls = (int)std::max<int64_t>(std::min<int64_t>(value, 1 << 30), -2);
            return RP_OK;
        case RP_OPT_DEFER_TICKS:
            h->opt_defer_ticks = (int)std::max<int64_t>(std::min<int64_t>(value, 1 << 30), -1);
            return RP_OK;
        case RP_OPT_CHUNK_ROWS:
            h->opt_chunk_rows = std::max<int64_t>(value, 0);
            return RP_OK;
        case RP_OPT_HOST_THREADS:
            h->opt_host_threads = (int)std::max<int64_t>(std::min<int64_t>(value, 256), -1);
            return RP_OK;

        default:
            return fail(RP_ERR_INVALID, "unknown option %d", option);
    }
}

int rp_projector_get_option(const rp_projector* h, int32_t option, int64_t* value) {
    if (!h || !value) return fail(RP_ERR_INVALID, "NULL argument");
    switch (option) {
        case RP_OPT_PIPELINE: *value = h->opt_pipeline; return RP_OK;
        case RP_OPT_DEFER_POLLS: *value = h->opt_defer_polls; return RP_OK;
        case RP_OPT_DEFER_TICKS: *value = h->opt_defer_ticks; return RP_OK;
        case RP_OPT_CHUNK_ROWS: *value = h->opt_chunk_rows; return RP_OK;
        case RP_OPT_HOST_THREADS: *value = h->opt_host_threads; return RP_OK;
        default: return fail(RP_ERR_INVALID, "unknown option %d", option);
    }
}

int rp_project_device(rp_projector* h, const rp_csr_in* a, const rp_csr_out* c, int32_t order,
                      void* workspace, int64_t workspace_bytes, void* stream, int64_t* total_nnz) {
    if (!h) return fail(RP_ERR_INVALID, "NULL projector");
    if (order != RP_ORDER_SCIPY && order != RP_ORDER_SORTED) return fail(RP_ERR_INVALID, "bad order");
    HIP_TRY(hipSetDevice(h->device));
    // under stream capture nothing may wait on the host: the caller's workspace, a known nnz(A) and
    // no total_nnz are then required (each of the others makes the call synchronise)
    hipStreamCaptureStatus cap_status = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cap_status) != hipSuccess) {
        (void)hipGetLastError();  // the legacy stream cannot capture; clear the sticky error
        cap_status = hipStreamCaptureStatusNone;
    }
    if (cap_status != hipStreamCaptureStatusNone && (total_nnz || !workspace || !a || a->nnz < 0))
        return fail(RP_ERR_INVALID, "under stream capture rp_project_device needs a caller workspace, a->nnz >= 0 "
                                    "and total_nnz == NULL (each of these would wait on the host)");
    // nnz(A) for tile sizing: given, or read from the two ends of indptr (tiny D2H)
    int64_t nnz_a = a ? a->nnz : -1;
    if (a && nnz_a < 0 && a->n_rows > 0 && a->indptr) {
        HIP_TRY(hipSetDevice(h->device));
        const int es = dtype_size(a->indptr_type);
        if (es == 0) return fail(RP_ERR_INVALID, "bad indptr type");
        int64_t first = 0, last = 0;
        HIP_TRY(hipMemcpyAsync(&first, a->indptr, es, hipMemcpyDeviceToHost, (hipStream_t)stream));
        HIP_TRY(hipMemcpyAsync(&last, (const char*)a->indptr + es * a->n_rows, es, hipMemcpyDeviceToHost,
                               (hipStream_t)stream));
        HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
        if (es == 4) {
            first = (int32_t)first;
            last = (int32_t)last;
        }
        nnz_a = last - first;
    }
    if (!workspace) {
        // the projector's own workspace is shared by every caller of this handle (and by the host
        // path): serialise on the handle and finish the work before releasing it, so no launch on
        // another stream can reset the look-back header or reallocate the buffer under this one
        std::lock_guard<std::mutex> lock(h->mu);
        int rc = project_device_impl(h, a, c, order, nullptr, 0, (hipStream_t)stream, total_nnz, nnz_a);
        if (rc == RP_OK) HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
        return rc;
    }
    // without total_nnz the call is fully asynchronous: the staging verdict stays on the device
    int choice = total_nnz ? -1 : kChoiceOnDevice;
    return project_device_impl(h, a, c, order, workspace, workspace_bytes, (hipStream_t)stream,
                               total_nnz, nnz_a, &choice);
}

int rp_project_host_begin(rp_projector* h, const rp_csr_in* a, int32_t order, rp_result** out,
                          int64_t* nnz) {
    if (!h || !a || !out || !nnz) return fail(RP_ERR_INVALID, "NULL argument");
    if (order != RP_ORDER_SCIPY && order != RP_ORDER_SORTED) return fail(RP_ERR_INVALID, "bad order");
    *out = nullptr;
    const int ips = dtype_size(a->indptr_type), vs = dtype_size(a->data_type);
    if (!ips || (a->data_type != RP_F32 && a->data_type != RP_F64)) return fail(RP_ERR_INVALID, "bad A types");
    if (a->n_rows < 0 || !a->indptr) return fail(RP_ERR_INVALID, "bad A");
    const int64_t n = a->n_rows;
    const int64_t b0 = ptr_at(a->indptr, a->indptr_type, 0);
    const int64_t nnz_a = ptr_at(a->indptr, a->indptr_type, n) - b0;
    if (nnz_a < 0) return fail(RP_ERR_INVALID, "A indptr decreasing");
    // the kernels index A through indptr: it must be monotone (O(n) here); the column indices are
    // checked on the device after the upload (O(nnz) there, not on the host)
    for (int64_t i = 0; i < n; ++i)
        if (ptr_at(a->indptr, a->indptr_type, i + 1) < ptr_at(a->indptr, a->indptr_type, i))
            return fail(RP_ERR_INVALID, "A indptr decreasing at row %lld", (long long)i);
    std::lock_guard<std::mutex> lock(h->mu);
    HIP_TRY(hipSetDevice(h->device));
    rp_result* r = new (std::nothrow) rp_result();
    if (!r) return fail(RP_ERR_NOMEM, "out of host memory");
    r->h = h;
    r->n_rows = n;
    r->value_type = a->data_type;
    int rc;
    // upload A (indptr rebased to 0, as int64)
    if ((rc = h->a_ptr.ensure(8 * (size_t)(n + 1), h->device)) ||
        (rc = h->a_idx.ensure(4 * (size_t)std::max<int64_t>(nnz_a, 1), h->device)) ||
        (rc = h->a_val.ensure((size_t)vs * (size_t)std::max<int64_t>(nnz_a, 1), h->device))) {
        delete r;
        return rc;
    }
    // indptr goes up as given (into the tail of a_ptr when int32) and is rebased to int64 on the device
    const size_t grid = (size_t)std::min<int64_t>(std::max<int64_t>((n + 256) / 256, 1), 65536);
    hipError_t e;
    if (a->indptr_type == RP_I64) {
        e = hipMemcpy(h->a_ptr.p, a->indptr, 8 * (size_t)(n + 1), hipMemcpyHostToDevice);
        if (e == hipSuccess && b0 != 0)
            hipLaunchKernelGGL((rebase_kernel<int64_t, int64_t>), dim3((unsigned)grid), dim3(256), 0, nullptr,
                               (const int64_t*)h->a_ptr.p, (int64_t*)h->a_ptr.p, n + 1, -b0);
    } else {
        if ((rc = r->cp.ensure(4 * (size_t)(n + 1), h->device))) {  // scratch for the int32 copy
            delete r;
            return rc;
        }
        e = hipMemcpy(r->cp.p, a->indptr, 4 * (size_t)(n + 1), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            hipLaunchKernelGGL((rebase_kernel<int32_t, int64_t>), dim3((unsigned)grid), dim3(256), 0, nullptr,
                               (const int32_t*)r->cp.p, (int64_t*)h->a_ptr.p, n + 1, -b0);
    }
    if (e == hipSuccess && nnz_a > 0)
        e = hipMemcpy(h->a_idx.p, a->indices + b0, 4 * (size_t)nnz_a, hipMemcpyHostToDevice);
    if (e == hipSuccess && nnz_a > 0)
        e = hipMemcpy(h->a_val.p, (const char*)a->data + (size_t)vs * (size_t)b0, (size_t)vs * (size_t)nnz_a,
                      hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        delete r;
        return fail(RP_ERR_HIP, "A upload: %s", hipGetErrorString(e));
    }
    if (nnz_a > 0) {
        if ((rc = h->ws_check.ensure(8, h->device))) {
            delete r;
            return rc;
        }
        const unsigned long long none = ~0ull;
        HIP_TRY(hipMemcpy(h->ws_check.p, &none, 8, hipMemcpyHostToDevice));
        const unsigned cg = (unsigned)std::min<int64_t>((nnz_a + 255) / 256, 16384);
        hipLaunchKernelGGL(check_columns_kernel, dim3(cg), dim3(256), 0, nullptr, (const int32_t*)h->a_idx.p,
                           nnz_a, h->m, (unsigned long long*)h->ws_check.p);
        unsigned long long bad = 0;
        HIP_TRY(hipMemcpy(&bad, h->ws_check.p, 8, hipMemcpyDeviceToHost));
        if (bad != ~0ull) {
            const int32_t j = a->indices[b0 + (int64_t)bad];
            delete r;
            return fail(RP_ERR_INVALID, "A column index %d out of range [0, %lld)", j, (long long)h->m);
        }
    }
    rp_csr_in ad{n, h->a_ptr.p, RP_I64, (const int32_t*)h->a_idx.p, h->a_val.p, a->data_type, nnz_a};
    // capacity guess from the expected products, exact retry on overflow
    const double ppe = h->m > 0 ? (double)h->nnz / (double)h->m : 0.0;
    int64_t cap = (int64_t)(1.25 * ppe * (double)nnz_a) + 1024;
    for (int attempt = 0; attempt < 2; ++attempt) {
        if ((rc = r->cp.ensure(8 * (size_t)(n + 1), h->device)) ||
            (rc = r->cj.ensure(4 * (size_t)cap, h->device)) ||
            (rc = r->cx.ensure((size_t)vs * (size_t)cap, h->device))) {
            delete r;
            return rc;
        }
        rp_csr_out cd{r->cp.p, RP_I64, r->cj.p, RP_I32, r->cx.p, cap};
        int64_t total = 0;
        rc = project_device_impl(h, &ad, &cd, order, nullptr, 0, nullptr, &total, nnz_a);
        if (rc == RP_ERR_CAPACITY && attempt == 0) {
            cap = total;
            continue;
        }
        if (rc) {
            delete r;
            return rc;
        }
        r->nnz = total;
        break;
    }
    *nnz = r->nnz;
    *out = r;
    return RP_OK;
}

namespace {
// D2H into caller memory that may be freshly allocated: the first touch of each page faults and
// zero-fills it, ~75 ms per GB in a process with the HIP runtime loaded, barely faster with more
// threads (scripts/probes/d2h_probe.py), versus ~56 GB/s for the copy into touched memory. The
// Python layer therefore hands out recycled memory (hostmem.py); for other callers a few worker
// threads pre-fault the destinations chunk by chunk, in copy order, while the calling thread copies
// the chunks already faulted in (4M KDD2012 rows: 30.5 -> 26.6 ms with 4 threads, 28.4 with 16).
struct D2HJob {
    void* dst;
    const void* src;
    size_t bytes;
};

unsigned host_threads(const rp_projector* h) {  // RP_OPT_HOST_THREADS; 0/1: no helper threads
    if (h->opt_host_threads >= 0) return (unsigned)h->opt_host_threads;
    const unsigned hw = std::thread::hardware_concurrency();
    return std::min(4u, hw > 1 ? hw : 1u);
}

int fetch_d2h(const rp_projector* h, const std::vector<D2HJob>& jobs) {
    constexpr size_t kChunk = 8u << 20, kPage = 4096, kMinPipelined = 16u << 20;
    size_t total = 0;
    for (const auto& j : jobs) total += j.bytes;
    const unsigned nt = host_threads(h);
    if (total < kMinPipelined || nt < 2) {
        for (const auto& j : jobs)
            if (j.bytes) HIP_TRY(hipMemcpy(j.dst, j.src, j.bytes, hipMemcpyDeviceToHost));
        return RP_OK;
    }
    std::vector<D2HJob> ch;
    for (const auto& j : jobs)
        for (size_t o = 0; o < j.bytes; o += kChunk)
            ch.push_back({(char*)j.dst + o, (const char*)j.src + o, std::min(kChunk, j.bytes - o)});
    std::vector<std::atomic<int>> ready(ch.size());
    for (auto& f : ready) f.store(0, std::memory_order_relaxed);
    std::atomic<bool> stop{false};
    const unsigned nw = (unsigned)std::min<size_t>(nt, ch.size());
    std::vector<std::thread> workers;
    workers.reserve(nw);
    for (unsigned w = 0; w < nw; ++w)
        workers.emplace_back([&, w] {
            for (size_t c = w; c < ch.size() && !stop.load(std::memory_order_relaxed); c += nw) {
                volatile char* d = (volatile char*)ch[c].dst;
                for (size_t o = 0; o < ch[c].bytes; o += kPage) d[o] = 0;  // overwritten by the copy
                ready[c].store(1, std::memory_order_release);
            }
        });
    hipError_t e = hipSuccess;
    for (size_t c = 0; c < ch.size() && e == hipSuccess; ++c) {
        while (!ready[c].load(std::memory_order_acquire)) std::this_thread::yield();
        e = hipMemcpy(ch[c].dst, ch[c].src, ch[c].bytes, hipMemcpyDeviceToHost);
    }
    stop.store(true, std::memory_order_relaxed);
    for (auto& t : workers) t.join();
    if (e != hipSuccess) return fail(RP_ERR_HIP, "result download: %s", hipGetErrorString(e));
    return RP_OK;
}
}  // namespace

int rp_result_fetch(rp_result* r, void* indptr, int32_t indptr_type, void* indices,
                    int32_t indices_type, void* data) {
    if (!r || !indptr) return fail(RP_ERR_INVALID, "NULL argument");
    if ((indptr_type != RP_I32 && indptr_type != RP_I64) || (indices_type != RP_I32 && indices_type != RP_I64))
        return fail(RP_ERR_INVALID, "bad index type");
    if (r->nnz > 0 && (!indices || !data)) return fail(RP_ERR_INVALID, "NULL output arrays");
    HIP_TRY(hipSetDevice(r->h->device));
    const int64_t n = r->n_rows;
    // type conversions run on the device (into a scratch buffer), then one copy each
    DevBuf conv;
    const size_t pbytes = indptr_type == RP_I32 ? (4 * (size_t)(n + 1) + 255) & ~size_t(255) : 0;
    const size_t cbytes = pbytes + (indices_type == RP_I64 ? 8 * (size_t)r->nnz : 0);
    if (cbytes) {
        int rc = conv.ensure(cbytes, r->h->device);
        if (rc) return rc;
    }
    auto grid_for = [](int64_t k) { return dim3((unsigned)std::min<int64_t>(std::max<int64_t>((k + 255) / 256, 1), 65536)); };
    std::vector<D2HJob> jobs;
    if (indptr_type == RP_I64) {
        jobs.push_back({indptr, r->cp.p, 8 * (size_t)(n + 1)});
    } else {
        hipLaunchKernelGGL((convert_kernel<int64_t, int32_t>), grid_for(n + 1), dim3(256), 0, nullptr,
                           (const int64_t*)r->cp.p, (int32_t*)conv.p, n + 1);
        HIP_TRY(hipGetLastError());
        jobs.push_back({indptr, conv.p, 4 * (size_t)(n + 1)});
    }
    if (r->nnz > 0) {
        if (indices_type == RP_I32) {
            jobs.push_back({indices, r->cj.p, 4 * (size_t)r->nnz});
        } else {
            int64_t* cj64 = reinterpret_cast<int64_t*>((char*)conv.p + pbytes);  // after the indptr
            hipLaunchKernelGGL((convert_kernel<int32_t, int64_t>), grid_for(r->nnz), dim3(256), 0, nullptr,
                               (const int32_t*)r->cj.p, cj64, r->nnz);
            HIP_TRY(hipGetLastError());
            jobs.push_back({indices, cj64, 8 * (size_t)r->nnz});
        }
        jobs.push_back({data, r->cx.p, (size_t)dtype_size(r->value_type) * (size_t)r->nnz});
    }
    return fetch_d2h(r->h, jobs);
}

int rp_result_free(rp_result* r) {
    delete r;
    return RP_OK;
}

int rp_project(rp_projector* h, const rp_csr_in* a, int32_t order, rp_alloc_fn alloc, void* user) {
    if (!alloc) return fail(RP_ERR_INVALID, "NULL allocation callback");
    rp_result* r = nullptr;
    int64_t nnz = 0;
    int rc = rp_project_host_begin(h, a, order, &r, &nnz);
    if (rc) return rc;
    void *ip = nullptr, *ix = nullptr, *dx = nullptr;
    int32_t ipt = RP_I64, ixt = RP_I32;
    if (alloc(user, r->n_rows, nnz, &ip, &ipt, &ix, &ixt, &dx) != 0) {
        rp_result_free(r);
        return fail(RP_ERR_NOMEM, "the allocation callback failed");
    }
    rc = rp_result_fetch(r, ip, ipt, ix, ixt, dx);
    rp_result_free(r);
    return rc;
}

}  // extern "C"

// ==========================================================================================
// Chunked host streaming (boundary 2 of SURVEY.md §8(d)): host CSR in -> host CSR out.
// The recipe projects host-resident partitions (code/clustermode/randomProjection.py:28-54,
// 107-113); here a host matrix of any size is cut into chunks of rows and three agents overlap:
//   uploader thread   chunk k+1: indptr/indices/data host -> device slot (hipMemcpyAsync + sync)
//   calling thread    chunk k:   rebase + input checks, the projection, per-chunk output offsets
//                                (a device running total, so no host round trip), conversions
//   downloader thread chunk k-1: indptr (global offsets) and entries device slot -> caller arrays
// Measured on the box (scripts/probes/pcie_probe2.hip): H2D 55 GB/s and D2H 48-55 GB/s at the
// same time; a pageable async copy blocks its calling thread for the whole transfer (so each
// direction gets a thread of its own), pinned ones return at once — both work here, pinned caller
// buffers (rp_host_alloc) only free the threads earlier. kStreamSlots device slots rotate.
namespace {
constexpr int kStreamSlots = 3;

template <typename IP>
__global__ void stream_rebase_kernel(const IP* __restrict__ raw, int64_t* __restrict__ out, int64_t n1,
                                     int64_t base0, unsigned long long* __restrict__ bad_row) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n1; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = (int64_t)raw[i];
        out[i] = v - base0;
        if (i > 0 && v < (int64_t)raw[i - 1]) atomicMin(bad_row, (unsigned long long)(i - 1));
    }
}

// info[0] = this chunk's first output position (running total before it), info[1] = its nnz,
// info[4] = the chunk's device error word (a look-back wait that expired: its total is not valid)
__global__ void stream_finish_kernel(const Workspace* __restrict__ ws, unsigned long long* __restrict__ total,
                                     unsigned long long* __restrict__ info) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const unsigned long long b = *total, k = ws->total;
        info[0] = b;
        info[1] = k;
        info[4] = ws->error;
        *total = b + k;
    }
}

template <typename OP>
__global__ void stream_indptr_kernel(const int64_t* __restrict__ cp, OP* __restrict__ out, int64_t n,
                                     const unsigned long long* __restrict__ info) {
    const int64_t b = (int64_t)info[0];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (OP)(cp[i] + b);
}

struct StreamSlot {
    DevBuf raw, ap, aj, ax;   // input chunk: indptr as given, rebased int64 indptr, indices, values
    DevBuf cp, cj, cx;        // output chunk: int64 chunk-relative indptr, int32 indices, values
    DevBuf optr, oidx;        // download forms: global indptr in the caller's type, int64 indices
    DevBuf ws, info;          // workspace; info = {base, nnz, first bad column pos, first bad row, error}
    size_t ws_need = 0;       // workspace bytes this chunk's plan needs (<= ws.bytes)
    int64_t cap = 0;
    hipEvent_t comp = nullptr;
};

struct StreamChunk {
    int64_t r0, rows, e0, nnz;
};

// Device output capacity of a stream slot for a chunk of `nnz` entries. The first chunks have only
// R's mean row length to go by (ppe = R.nnz / m: the expected products per entry for uniform
// columns), so they get 25% headroom on it; once chunks have come back, the largest measured output
// per entry (`seen`, the exact nnz of downloaded chunks / their entries) + 10% governs. Power-law
// columns shift the mean R row length under an entry (Zipf(1.1) on KDD2012's R: 0.576 kept outputs
// per entry vs 0.554 uniform), which a slot sized at 1.02x the uniform expectation did not hold:
// every chunk was recomputed alone after the pipeline (76 M rows/s instead of ~540 M).
int64_t stream_slot_cap(double ppe, double seen, int64_t nnz) {
    const double ex = std::max(1.25 * ppe, 1.10 * seen) * (double)nnz;
    return (int64_t)(ex + 8.0 * std::sqrt(ex + 1.0)) + 4096;
}

struct StreamSync {
    std::mutex mu;
    std::condition_variable cv;
    int64_t uploaded = 0, launched = 0, downloaded = 0;
    int err = RP_OK;
    std::string msg;
    void set_error(int code) {  // first error wins; the message is this thread's rp_last_error
        std::lock_guard<std::mutex> l(mu);
        if (err == RP_OK) {
            err = code;
            msg = g_err;
        }
        cv.notify_all();
    }
    template <typename P>
    bool wait(P pred) {  // false if an error stopped the pipeline
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return err != RP_OK || pred(); });
        return err == RP_OK;
    }
    void bump(int64_t& ctr) {
        std::lock_guard<std::mutex> l(mu);
        ++ctr;
        cv.notify_all();
    }
};

size_t grid_for(int64_t n) { return (size_t)std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 16384); }

int stream_upload(const rp_csr_in* a, const StreamChunk& ck, StreamSlot& s, hipStream_t st, int ips, int vs) {
    HIP_TRY(hipMemcpyAsync(s.raw.p, (const char*)a->indptr + (size_t)ips * ck.r0, (size_t)ips * (ck.rows + 1),
                           hipMemcpyHostToDevice, st));
    if (ck.nnz > 0) {
        HIP_TRY(hipMemcpyAsync(s.aj.p, a->indices + ck.e0, 4 * (size_t)ck.nnz, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(s.ax.p, (const char*)a->data + (size_t)vs * ck.e0, (size_t)vs * ck.nnz,
                               hipMemcpyHostToDevice, st));
    }
    HIP_TRY(poll_stream(st));
    return RP_OK;
}

int stream_project(rp_projector* h, const StreamChunk& ck, StreamSlot& s, int order, int vt, int out_ip, int out_ix,
                   unsigned long long* total, bool last, hipStream_t st, int* choice);

// the chunk's kernels on the compute stream; output capacity s.cap (the exact nnz lands in info[1])
int stream_compute(rp_projector* h, const rp_csr_in* a, const StreamChunk& ck, StreamSlot& s, int order,
                   int ip_type, int vt,
                   int out_ip, int out_ix, unsigned long long* total, bool last, hipStream_t st, int* choice) {
    unsigned long long* info = (unsigned long long*)s.info.p;
    const unsigned long long init[5] = {0, 0, ~0ull, ~0ull, 0};
    HIP_TRY(hipMemcpyAsync(info, init, sizeof init, hipMemcpyHostToDevice, st));
    const int64_t e_base = ck.e0;
    if (ip_type == RP_I64)
        hipLaunchKernelGGL((stream_rebase_kernel<int64_t>), dim3(grid_for(ck.rows + 1)), dim3(256), 0, st,
                           (const int64_t*)s.raw.p, (int64_t*)s.ap.p, ck.rows + 1, e_base, info + 3);
    else
        hipLaunchKernelGGL((stream_rebase_kernel<int32_t>), dim3(grid_for(ck.rows + 1)), dim3(256), 0, st,
                           (const int32_t*)s.raw.p, (int64_t*)s.ap.p, ck.rows + 1, e_base, info + 3);
    HIP_TRY(hipGetLastError());
    if (ck.nnz > 0) {
        hipLaunchKernelGGL(check_columns_kernel, dim3(grid_for(ck.nnz)), dim3(256), 0, st, (const int32_t*)s.aj.p,
                           ck.nnz, h->m, info + 2);
        HIP_TRY(hipGetLastError());
    }
    // a decreasing indptr or a column outside [0, m) would send the kernels out of bounds: check
    // before projecting (a short wait on this stream only; the copy threads keep going)
    unsigned long long chk[4];
    HIP_TRY(hipMemcpyAsync(chk, info, sizeof chk, hipMemcpyDeviceToHost, st));
    HIP_TRY(poll_stream(st));
    if (chk[3] != ~0ull)
        return fail(RP_ERR_INVALID, "A indptr decreasing at row %lld", (long long)(ck.r0 + (int64_t)chk[3]));
    if (chk[2] != ~0ull)
        return fail(RP_ERR_INVALID, "A column index %d out of range [0, %lld)", a->indices[ck.e0 + (int64_t)chk[2]],
                    (long long)h->m);
    return stream_project(h, ck, s, order, vt, out_ip, out_ix, total, last, st, choice);
}

// the projection part of a chunk: its CSR is in s.ap (int64, from 0) / s.aj / s.ax on the device;
// output offsets chained on the device through `total`; *choice: the staging verdict sampled on the
// first chunk (-1 before it), reused by the others
int stream_project(rp_projector* h, const StreamChunk& ck, StreamSlot& s, int order, int vt, int out_ip, int out_ix,
                   unsigned long long* total, bool last, hipStream_t st, int* choice) {
    unsigned long long* info = (unsigned long long*)s.info.p;
    rp_csr_in ad{ck.rows, s.ap.p, RP_I64, (const int32_t*)s.aj.p, s.ax.p, vt, ck.nnz};
    rp_csr_out cd{s.cp.p, RP_I64, s.cj.p, RP_I32, s.cx.p, s.cap};
    int rc = project_device_impl(h, &ad, &cd, order, s.ws.p, (int64_t)s.ws_need, st, nullptr, ck.nnz, choice);
    if (rc) return rc;
    hipLaunchKernelGGL(stream_finish_kernel, dim3(1), dim3(64), 0, st, (const Workspace*)s.ws.p, total, info);
    const int64_t np = ck.rows + (last ? 1 : 0);  // the next chunk writes the shared boundary entry
    if (out_ip == RP_I64)
        hipLaunchKernelGGL((stream_indptr_kernel<int64_t>), dim3(grid_for(np)), dim3(256), 0, st,
                           (const int64_t*)s.cp.p, (int64_t*)s.optr.p, np, (const unsigned long long*)info);
    else
        hipLaunchKernelGGL((stream_indptr_kernel<int32_t>), dim3(grid_for(np)), dim3(256), 0, st,
                           (const int64_t*)s.cp.p, (int32_t*)s.optr.p, np, (const unsigned long long*)info);
    HIP_TRY(hipGetLastError());
    if (out_ix == RP_I64 && s.cap > 0) {
        hipLaunchKernelGGL((convert_kernel<int32_t, int64_t>), dim3(grid_for(s.cap)), dim3(256), 0, st,
                           (const int32_t*)s.cj.p, (int64_t*)s.oidx.p, s.cap);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(s.comp, st));
    return RP_OK;
}

// download chunk results into the caller's arrays; *redo = entries did not fit the device slot
int stream_download(const StreamChunk& ck, StreamSlot& s, const rp_csr_in* a, const rp_csr_out* c, bool last,
                    hipStream_t st, int vs, int64_t* nnz_out, bool* redo) {
    HIP_TRY(poll_event(s.comp));
    unsigned long long info[5];
    HIP_TRY(hipMemcpyAsync(info, s.info.p, sizeof info, hipMemcpyDeviceToHost, st));
    HIP_TRY(poll_stream(st));
    if (info[4]) return fail(RP_ERR_TIMEOUT, "device look-back wait expired (rows %lld..)", (long long)ck.r0);
    const int64_t base = (int64_t)info[0], k = (int64_t)info[1];
    *nnz_out = k;
    const int ops = dtype_size(c->indptr_type), oxs = dtype_size(c->indices_type);
    const int64_t np = ck.rows + (last ? 1 : 0);
    HIP_TRY(hipMemcpyAsync((char*)c->indptr + (size_t)ops * ck.r0, s.optr.p, (size_t)ops * np, hipMemcpyDeviceToHost, st));
    *redo = k > s.cap;
    const int64_t fit = std::max<int64_t>(0, std::min<int64_t>(k, c->capacity - base));
    if (!*redo && fit > 0) {
        const void* src_ix = c->indices_type == RP_I64 ? s.oidx.p : s.cj.p;
        HIP_TRY(hipMemcpyAsync((char*)c->indices + (size_t)oxs * base, src_ix, (size_t)oxs * fit,
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync((char*)c->data + (size_t)vs * base, s.cx.p, (size_t)vs * fit, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(poll_stream(st));
    return RP_OK;
}

int stream_alloc_slot(rp_projector* h, StreamSlot& s, int64_t rows, int64_t nnz, int64_t cap, int ips, int vs,
                      int out_ip, int out_ix) {
    const int dev = h->device;
    int rc;
    if ((rc = s.raw.grow((size_t)ips * (rows + 1), dev)) || (rc = s.ap.grow(8 * (size_t)(rows + 1), dev)) ||
        (rc = s.aj.grow(4 * (size_t)std::max<int64_t>(nnz, 1), dev)) ||
        (rc = s.ax.grow((size_t)vs * std::max<int64_t>(nnz, 1), dev)) ||
        (rc = s.cp.grow(8 * (size_t)(rows + 1), dev)) ||
        (rc = s.cj.grow(4 * (size_t)std::max<int64_t>(cap, 1), dev)) ||
        (rc = s.cx.grow((size_t)vs * std::max<int64_t>(cap, 1), dev)) ||
        (rc = s.optr.grow((size_t)dtype_size(out_ip) * (rows + 1), dev)) ||
        (rc = s.info.grow(64, dev)))
        return rc;
    if (out_ix == RP_I64 && (rc = s.oidx.grow(8 * (size_t)std::max<int64_t>(cap, 1), dev))) return rc;
    const int64_t wsb = rp_project_workspace_bytes(h, rows, nnz);
    if (wsb < 0) return fail(RP_ERR_INVALID, "workspace size");
    if ((rc = s.ws.grow((size_t)wsb, dev))) return rc;
    s.ws_need = (size_t)wsb;
    s.cap = cap;
    return RP_OK;
}
}  // namespace

extern "C" {

int rp_project_stream(rp_projector* h, const rp_csr_in* a, int32_t order, int64_t chunk_rows,
                      const rp_csr_out* c, int64_t* total_nnz) {
    if (!h || !a || !c) return fail(RP_ERR_INVALID, "NULL argument");
    if (order != RP_ORDER_SCIPY && order != RP_ORDER_SORTED) return fail(RP_ERR_INVALID, "bad order");
    const int ips = dtype_size(a->indptr_type), vs = dtype_size(a->data_type);
    if (!ips || (a->data_type != RP_F32 && a->data_type != RP_F64)) return fail(RP_ERR_INVALID, "bad A types");
    if (a->data_type == RP_F32 && h->value_type == RP_F64)
        return fail(RP_ERR_INVALID, "compute type must be upcast(A, R) = float64 for a float64 R");
    if ((c->indptr_type != RP_I32 && c->indptr_type != RP_I64) || (c->indices_type != RP_I32 && c->indices_type != RP_I64))
        return fail(RP_ERR_INVALID, "bad output index types");
    if (a->n_rows < 0 || !a->indptr || !c->indptr) return fail(RP_ERR_INVALID, "bad CSR arrays");
    if (c->capacity < 0) return fail(RP_ERR_INVALID, "negative output capacity");
    if (c->capacity > 0 && (!c->indices || !c->data)) return fail(RP_ERR_INVALID, "NULL output arrays");
    const int64_t n = a->n_rows;
    int choice = -1;  // staged or direct gathers: sampled on the first chunk, kept for the call
    if (chunk_rows <= 0) chunk_rows = kStreamChunkRows;
    // chunk plan from indptr at chunk boundaries (the rows inside a chunk are checked on the device)
    std::vector<StreamChunk> chunks;
    const int64_t b0 = ptr_at(a->indptr, a->indptr_type, 0);
    int64_t prev = b0, max_rows = 0, max_nnz = 0;
    if (b0 < 0) return fail(RP_ERR_INVALID, "A indptr[0] < 0");
    for (int64_t r = 0; r < n; r += chunk_rows) {
        const int64_t rows = std::min(chunk_rows, n - r);
        const int64_t e1 = ptr_at(a->indptr, a->indptr_type, r + rows);
        if (e1 < prev) return fail(RP_ERR_INVALID, "A indptr decreasing before row %lld", (long long)(r + rows));
        chunks.push_back({r, rows, prev, e1 - prev});
        max_rows = std::max(max_rows, rows);
        max_nnz = std::max(max_nnz, e1 - prev);
        prev = e1;
    }
    if (a->nnz >= 0 && a->nnz < prev - b0) return fail(RP_ERR_INVALID, "A nnz %lld < indptr range %lld",
                                                      (long long)a->nnz, (long long)(prev - b0));
    std::lock_guard<std::mutex> lock(h->mu);
    HIP_TRY(hipSetDevice(h->device));
    if (chunks.empty()) {
        if (c->indptr_type == RP_I64) ((int64_t*)c->indptr)[0] = 0; else ((int32_t*)c->indptr)[0] = 0;
        if (total_nnz) *total_nnz = 0;
        return RP_OK;
    }
    // device output capacity per slot (stream_slot_cap): from R's mean row length for the first
    // chunks, then from the measured output per entry of the chunks already downloaded (a slot
    // grows before it takes a chunk that would not fit); a chunk beyond its slot anyway is
    // recomputed alone once the pipeline has drained (counted: rp_project_stream_stats)
    const double ppe = h->m > 0 ? (double)h->nnz / (double)h->m : 0.0;
    const int64_t cap = stream_slot_cap(ppe, 0.0, max_nnz);
    h->st_chunks = (int64_t)chunks.size();
    h->st_redo = h->st_regrow = 0;
    StreamSlot slots[kStreamSlots];
    const int ns = (int)std::min<size_t>(kStreamSlots, chunks.size());
    int rc;
    for (int i = 0; i < ns; ++i) {
        if ((rc = stream_alloc_slot(h, slots[i], max_rows, max_nnz, cap, ips, vs, c->indptr_type, c->indices_type)))
            return rc;
        HIP_TRY(hipEventCreateWithFlags(&slots[i].comp, hipEventDisableTiming));
    }
    DevBuf totbuf;
    if ((rc = totbuf.ensure(8, h->device))) return rc;
    hipStream_t st_up = nullptr, st_comp = nullptr, st_down = nullptr;
    auto cleanup = [&] {
        for (auto& s : slots)
            if (s.comp) (void)hipEventDestroy(s.comp);
        for (hipStream_t s : {st_up, st_comp, st_down})
            if (s) (void)hipStreamDestroy(s);
    };
    if (hipStreamCreateWithFlags(&st_up, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&st_comp, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&st_down, hipStreamNonBlocking) != hipSuccess) {
        cleanup();
        return fail(RP_ERR_HIP, "stream creation failed");
    }
    if (hipMemsetAsync(totbuf.p, 0, 8, st_comp) != hipSuccess) {
        cleanup();
        return fail(RP_ERR_HIP, "memset failed");
    }
    const int64_t K = (int64_t)chunks.size();
    StreamSync sy;
    std::vector<int64_t> knnz((size_t)K, 0);
    std::vector<char> redo((size_t)K, 0);
    const int dev = h->device;
    std::thread up([&] {
        if (hipSetDevice(dev) != hipSuccess) return sy.set_error(fail(RP_ERR_HIP, "hipSetDevice"));
        for (int64_t k = 0; k < K; ++k) {
            StreamSlot& s = slots[k % ns];
            // the slot's input is free once chunk k - ns's kernels have run
            if (!sy.wait([&] { return sy.launched >= k - ns + 1 || k < ns; })) return;
            if (k >= ns && poll_event(s.comp) != hipSuccess)
                return sy.set_error(fail(RP_ERR_HIP, "event sync (upload)"));
            if (int r = stream_upload(a, chunks[(size_t)k], s, st_up, ips, vs)) return sy.set_error(r);
            sy.bump(sy.uploaded);
        }
    });
    std::thread down([&] {
        if (hipSetDevice(dev) != hipSuccess) return sy.set_error(fail(RP_ERR_HIP, "hipSetDevice"));
        for (int64_t k = 0; k < K; ++k) {
            if (!sy.wait([&] { return sy.launched > k; })) return;
            bool rd = false;
            if (int r = stream_download(chunks[(size_t)k], slots[k % ns], a, c, k == K - 1, st_down, vs,
                                        &knnz[(size_t)k], &rd))
                return sy.set_error(r);
            redo[(size_t)k] = rd;
            sy.bump(sy.downloaded);
        }
    });
    double seen = 0.0;  // largest output per entry of the chunks downloaded so far
    int64_t folded = 0;
    for (int64_t k = 0; k < K && sy.err == RP_OK; ++k) {
        if (!sy.wait([&] { return sy.uploaded > k && sy.downloaded >= k - ns + 1; })) break;
        for (; folded <= k - ns; ++folded)  // downloaded (the wait above): knnz is final
            if (chunks[(size_t)folded].nnz > 0)
                seen = std::max(seen, (double)knnz[(size_t)folded] / (double)chunks[(size_t)folded].nnz);
        StreamSlot& sk = slots[k % ns];
        const int64_t want = stream_slot_cap(ppe, seen, chunks[(size_t)k].nnz);
        if (want > sk.cap) {  // the slot's previous chunk has been downloaded: its output may move
            if ((rc = stream_alloc_slot(h, sk, max_rows, max_nnz, want, ips, vs, c->indptr_type, c->indices_type))) {
                sy.set_error(rc);
                break;
            }
            ++h->st_regrow;
        }
        if ((rc = stream_compute(h, a, chunks[(size_t)k], slots[k % ns], order, a->indptr_type, a->data_type,
                                 c->indptr_type, c->indices_type, (unsigned long long*)totbuf.p, k == K - 1,
                                 st_comp, &choice))) {
            sy.set_error(rc);
            break;
        }
        sy.bump(sy.launched);
    }
    up.join();
    down.join();
    if (sy.err != RP_OK) {
        (void)hipStreamSynchronize(st_comp);
        cleanup();
        g_err = sy.msg;
        return sy.err;
    }
    // chunks whose entries exceeded the slot: recompute alone with their exact size
    int64_t base = 0, total = 0;
    for (int64_t k = 0; k < K; ++k) total += knnz[(size_t)k];
    for (int64_t k = 0; k < K && rc == RP_OK; base += knnz[(size_t)k], ++k) {
        if (!redo[(size_t)k]) continue;
        ++h->st_redo;
        StreamSlot& s = slots[0];
        const StreamChunk& ck = chunks[(size_t)k];
        if ((rc = stream_alloc_slot(h, s, max_rows, max_nnz, knnz[(size_t)k], ips, vs, c->indptr_type,
                                    c->indices_type)) ||
            (rc = stream_upload(a, ck, s, st_up, ips, vs)))
            break;
        unsigned long long tot0 = (unsigned long long)base;  // the chunk's base again
        if (hipMemcpyAsync(totbuf.p, &tot0, 8, hipMemcpyHostToDevice, st_comp) != hipSuccess) {
            rc = fail(RP_ERR_HIP, "memcpy");
            break;
        }
        if ((rc = stream_compute(h, a, ck, s, order, a->indptr_type, a->data_type, c->indptr_type, c->indices_type,
                                 (unsigned long long*)totbuf.p, k == K - 1, st_comp, &choice)))
            break;
        int64_t kk = 0;
        bool rd = false;
        rc = stream_download(ck, s, a, c, k == K - 1, st_down, vs, &kk, &rd);
        if (rc == RP_OK && (rd || kk != knnz[(size_t)k])) rc = fail(RP_ERR_HIP, "chunk recompute mismatch");
    }
    (void)hipStreamSynchronize(st_comp);
    cleanup();
    if (rc) return rc;
    if (total_nnz) *total_nnz = total;
    if (total > c->capacity)
        return fail(RP_ERR_CAPACITY, "output capacity %lld < nnz %lld", (long long)c->capacity, (long long)total);
    if (c->indptr_type == RP_I32 && total > INT32_MAX)
        return fail(RP_ERR_CAPACITY, "nnz %lld needs an int64 output indptr", (long long)total);
    return RP_OK;
}

// Boundary 3 (libsvm text -> projected CSR), chunked like rp_project_stream: chunk k+1's text
// uploads while chunk k is parsed and projected and chunk k-1's result downloads. A chunk is a run of
// whole lines (a Spark text partition); its rows land at the running row total, its entries at the
// running output total (chained on the device). Parse scratch and slot buffers grow only, so the
// steady state allocates nothing.
namespace {
struct TextSlot {
    DevBuf text, labels;
    LibsvmScratch ps;
    StreamSlot s;
};
struct TextChunk {
    int64_t b0, bytes;
};

int64_t lines_before(const char* text, int64_t b) {  // error reporting only
    int64_t n = 0;
    for (const char* p = text; (p = (const char*)memchr(p, '\n', (size_t)(text + b - p))) != nullptr; ++p) ++n;
    return n;
}
}  // namespace

int rp_libsvm_project_stream(rp_projector* h, const char* text, int64_t n_bytes, int32_t order, int64_t chunk_bytes,
                             double* labels, int64_t cap_rows, const rp_csr_out* c, int64_t* n_rows,
                             int64_t* total_nnz, int64_t* err_line) {
    if (err_line) *err_line = -1;
    if (!h || !c || !n_rows || n_bytes < 0 || (n_bytes > 0 && !text)) return fail(RP_ERR_INVALID, "bad argument");
    if (order != RP_ORDER_SCIPY && order != RP_ORDER_SORTED) return fail(RP_ERR_INVALID, "bad order");
    if (h->value_type != RP_F32)
        return fail(RP_ERR_UNSUPPORTED, "libsvm values are float32 (the recipe's astype): R must be float32");
    if ((c->indptr_type != RP_I32 && c->indptr_type != RP_I64) || (c->indices_type != RP_I32 && c->indices_type != RP_I64))
        return fail(RP_ERR_INVALID, "bad output index types");
    if (c->capacity < 0 || cap_rows < 0) return fail(RP_ERR_INVALID, "negative output capacity");
    if (!c->indptr || (c->capacity > 0 && (!c->indices || !c->data)) || (cap_rows > 0 && !labels))
        return fail(RP_ERR_INVALID, "NULL output arrays");
    if (chunk_bytes <= 0) chunk_bytes = 64ll << 20;
    int choice = -1;  // staged or direct gathers: sampled on the first chunk, kept for the call
    std::vector<TextChunk> chunks;
    for (int64_t b = 0; b < n_bytes;) {
        int64_t e = std::min(n_bytes, b + chunk_bytes);
        if (e < n_bytes) {  // end after the last newline inside, or after the line that spans the cut
            const char* nl = (const char*)memrchr(text + b, '\n', (size_t)(e - b));
            if (nl) {
                e = nl - text + 1;
            } else {
                const char* nx = (const char*)memchr(text + e, '\n', (size_t)(n_bytes - e));
                e = nx ? nx - text + 1 : n_bytes;
            }
        }
        chunks.push_back({b, e - b});
        b = e;
    }
    std::lock_guard<std::mutex> lock(h->mu);
    HIP_TRY(hipSetDevice(h->device));
    *n_rows = 0;
    if (total_nnz) *total_nnz = 0;
    if (chunks.empty()) {
        if (c->indptr_type == RP_I64) ((int64_t*)c->indptr)[0] = 0; else ((int32_t*)c->indptr)[0] = 0;
        return RP_OK;
    }
    const int ns = (int)std::min<size_t>(kStreamSlots, chunks.size());
    TextSlot slots[kStreamSlots];
    std::vector<StreamChunk> cks(chunks.size());
    int rc;
    for (int i = 0; i < ns; ++i) HIP_TRY(hipEventCreateWithFlags(&slots[i].s.comp, hipEventDisableTiming));
    DevBuf totbuf;
    hipStream_t st_up = nullptr, st_comp = nullptr, st_down = nullptr;
    auto cleanup = [&] {
        for (auto& t : slots)
            if (t.s.comp) (void)hipEventDestroy(t.s.comp);
        for (hipStream_t q : {st_up, st_comp, st_down})
            if (q) (void)hipStreamDestroy(q);
    };
    if ((rc = totbuf.ensure(8, h->device))) {
        cleanup();
        return rc;
    }
    if (hipStreamCreateWithFlags(&st_up, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&st_comp, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&st_down, hipStreamNonBlocking) != hipSuccess ||
        hipMemsetAsync(totbuf.p, 0, 8, st_comp) != hipSuccess) {
        cleanup();
        return fail(RP_ERR_HIP, "stream setup failed");
    }
    const double ppe = h->m > 0 ? (double)h->nnz / (double)h->m : 0.0;
    double seen = 0.0;  // largest output per entry of the chunks downloaded so far (stream_slot_cap)
    auto out_cap = [&](int64_t nnz) { return stream_slot_cap(ppe, seen, nnz); };
    h->st_chunks = (int64_t)chunks.size();
    h->st_redo = h->st_regrow = 0;
    const int dev = h->device;
    const int64_t K = (int64_t)chunks.size();
    StreamSync sy;
    std::vector<int64_t> knnz((size_t)K, 0);
    std::vector<char> redo((size_t)K, 0);
    int64_t bad_line = -1;
    auto upload = [&](int64_t k, TextSlot& t) -> int {
        const TextChunk& tc = chunks[(size_t)k];
        if (int r = t.text.grow((size_t)tc.bytes + 16, dev)) return r;
        HIP_TRY(hipMemcpyAsync(t.text.p, text + tc.b0, (size_t)tc.bytes, hipMemcpyHostToDevice, st_up));
        HIP_TRY(poll_stream(st_up));
        return RP_OK;
    };
    // parse chunk k in slot t (on st_comp) into t.s.ap/aj/ax and t.labels; fills cks[k] but r0
    auto parse = [&](int64_t k, TextSlot& t, int64_t cap_out) -> int {
        const TextChunk& tc = chunks[(size_t)k];
        int64_t rows = 0, nnz = 0, el = -1;
        int r = libsvm_parse(t.ps, dev, (const char*)t.text.p, tc.bytes, h->m, nullptr, nullptr, RP_I64, nullptr,
                             nullptr, 0, 0, st_comp, &rows, &nnz, &el);
        if (r) return r;
        const int64_t cap = cap_out >= 0 ? cap_out : out_cap(nnz);
        if (cap_out < 0 && 1.10 * seen > 1.25 * ppe) ++h->st_regrow;  // sized from measured output
        if ((r = t.labels.grow(8 * (size_t)std::max<int64_t>(rows, 1), dev)) ||
            (r = stream_alloc_slot(h, t.s, rows, nnz, cap, 8, 4, c->indptr_type, c->indices_type)))
            return r;
        r = libsvm_parse(t.ps, dev, (const char*)t.text.p, tc.bytes, h->m, (double*)t.labels.p, t.s.ap.p, RP_I64,
                         (int32_t*)t.s.aj.p, (float*)t.s.ax.p, rows, nnz, st_comp, &rows, &nnz, &el,
                         /*reuse_counts=*/true);  // the count call just above: its line tables stand
        if (r == RP_ERR_INVALID && el >= 0) bad_line = lines_before(text, tc.b0) + el;
        if (r) return r;
        cks[(size_t)k].rows = rows;
        cks[(size_t)k].nnz = nnz;
        cks[(size_t)k].e0 = 0;
        return RP_OK;
    };
    auto download = [&](int64_t k, TextSlot& t, int64_t* kn, bool* rd) -> int {
        const StreamChunk& ck = cks[(size_t)k];
        HIP_TRY(poll_event(t.s.comp));
        if (ck.rows > 0)
            HIP_TRY(hipMemcpyAsync(labels + ck.r0, t.labels.p, 8 * (size_t)ck.rows, hipMemcpyDeviceToHost, st_down));
        return stream_download(ck, t.s, nullptr, c, k == K - 1, st_down, 4, kn, rd);
    };
    std::thread up([&] {
        if (hipSetDevice(dev) != hipSuccess) return sy.set_error(fail(RP_ERR_HIP, "hipSetDevice"));
        for (int64_t k = 0; k < K; ++k) {
            TextSlot& t = slots[k % ns];
            if (!sy.wait([&] { return sy.launched >= k - ns + 1 || k < ns; })) return;
            if (k >= ns && poll_event(t.s.comp) != hipSuccess)
                return sy.set_error(fail(RP_ERR_HIP, "event sync (upload)"));
            if (int r = upload(k, t)) return sy.set_error(r);
            sy.bump(sy.uploaded);
        }
    });
    std::thread down([&] {
        if (hipSetDevice(dev) != hipSuccess) return sy.set_error(fail(RP_ERR_HIP, "hipSetDevice"));
        for (int64_t k = 0; k < K; ++k) {
            if (!sy.wait([&] { return sy.launched > k; })) return;
            bool rd = false;
            if (int r = download(k, slots[k % ns], &knnz[(size_t)k], &rd)) return sy.set_error(r);
            redo[(size_t)k] = rd;
            sy.bump(sy.downloaded);
        }
    });
    int64_t rows_total = 0, folded = 0;
    for (int64_t k = 0; k < K && sy.err == RP_OK; ++k) {
        if (!sy.wait([&] { return sy.uploaded > k && sy.downloaded >= k - ns + 1; })) break;
        for (; folded <= k - ns; ++folded)  // downloaded (the wait above): knnz is final
            if (cks[(size_t)folded].nnz > 0)
                seen = std::max(seen, (double)knnz[(size_t)folded] / (double)cks[(size_t)folded].nnz);
        TextSlot& t = slots[k % ns];
        if ((rc = parse(k, t, -1))) {
            sy.set_error(rc);
            break;
        }
        cks[(size_t)k].r0 = rows_total;
        rows_total += cks[(size_t)k].rows;
        if (rows_total > cap_rows) {
            sy.set_error(fail(RP_ERR_CAPACITY, "more than %lld rows (cap_rows)", (long long)cap_rows));
            break;
        }
        if ((rc = stream_project(h, cks[(size_t)k], t.s, order, RP_F32, c->indptr_type, c->indices_type,
                                 (unsigned long long*)totbuf.p, k == K - 1, st_comp, &choice))) {
            sy.set_error(rc);
            break;
        }
        sy.bump(sy.launched);
    }
    up.join();
    down.join();
    if (sy.err != RP_OK) {
        (void)hipStreamSynchronize(st_comp);
        cleanup();
        g_err = sy.msg;
        if (err_line) *err_line = bad_line;
        if (sy.err == RP_ERR_CAPACITY) *n_rows = rows_total;
        return sy.err;
    }
    // chunks whose entries exceeded their slot: parsed and projected again alone, exact size
    int64_t base = 0, total = 0;
    for (int64_t k = 0; k < K; ++k) total += knnz[(size_t)k];
    rc = RP_OK;
    for (int64_t k = 0; k < K && rc == RP_OK; base += knnz[(size_t)k], ++k) {
        if (!redo[(size_t)k]) continue;
        ++h->st_redo;
        TextSlot& t = slots[0];
        const int64_t r0 = cks[(size_t)k].r0;
        if ((rc = upload(k, t)) || (rc = parse(k, t, knnz[(size_t)k]))) break;
        cks[(size_t)k].r0 = r0;
        unsigned long long tot0 = (unsigned long long)base;
        if (hipMemcpyAsync(totbuf.p, &tot0, 8, hipMemcpyHostToDevice, st_comp) != hipSuccess) {
            rc = fail(RP_ERR_HIP, "memcpy");
            break;
        }
        if ((rc = stream_project(h, cks[(size_t)k], t.s, order, RP_F32, c->indptr_type, c->indices_type,
                                 (unsigned long long*)totbuf.p, k == K - 1, st_comp, &choice)))
            break;
        int64_t kk = 0;
        bool rd = false;
        rc = download(k, t, &kk, &rd);
        if (rc == RP_OK && (rd || kk != knnz[(size_t)k])) rc = fail(RP_ERR_HIP, "chunk recompute mismatch");
    }
    (void)hipStreamSynchronize(st_comp);
    cleanup();
    if (rc) return rc;
    *n_rows = rows_total;
    if (total_nnz) *total_nnz = total;
    if (total > c->capacity)
        return fail(RP_ERR_CAPACITY, "output capacity %lld < nnz %lld", (long long)c->capacity, (long long)total);
    if (c->indptr_type == RP_I32 && total > INT32_MAX)
        return fail(RP_ERR_CAPACITY, "nnz %lld needs an int64 output indptr", (long long)total);
    return RP_OK;
}

int rp_project_stream_stats(rp_projector* h, int64_t* chunks, int64_t* recomputed, int64_t* regrown) {
    if (!h) return fail(RP_ERR_INVALID, "NULL projector");
    std::lock_guard<std::mutex> lock(h->mu);  // the stream calls hold it while they run
    if (chunks) *chunks = h->st_chunks;
    if (recomputed) *recomputed = h->st_redo;
    if (regrown) *regrown = h->st_regrow;
    return RP_OK;
}

// pinned (page-locked) host memory for callers that want the stream path's copies fully
// asynchronous (a data loader filling input chunks, result arrays reused across calls)
int rp_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes < 0) return fail(RP_ERR_INVALID, "bad argument");
    *out = nullptr;
    HIP_TRY(hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault));
    return RP_OK;
}

int rp_host_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return RP_OK;
}

int rp_synth_rows_device(int device, int64_t n_rows, int64_t m, double mean_extra,
                         int32_t max_row_nnz, int32_t dist, double zipf_s, uint64_t seed,
                         void* indptr, int32_t indptr_type, int32_t* indices, float* data,
                         void* stream, int64_t* nnz) {
    if (!indptr || n_rows < 0 || m <= 0 || !nnz) return fail(RP_ERR_INVALID, "bad argument");
    if (indptr_type != RP_I32 && indptr_type != RP_I64) return fail(RP_ERR_INVALID, "bad indptr type");
    if (max_row_nnz < 1 || max_row_nnz > kSynthMaxK) return fail(RP_ERR_INVALID, "max_row_nnz in [1, %d]", kSynthMaxK);
    if (dist != 0 && dist != 1) return fail(RP_ERR_INVALID, "dist must be 0 (uniform) or 1 (power-law)");
    if (dist == 1 && !(zipf_s > 1.0)) return fail(RP_ERR_INVALID, "zipf_s must be > 1");
    HIP_TRY(hipSetDevice(device));
    hipStream_t st = (hipStream_t)stream;
    DevBuf ptr64, tmp;
    int rc = ptr64.ensure(8 * (size_t)(n_rows + 1), device);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(ptr64.p, 0, 8, st));
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>((n_rows + 255) / 256, 1), 65536);
    hipLaunchKernelGGL((synth_count_kernel<int64_t>), dim3(grid), dim3(256), 0, st, n_rows, seed,
                       mean_extra, max_row_nnz, m, (int64_t*)ptr64.p);
    HIP_TRY(hipGetLastError());
    rc = inclusive_scan_i64((int64_t*)ptr64.p + 1, n_rows, st, tmp, device);
    if (rc) return rc;
    int64_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, (int64_t*)ptr64.p + n_rows, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(poll_stream(st));
    if (indptr_type == RP_I32 && total >= ((int64_t)1 << 31))
        return fail(RP_ERR_UNSUPPORTED, "nnz %lld needs int64 indptr", (long long)total);
    if (indptr_type == RP_I64) {
        HIP_TRY(hipMemcpyAsync(indptr, ptr64.p, 8 * (size_t)(n_rows + 1), hipMemcpyDeviceToDevice, st));
    } else {
        hipLaunchKernelGGL((convert_kernel<int64_t, int32_t>), dim3(grid), dim3(256), 0, st,
                           (const int64_t*)ptr64.p, (int32_t*)indptr, n_rows + 1);
        HIP_TRY(hipGetLastError());
    }
    if (indices) {
        if (!data) return fail(RP_ERR_INVALID, "NULL data");
        const uint64_t perm_b = (seed * 0x9E3779B97F4A7C15ull) % (uint64_t)m;
        uint64_t perm_a = 2654435761ull % (uint64_t)m;
        auto gcd = [](uint64_t x, uint64_t y) { while (y) { uint64_t t = x % y; x = y; y = t; } return x; };
        while (perm_a == 0 || gcd(perm_a, (uint64_t)m) != 1) perm_a = (perm_a + 1) % (uint64_t)m;
        hipLaunchKernelGGL(synth_fill_kernel, dim3(grid), dim3(256), 0, st, n_rows, m, seed, dist, zipf_s,
                           perm_a, perm_b, (const int64_t*)ptr64.p, indices, data);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(poll_stream(st));
    *nnz = total;
    return RP_OK;
}

}  // extern "C"
