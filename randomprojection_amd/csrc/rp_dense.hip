// rp_dense.hip — the dense Gaussian projection as a hand-written gfx950 MFMA GEMM
// (BASELINE.json configs[4]).
//
// Reference semantics: sklearn GaussianRandomProjection.transform(X) = X @ components_.T
// (sklearn/random_projection.py:569-612): Y[n x p] = X[n x m] . G[p x m]^T. Both operands are
// row-major with the contraction index m contiguous ("NT" GEMM), the layout the MFMA operand
// fragments want: a lane's A and B elements are consecutive in memory.
//
//   bf16: bf16 operands, f32 accumulate, f32 result (v_mfma_f32_16x16x32_bf16 / _32x32x16_bf16).
//   f32:  exact f32 products (gfx950 has no xf32), f32 accumulate (v_mfma_f32_16x16x4_f32 / _32x32x2_f32).
//
// Kernel families (rp_dense_project_device's `variant` picks one for measurements):
//  * dense_ring_kernel (variant 11, the default): 256 x 256 tile, 8 waves of 128 x 64, 16 x 16
//    MFMAs, operands staged global -> LDS by global_load_lds_dwordx4 (no VGPR round trip) into a
//    ring of four 64-B-per-row K-tile buffers, three K-tiles in flight while one is multiplied, one
//    barrier per K-tile (description above the kernel);
//  * dense_glds_kernel (variant 10): the same tile and staging with two 128-B-per-row buffers, the
//    next K-tile in flight during this one's MFMAs;
//  * f64: dense_ring_f64_kernel (the default): 256 x 128 tile, 8 waves of 64 x 64 in
//    v_mfma_f64_16x16x4_f64, three 48 KB K-tile buffers (two K-tiles in flight); variant 10 selects
//    the two-buffer dense_glds_f64_kernel (measured 58.7 vs 69.8 TF, profiles/r04_dense_fp64*);
//  * dense_nt_kernel (variants 0-9; variant 5 = 256 x 256, 8 waves, 32 x 32 MFMAs, two LDS stages, the
//    round-2 default): the next K step loaded global -> registers during the MFMAs, then written to
//    the other LDS buffer (one barrier per step); LDS rows of 128 B XOR-swizzled (chunk c of row r at
//    c ^ (r & 7)); f32 permutes the K order inside a step so every lane reads 64 contiguous bytes.
// Block -> tile map is XCD-aware in both: XCD x (workgroup i runs on XCD i % 8) takes the M tiles
// congruent to x mod 8 and walks each M tile's N tiles back to back, so an X tile is fetched from
// HBM once and re-read from that XCD's L2.
#include <atomic>
#include <type_traits>

#include "rp_common.h"

using namespace rpd;

namespace {

constexpr int kRowBytes = 128;  // one K step of a row (64 bf16 / 32 f32), 8 chunks of 16 B

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

template <typename T>
struct DenseStep;

// bf16: K step 64 elements = 4 MFMA k-substeps of 16; lane (r, h) reads chunk 2s + h of its row
template <>
struct DenseStep<uint16_t> {
    static constexpr int kElems = 64;
    template <int TM, int TN>
    __device__ static void compute(const uint4* __restrict__ sA, const uint4* __restrict__ sB, int ra0, int rb0,
                                   int lane, f32x16 (&acc)[TM][TN]) {
        const int r = lane & 31, h = lane >> 5;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            bf16x8 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = __builtin_bit_cast(bf16x8, sA[swz(ra0 + i * 32 + r, 2 * s + h)]);
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = __builtin_bit_cast(bf16x8, sB[swz(rb0 + j * 32 + r, 2 * s + h)]);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    }
};

// f32: K step 32 elements = 16 MFMAs of K = 2; MFMA t, lane half h uses k = 16h + t (a permutation
// of the step's K order, the same for A and B): lane (r, h) reads chunks 4h .. 4h + 3 of its row
template <>
struct DenseStep<float> {
    static constexpr int kElems = 32;
    template <int TM, int TN>
    __device__ static void compute(const uint4* __restrict__ sA, const uint4* __restrict__ sB, int ra0, int rb0,
                                   int lane, f32x16 (&acc)[TM][TN]) {
        const int r = lane & 31, h = lane >> 5;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = sA[swz(ra0 + i * 32 + r, 4 * h + q)];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = sB[swz(rb0 + j * 32 + r, 4 * h + q)];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const uint32_t ua = e == 0 ? a[i].x : e == 1 ? a[i].y : e == 2 ? a[i].z : a[i].w;
                        const uint32_t ub = e == 0 ? b[j].x : e == 1 ? b[j].y : e == 2 ? b[j].z : b[j].w;
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(ua), __uint_as_float(ub),
                                                                         acc[i][j], 0, 0, 0);
                    }
        }
    }
};

// Block tile (WM*TM*32) x (WN*TN*32): WM x WN waves, each TM x TN MFMA tiles of 32 x 32. STAGES = 2:
// two LDS buffers, the next step loaded to registers during the MFMAs and written to the other
// buffer (one barrier per step); STAGES = 1: one buffer, written after a barrier (half the LDS,
// so twice the blocks per CU). Rows past M / N are read as zeros and not stored.
template <typename T, int WM, int WN, int TM, int TN, int STAGES, int DEPTH = 1>
__global__ void __launch_bounds__(64 * WM * WN)
dense_nt_kernel(const T* __restrict__ A, const T* __restrict__ B, float* __restrict__ C, int64_t M, int N, int K,
                int64_t ldc, unsigned m_tiles, unsigned n_tiles) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = 64 * WM * WN;
    constexpr int PA = BM * 8 / NT, PB = BN * 8 / NT;  // 16-B chunks per thread per step
    static_assert(PA * NT == BM * 8 && PB * NT == BN * 8, "tile/threads");
    __shared__ uint4 lds[STAGES][(BM + BN) * 8];
    // XCD-aware tile order (see the file header)
    const unsigned i = blockIdx.x, xcd = i & 7u, j = i >> 3;
    const unsigned mt = (j / n_tiles) * 8u + xcd, nt = j % n_tiles;
    if (mt >= m_tiles) return;  // uniform
    const int64_t m0 = (int64_t)mt * BM;
    const int n0 = (int)nt * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w / WN, wn = w % WN;
    constexpr int kE = DenseStep<T>::kElems;
    const int steps = K / kE;
    constexpr int RPP = NT / 8;  // rows covered by one pass of the block (8 chunks per row)
    const int srow = tid >> 3, sch = tid & 7;
    const char* __restrict__ ga[PA];
    const char* __restrict__ gb[PB];
    bool va[PA], vb[PB];
#pragma unroll
    for (int q = 0; q < PA; ++q) {
        const int64_t ra = m0 + srow + RPP * q;
        va[q] = ra < M;
        ga[q] = reinterpret_cast<const char*>(A + (va[q] ? ra : 0) * (int64_t)K) + sch * 16;
    }
#pragma unroll
    for (int q = 0; q < PB; ++q) {
        const int rb = n0 + srow + RPP * q;
        vb[q] = rb < N;
        gb[q] = reinterpret_cast<const char*>(B + (int64_t)(vb[q] ? rb : 0) * K) + sch * 16;
    }
    uint4 ra[PA], rb[PB];
    auto load_to = [&](uint4 (&xa)[PA], uint4 (&xb)[PB], int s) {
        const int64_t off = (int64_t)s * kRowBytes;
#pragma unroll
        for (int q = 0; q < PA; ++q) xa[q] = *reinterpret_cast<const uint4*>(ga[q] + off);
#pragma unroll
        for (int q = 0; q < PB; ++q) xb[q] = *reinterpret_cast<const uint4*>(gb[q] + off);
    };
    auto store_from = [&](const uint4 (&xa)[PA], const uint4 (&xb)[PB], int buf) {
        const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < PA; ++q) lds[buf][swz(srow + RPP * q, sch)] = va[q] ? xa[q] : z;
#pragma unroll
        for (int q = 0; q < PB; ++q) lds[buf][BM * 8 + swz(srow + RPP * q, sch)] = vb[q] ? xb[q] : z;
    };
    auto load = [&](int s) { load_to(ra, rb, s); };
    auto store = [&](int buf) { store_from(ra, rb, buf); };
    f32x16 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;
    const int ra0 = wm * TM * 32, rb0 = wn * TN * 32;
    if constexpr (DEPTH == 2 && STAGES == 2) {
        // two register sets, each step's tiles loaded two steps ahead (no copies between the sets):
        // step s computes from LDS buffer s & 1 while its successor's registers are already loaded
        uint4 ra2[PA], rb2[PB];
        load(0);
        store(0);
        __syncthreads();
        if (steps > 1) load(1);
        for (int s = 0; s < steps; s += 2) {
            if (s + 2 < steps) load_to(ra2, rb2, s + 2);
            DenseStep<T>::template compute<TM, TN>(lds[0], lds[0] + BM * 8, ra0, rb0, lane, acc);
            if (s + 1 < steps) store(1);
            __syncthreads();
            if (s + 1 >= steps) break;
            if (s + 3 < steps) load(s + 3);
            DenseStep<T>::template compute<TM, TN>(lds[1], lds[1] + BM * 8, ra0, rb0, lane, acc);
            if (s + 2 < steps) store_from(ra2, rb2, 0);
            __syncthreads();
        }
    } else {
    load(0);
    store(0);
    __syncthreads();
    for (int s = 0; s < steps; ++s) {
        const int cur = STAGES == 2 ? (s & 1) : 0;
        if (s + 1 < steps) load(s + 1);  // in flight while this step's MFMAs run
        DenseStep<T>::template compute<TM, TN>(lds[cur], lds[cur] + BM * 8, ra0, rb0, lane, acc);
        if (STAGES == 2) {
            if (s + 1 < steps) store(cur ^ 1);  // the other buffer: last read before the previous barrier
            __syncthreads();
        } else {
            __syncthreads();
            if (s + 1 < steps) store(0);
            __syncthreads();
        }
    }
    }
    // epilogue: lane holds column lane & 31 of each 32 x 32 tile, rows
    // (e & 3) + 8 (e >> 2) + 4 (lane >> 5) for e < 16
    const int col = lane & 31, rh = 4 * (lane >> 5);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const int c = n0 + rb0 + b * 32 + col;
            if (c >= N) continue;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t r = m0 + ra0 + a * 32 + (e & 3) + 8 * (e >> 2) + rh;
                if (r < M) C[r * ldc + c] = acc[a][b][e];
            }
        }
}

// LDS-direct staging (the default): tile 256 x 256, K-tile = 128 B of every row (64 bf16 / 32 f32),
// 8 waves (2 M x 4 N), each wave 128 x 64 of C as 8 x 4 tiles of 16 x 16.
//   bf16: v_mfma_f32_16x16x32_bf16, lane l: A[row l & 15][k 8(l >> 4) .. +7] (16 B), the same for B's
//         row = C's column;
//   f32:  v_mfma_f32_16x16x4_f32 (exact f32 products), lane l: A[row l & 15][k = l >> 4]; a lane reads
//         16 B = 4 consecutive k and feeds element e to MFMA e, so MFMA (s, e) sums k = 16s + 4q + e
//         over the lane groups q — a permutation of the K-tile, the same for A and B.
//   C (both): col l & 15, rows 4(l >> 4) + r.
// Operands go global -> LDS with global_load_lds_dwordx4 (16 B per lane, no VGPR round trip): per
// K-tile 4 instructions per thread for A and 4 for B. The LDS image is lane-linear (128-B rows of 8
// chunks); the XOR swizzle (chunk c of row r holds global chunk c ^ (r & 7)) is applied on the
// per-lane SOURCE address, so a 16-lane group's fragment reads (16 rows, one chunk) hit 16 distinct
// 16-B bank slots. Two K-tile buffers: K-tile t + 1 is issued before K-tile t's MFMAs, one vmcnt(0) +
// barrier per K-tile. All LDS in ONE __shared__ array (a second one makes hipcc wait vmcnt(0) before
// the first ds_read). Rows past M / N are read (clamped) and never stored.
typedef short bf16x8s __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool BF16>
__global__ void __launch_bounds__(512)
dense_glds_kernel(const void* __restrict__ Av, const void* __restrict__ Bv, float* __restrict__ C,
                  int64_t M, int N, int K, int64_t ldc, unsigned m_tiles, unsigned n_tiles) {
    constexpr int BM = 256, BN = 256, KC = 8;       // KC: 16-B chunks per 128-B row slice
    constexpr int ES = BF16 ? 2 : 4, KT = 128 / ES;  // element size, elements per K-tile
    __shared__ uint4 lds[2 * (BM + BN) * KC];       // 2 x 64 KB
    const unsigned bi = blockIdx.x, xcd = bi & 7u, j = bi >> 3;
    const unsigned mt = (j / n_tiles) * 8u + xcd, nt = j % n_tiles;
    if (mt >= m_tiles) return;  // uniform
    const int64_t m0 = (int64_t)mt * BM;
    const int n0 = (int)nt * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 2, wn = w & 3;
    const int steps = K / KT;
    // staging sources: instruction i moves LDS chunks [i * 512 + 64 w, + 64) of the A (B) image
    const int srow = tid >> 3, sch = tid & 7, sxc = sch ^ (srow & 7);
    const char* ga[4];
    const char* gb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t ra = std::min<int64_t>(m0 + i * 64 + srow, M - 1);
        const int rb = std::min(n0 + i * 64 + srow, N - 1);
        ga[i] = reinterpret_cast<const char*>(Av) + (ra * (int64_t)K + sxc * (16 / ES)) * ES;
        gb[i] = reinterpret_cast<const char*>(Bv) + ((int64_t)rb * K + sxc * (16 / ES)) * ES;
    }
    auto stage = [&](int kt, int buf) {
        uint4* base = lds + buf * (BM + BN) * KC;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds(ga[i] + (int64_t)kt * 128, base + i * 512 + 64 * w, 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds(gb[i] + (int64_t)kt * 128, base + BM * KC + i * 512 + 64 * w, 16, 0, 0);
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fq = lane >> 4;
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < steps; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < steps) stage(kt + 1, cur ^ 1);  // buffer cur ^ 1: last read before the previous barrier
        const uint4* sa = lds + cur * (BM + BN) * KC;
        const uint4* sb = sa + BM * KC;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int cc = 4 * s + fq;
            uint4 bfr[4];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int r = wn * 64 + ni * 16 + fr;
                bfr[ni] = sb[r * KC + (cc ^ (r & 7))];
            }
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                const int r = wm * 128 + mi * 16 + fr;
                const uint4 afr = sa[r * KC + (cc ^ (r & 7))];
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    if constexpr (BF16) {
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8s, afr), __builtin_bit_cast(bf16x8s, bfr[ni]), acc[mi][ni], 0, 0, 0);
                    } else {
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(afr.x), __uint_as_float(bfr[ni].x),
                                                                          acc[mi][ni], 0, 0, 0);
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(afr.y), __uint_as_float(bfr[ni].y),
                                                                          acc[mi][ni], 0, 0, 0);
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(afr.z), __uint_as_float(bfr[ni].z),
                                                                          acc[mi][ni], 0, 0, 0);
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(afr.w), __uint_as_float(bfr[ni].w),
                                                                          acc[mi][ni], 0, 0, 0);
                    }
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int c = n0 + wn * 64 + ni * 16 + fr;
            if (c >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = m0 + wm * 128 + mi * 16 + 4 * fq + r;
                if (row < M) C[row * ldc + c] = acc[mi][ni][r];
            }
        }
}

template <bool BF16>
int launch_dense_glds(const void* X, const void* G, float* Y, int64_t n, int64_t m, int64_t p, int64_t ldy,
                      hipStream_t st) {
    const unsigned m_tiles = (unsigned)((n + 255) / 256), n_tiles = (unsigned)((p + 255) / 256);
    const uint64_t blocks = (uint64_t)((m_tiles + 7) / 8) * 8ull * n_tiles;
    if (blocks >= (1ull << 31)) return fail(RP_ERR_UNSUPPORTED, "too many rows for one launch");
    hipLaunchKernelGGL((dense_glds_kernel<BF16>), dim3((unsigned)blocks), dim3(512), 0, st, X, G, Y, n, (int)p, (int)m,
                       ldy, m_tiles, n_tiles);
    HIP_TRY(hipGetLastError());
    return RP_OK;
}

// Four-stage ring (variant 11): the same 256 x 256 tile and 8 waves of 128 x 64 in 16 x 16 MFMAs, but
// K-tiles of 64 B per row (32 bf16 / 16 f32) in a ring of four 32 KB LDS buffers, so three K-tiles
// are in flight while one is multiplied (the two-buffer kernel keeps one, ~1 us ahead: less than a
// loaded HBM round trip). Per K-tile: wait for the oldest stage (vmcnt(8) with two younger stages
// still in flight), one barrier, issue the K-tile three ahead into the buffer everyone finished,
// then one MFMA substep (bf16: 32 x 16x16x32; f32: 128 x 16x16x4 over the lane groups' 4 k each).
// LDS rows of 4 chunks; chunk c of row r at c ^ F(r), F(r) = -(r >> 2) & 3, which makes each of
// ds_read_b128's 16-lane groups hit 16 distinct 16-B bank slots (rows 16 B x 4 apart share banks
// only across groups).
template <bool BF16, int NS = 4>
__global__ void __launch_bounds__(512)
dense_ring_kernel(const void* __restrict__ Av, const void* __restrict__ Bv, float* __restrict__ C,
                  int64_t M, int N, int K, int64_t ldc, unsigned m_tiles, unsigned n_tiles) {
    constexpr int BM = 256, BN = 256, KC = 4;  // KC: 16-B chunks per 64-B row slice; NS ring buffers
    constexpr int ES = BF16 ? 2 : 4, KT = 64 / ES;     // element size, elements per K-tile
    constexpr int SZ = (BM + BN) * KC;                  // chunks per stage
    __shared__ uint4 lds[NS * SZ];                      // NS x 32 KB
    const unsigned bi = blockIdx.x, xcd = bi & 7u, j = bi >> 3;
    const unsigned mt = (j / n_tiles) * 8u + xcd, nt = j % n_tiles;
    if (mt >= m_tiles) return;  // uniform
    const int64_t m0 = (int64_t)mt * BM;
    const int n0 = (int)nt * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 2, wn = w & 3;
    const int steps = K / KT;
    auto F = [](int r) { return (4 - ((r >> 2) & 3)) & 3; };
    // staging: instruction i moves LDS chunks [i * 512 + 64 w, + 64) = rows i * 128 + tid / 4
    const int srow = tid >> 2, sxc = (tid & 3) ^ F(srow);
    const char* ga[2];
    const char* gb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int64_t ra = std::min<int64_t>(m0 + i * 128 + srow, M - 1);
        const int rb = std::min(n0 + i * 128 + srow, N - 1);
        ga[i] = reinterpret_cast<const char*>(Av) + (ra * (int64_t)K + sxc * (16 / ES)) * ES;
        gb[i] = reinterpret_cast<const char*>(Bv) + ((int64_t)rb * K + sxc * (16 / ES)) * ES;
    }
    // global_load_lds_dwordx4 issued as inline asm: the compiler does not see these LDS writes, so
    // it inserts no vmcnt(0) before this wave's ds_reads or the barrier (it would wait for all
    // three stages in flight); the vmcnt waits below are explicit. M0 = the wave's LDS destination.
    const uint32_t lds0 = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)reinterpret_cast<uintptr_t>(lds + 64 * w));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: the clobber keeps the compiler's own uses safe
    auto dma = [&](const char* g, uint32_t l) {
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
    };
#pragma clang diagnostic pop
    auto stage = [&](int kt) {
        const uint32_t base = lds0 + (uint32_t)((kt % NS) * SZ) * 16u;
#pragma unroll
        for (int i = 0; i < 2; ++i) dma(ga[i] + (int64_t)kt * 64, base + i * 512 * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i) dma(gb[i] + (int64_t)kt * 64, base + (BM * KC + i * 512) * 16);
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fq = lane >> 4;
    for (int kt = 0; kt < NS - 1 && kt < steps; ++kt) stage(kt);
    for (int kt = 0; kt < steps; ++kt) {
        // K-tile kt landed (this wave's loads; the barrier: everyone's); younger stages stay in flight
        // (4 loads per stage and thread; NS - 2 younger stages at most)
        const int younger = std::min(NS - 2, steps - 1 - kt);
        if (younger >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (kt + NS - 1 < steps) stage(kt + NS - 1);  // into the buffer of K-tile kt - 1: all done with it
        const uint4* sa = lds + (kt % NS) * SZ;
        const uint4* sb = sa + BM * KC;
        uint4 bfr[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int r = wn * 64 + ni * 16 + fr;
            bfr[ni] = sb[r * KC + (fq ^ F(r))];
        }
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
            const int r = wm * 128 + mi * 16 + fr;
            const uint4 afr = sa[r * KC + (fq ^ F(r))];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                if constexpr (BF16) {
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8s, afr), __builtin_bit_cast(bf16x8s, bfr[ni]), acc[mi][ni], 0, 0, 0);
                } else {
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(afr.x), __uint_as_float(bfr[ni].x),
                                                                      acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(afr.y), __uint_as_float(bfr[ni].y),
                                                                      acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(afr.z), __uint_as_float(bfr[ni].z),
                                                                      acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(afr.w), __uint_as_float(bfr[ni].w),
                                                                      acc[mi][ni], 0, 0, 0);
                }
            }
        }
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int c = n0 + wn * 64 + ni * 16 + fr;
            if (c >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = m0 + wm * 128 + mi * 16 + 4 * fq + r;
                if (row < M) C[row * ldc + c] = acc[mi][ni][r];
            }
        }
}

template <bool BF16, int NS = 4>
int launch_dense_ring(const void* X, const void* G, float* Y, int64_t n, int64_t m, int64_t p, int64_t ldy,
                      hipStream_t st) {
    const unsigned m_tiles = (unsigned)((n + 255) / 256), n_tiles = (unsigned)((p + 255) / 256);
    const uint64_t blocks = (uint64_t)((m_tiles + 7) / 8) * 8ull * n_tiles;
    if (blocks >= (1ull << 31)) return fail(RP_ERR_UNSUPPORTED, "too many rows for one launch");
    hipLaunchKernelGGL((dense_ring_kernel<BF16, NS>), dim3((unsigned)blocks), dim3(512), 0, st, X, G, Y, n, (int)p, (int)m,
                       ldy, m_tiles, n_tiles);
    HIP_TRY(hipGetLastError());
    return RP_OK;
}

// f64 (sklearn computes in X's dtype): v_mfma_f64_16x16x4_f64 — lane l supplies A[row l & 15][k = l >> 4]
// (one double), C/D: col l & 15, row (l >> 4) + 4 r (NOT the f32 map). Tile 256 x 128, 8 waves (4 M x
// 2 N) of 64 x 64 = 4 x 4 MFMA tiles (128 accumulator VGPRs); K-tile = 128 B of a row = 16 doubles; a
// lane reads 16 B = 2 consecutive k and feeds element e to MFMA e, so MFMA (s, e) sums
// k = 8s + 2q + e over the lane groups q (a permutation of the K-tile, the same for A and B). Staging
// as dense_glds_kernel (global_load_lds_dwordx4, source-side XOR swizzle, two K-tile buffers).
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512)
dense_glds_f64_kernel(const double* __restrict__ A, const double* __restrict__ B, double* __restrict__ C,
                      int64_t M, int N, int K, int64_t ldc, unsigned m_tiles, unsigned n_tiles) {
    constexpr int BM = 256, BN = 128, KC = 8, KT = 16;
    __shared__ uint4 lds[2 * (BM + BN) * KC];  // 2 x 48 KB
    const unsigned bi = blockIdx.x, xcd = bi & 7u, j = bi >> 3;
    const unsigned mt = (j / n_tiles) * 8u + xcd, nt = j % n_tiles;
    if (mt >= m_tiles) return;  // uniform
    const int64_t m0 = (int64_t)mt * BM;
    const int n0 = (int)nt * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
    const int steps = K / KT;
    const int srow = tid >> 3, sch = tid & 7, sxc = sch ^ (srow & 7);
    const double* ga[4];
    const double* gb[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) ga[i] = A + std::min<int64_t>(m0 + i * 64 + srow, M - 1) * (int64_t)K + sxc * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) gb[i] = B + (int64_t)std::min(n0 + i * 64 + srow, N - 1) * K + sxc * 2;
    auto stage = [&](int kt, int buf) {
        uint4* base = lds + buf * (BM + BN) * KC;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds(ga[i] + (int64_t)kt * KT, base + i * 512 + 64 * w, 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds(gb[i] + (int64_t)kt * KT, base + BM * KC + i * 512 + 64 * w, 16, 0, 0);
    };
    f64x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int fr = lane & 15, fq = lane >> 4;
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < steps; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < steps) stage(kt + 1, cur ^ 1);
        const uint4* sa = lds + cur * (BM + BN) * KC;
        const uint4* sb = sa + BM * KC;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int cc = 4 * s + fq;
            uint4 bfr[4];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int r = wn * 64 + ni * 16 + fr;
                bfr[ni] = sb[r * KC + (cc ^ (r & 7))];
            }
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const int r = wm * 64 + mi * 16 + fr;
                const uint4 afr = sa[r * KC + (cc ^ (r & 7))];
                const double a0 = __hiloint2double((int)afr.y, (int)afr.x), a1 = __hiloint2double((int)afr.w, (int)afr.z);
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    const double b0 = __hiloint2double((int)bfr[ni].y, (int)bfr[ni].x);
                    const double b1 = __hiloint2double((int)bfr[ni].w, (int)bfr[ni].z);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[mi][ni], 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int c = n0 + wn * 64 + ni * 16 + fr;
            if (c >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = m0 + wm * 64 + mi * 16 + fq + 4 * r;
                if (row < M) C[row * ldc + c] = acc[mi][ni][r];
            }
        }
}

// f64 ring (the default): dense_glds_f64_kernel's tile, fragments and swizzle, but NS = 3 K-tile
// buffers of 48 KB (144 KB of LDS), so two K-tiles are in flight while one is multiplied (the
// two-buffer kernel waits vmcnt(0) at the end of every K-tile for the one it issued at the start).
// The LDS-direct loads are inline asm as in dense_ring_kernel: the compiler then inserts no vmcnt(0)
// before the fragment reads; the waits below are explicit (6 loads per thread per K-tile).
__global__ void __launch_bounds__(512)
dense_ring_f64_kernel(const double* __restrict__ A, const double* __restrict__ B, double* __restrict__ C,
                      int64_t M, int N, int K, int64_t ldc, unsigned m_tiles, unsigned n_tiles) {
    constexpr int BM = 256, BN = 128, KC = 8, KT = 16, NS = 3;
    constexpr int SZ = (BM + BN) * KC;  // uint4 per stage
    __shared__ uint4 lds[NS * SZ];
    const unsigned bi = blockIdx.x, xcd = bi & 7u, j = bi >> 3;
    const unsigned mt = (j / n_tiles) * 8u + xcd, nt = j % n_tiles;
    if (mt >= m_tiles) return;  // uniform
    const int64_t m0 = (int64_t)mt * BM;
    const int n0 = (int)nt * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
    const int steps = K / KT;
    const int srow = tid >> 3, sch = tid & 7, sxc = sch ^ (srow & 7);
    const double* ga[4];
    const double* gb[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) ga[i] = A + std::min<int64_t>(m0 + i * 64 + srow, M - 1) * (int64_t)K + sxc * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) gb[i] = B + (int64_t)std::min(n0 + i * 64 + srow, N - 1) * K + sxc * 2;
    const uint32_t lds0 = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)reinterpret_cast<uintptr_t>(lds + 64 * w));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: the clobber keeps the compiler's own uses safe
    auto dma = [&](const double* g, uint32_t l) {
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
    };
#pragma clang diagnostic pop
    auto stage = [&](int kt) {
        const uint32_t base = lds0 + (uint32_t)((kt % NS) * SZ) * 16u;
#pragma unroll
        for (int i = 0; i < 4; ++i) dma(ga[i] + (int64_t)kt * KT, base + i * 512 * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i) dma(gb[i] + (int64_t)kt * KT, base + (BM * KC + i * 512) * 16);
    };
    f64x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int fr = lane & 15, fq = lane >> 4;
    for (int kt = 0; kt < NS - 1 && kt < steps; ++kt) stage(kt);
    for (int kt = 0; kt < steps; ++kt) {
        // K-tile kt landed (this wave's loads; the barrier: everyone's); at most one younger in flight
        if (kt + 1 < steps) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (kt + NS - 1 < steps) stage(kt + NS - 1);  // into the buffer of K-tile kt - 1: all done with it
        const uint4* sa = lds + (kt % NS) * SZ;
        const uint4* sb = sa + BM * KC;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int cc = 4 * s + fq;
            uint4 bfr[4];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int r = wn * 64 + ni * 16 + fr;
                bfr[ni] = sb[r * KC + (cc ^ (r & 7))];
            }
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const int r = wm * 64 + mi * 16 + fr;
                const uint4 afr = sa[r * KC + (cc ^ (r & 7))];
                const double a0 = __hiloint2double((int)afr.y, (int)afr.x), a1 = __hiloint2double((int)afr.w, (int)afr.z);
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    const double b0 = __hiloint2double((int)bfr[ni].y, (int)bfr[ni].x);
                    const double b1 = __hiloint2double((int)bfr[ni].w, (int)bfr[ni].z);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[mi][ni], 0, 0, 0);
                }
            }
        }
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int c = n0 + wn * 64 + ni * 16 + fr;
            if (c >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = m0 + wm * 64 + mi * 16 + fq + 4 * r;
                if (row < M) C[row * ldc + c] = acc[mi][ni][r];
            }
        }
}

int launch_dense_f64(const void* X, const void* G, double* Y, int64_t n, int64_t m, int64_t p, int64_t ldy,
                     hipStream_t st, bool ring) {
    const unsigned m_tiles = (unsigned)((n + 255) / 256), n_tiles = (unsigned)((p + 127) / 128);
    const uint64_t blocks = (uint64_t)((m_tiles + 7) / 8) * 8ull * n_tiles;
    if (blocks >= (1ull << 31)) return fail(RP_ERR_UNSUPPORTED, "too many rows for one launch");
    if (ring)
        hipLaunchKernelGGL(dense_ring_f64_kernel, dim3((unsigned)blocks), dim3(512), 0, st, (const double*)X,
                           (const double*)G, Y, n, (int)p, (int)m, ldy, m_tiles, n_tiles);
    else
        hipLaunchKernelGGL(dense_glds_f64_kernel, dim3((unsigned)blocks), dim3(512), 0, st, (const double*)X,
                           (const double*)G, Y, n, (int)p, (int)m, ldy, m_tiles, n_tiles);
    HIP_TRY(hipGetLastError());
    return RP_OK;
}

template <typename T, int WM, int WN, int TM, int TN, int STAGES, int DEPTH = 1>
int launch_dense(const void* X, const void* G, float* Y, int64_t n, int64_t m, int64_t p, int64_t ldy,
                 hipStream_t st) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    const unsigned m_tiles = (unsigned)((n + BM - 1) / BM), n_tiles = (unsigned)((p + BN - 1) / BN);
    const uint64_t blocks = (uint64_t)((m_tiles + 7) / 8) * 8ull * n_tiles;
    if (blocks >= (1ull << 31)) return fail(RP_ERR_UNSUPPORTED, "too many rows for one launch");
    hipLaunchKernelGGL((dense_nt_kernel<T, WM, WN, TM, TN, STAGES, DEPTH>), dim3((unsigned)blocks), dim3(64 * WM * WN), 0,
                       st, (const T*)X, (const T*)G, Y, n, (int)p, (int)m, ldy, m_tiles, n_tiles);
    HIP_TRY(hipGetLastError());
    return RP_OK;
}

// tile variants (the `variant` argument, measurements): 0 = 128x128 2 stages, 1 = 128x128 1 stage,
// 2 = 256x128 1 stage, 3 = 128x256 2 stages (8 waves), 4 = 256x256 1 stage (8 waves), 5 = 256x256
// 2 stages (128 KB LDS, 8 waves)
// defaults: the four-stage LDS-direct ring for both (measured, profiles/r03_dense_*: bf16 1114 TF vs
// 980 for the two-buffer kernel (variant 10) and 353 for variant 5; f32 145 TF vs 133 and 97;
// hipBLASLt on the same shapes 1302 / 154 TF)
constexpr int kDenseVariantBf16 = 11, kDenseVariantF32 = 11;
template <typename T>
int dispatch_dense(int v, const void* X, const void* G, float* Y, int64_t n, int64_t m, int64_t p, int64_t ldy,
                   hipStream_t st) {
    if (v == 10) return launch_dense_glds<std::is_same<T, uint16_t>::value>(X, G, Y, n, m, p, ldy, st);
    if (v == 11) return launch_dense_ring<std::is_same<T, uint16_t>::value>(X, G, Y, n, m, p, ldy, st);
    switch (v) {
        case 1: return launch_dense<T, 2, 2, 2, 2, 1>(X, G, Y, n, m, p, ldy, st);
        case 2: return launch_dense<T, 2, 2, 4, 2, 1>(X, G, Y, n, m, p, ldy, st);
        case 3: return launch_dense<T, 2, 4, 2, 2, 2>(X, G, Y, n, m, p, ldy, st);
        case 4: return launch_dense<T, 2, 4, 4, 2, 1>(X, G, Y, n, m, p, ldy, st);
        case 5: return launch_dense<T, 2, 4, 4, 2, 2>(X, G, Y, n, m, p, ldy, st);
        case 6: return launch_dense<T, 2, 4, 4, 2, 2, 2>(X, G, Y, n, m, p, ldy, st);
        case 7: return launch_dense<T, 2, 2, 2, 2, 2, 2>(X, G, Y, n, m, p, ldy, st);
        case 8: return launch_dense<T, 2, 2, 4, 4, 2, 2>(X, G, Y, n, m, p, ldy, st);
        case 9: return launch_dense<T, 2, 2, 4, 4, 2, 1>(X, G, Y, n, m, p, ldy, st);
        default: return launch_dense<T, 2, 2, 2, 2, 2>(X, G, Y, n, m, p, ldy, st);
    }
}

}  // namespace

extern "C" int rp_dense_project_device(int device, const void* X, int32_t dtype, int64_t n, int64_t m,
                                       const void* G, int64_t p, void* Y, int64_t ldy, void* stream,
                                       int32_t variant) {
    if (!X || !G || !Y) return fail(RP_ERR_INVALID, "NULL operand");
    if (variant < -1 || variant > 11) return fail(RP_ERR_INVALID, "variant must be -1 (default) or 0..11");
    if (dtype != RP_F32 && dtype != RP_BF16 && dtype != RP_F64)
        return fail(RP_ERR_INVALID, "dtype must be RP_F32, RP_BF16 or RP_F64");
    if (n < 0 || m <= 0 || p <= 0 || ldy < p) return fail(RP_ERR_INVALID, "bad shape");
    const int step = dtype == RP_BF16 ? 64 : dtype == RP_F32 ? 32 : 16;
    if (m % step) return fail(RP_ERR_UNSUPPORTED, "m=%lld must be a multiple of %d", (long long)m, step);
    if (m > INT32_MAX || p > INT32_MAX) return fail(RP_ERR_UNSUPPORTED, "m or p too large");
    const uintptr_t al = (uintptr_t)X | (uintptr_t)G;
    if (al & 15) return fail(RP_ERR_INVALID, "X and G must be 16-byte aligned");
    if (n == 0) return RP_OK;
    HIP_TRY(hipSetDevice(device));
    const int sv = variant;  // per call (measurements); -1 = the default
    const int v = sv >= 0 ? sv : (dtype == RP_BF16 ? kDenseVariantBf16 : kDenseVariantF32);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == RP_F64) return launch_dense_f64(X, G, (double*)Y, n, m, p, ldy, st, sv != 10);  // 10: two buffers
    return dtype == RP_BF16 ? dispatch_dense<uint16_t>(v, X, G, (float*)Y, n, m, p, ldy, st)
                            : dispatch_dense<float>(v, X, G, (float*)Y, n, m, p, ldy, st);
}
