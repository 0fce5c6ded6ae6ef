// rp_dense.hip — the dense Gaussian projection as a hand-written gfx950 MFMA GEMM
// (BASELINE.json configs[4]).
//
// Reference semantics: sklearn GaussianRandomProjection.transform(X) = X @ components_.T
// (sklearn/random_projection.py:569-612): Y[n x p] = X[n x m] . G[p x m]^T. Both operands are
// row-major with the contraction index m contiguous ("NT" GEMM), the layout the MFMA operand
// fragments want: a lane's A and B elements are consecutive in memory.
//
//   bf16: v_mfma_f32_32x32x16_bf16 — bf16 operands, f32 accumulate, f32 result.
//   f32:  v_mfma_f32_32x32x2_f32   — exact f32 products (gfx950 has no xf32), f32 accumulate.
//
// Block tile 128 x 128, 4 waves (2 x 2), each wave 64 x 64 = 2 x 2 MFMA tiles of 32 x 32. K step
// 128 bytes of a row (64 bf16 / 32 f32): the next step's tiles are loaded global -> registers
// while the current step's MFMAs run, then written to the other LDS buffer (two buffers, one
// barrier per step). LDS rows are 128 B (8 chunks of 16 B) stored XOR-swizzled (chunk c of row r
// at c ^ (r & 7)) so a wave's 16-B fragment reads of 8 consecutive rows hit distinct banks.
// f32: the K order inside a step is permuted (lane half h takes k = 16h + t for MFMA t) so every
// lane reads 64 contiguous bytes per operand per step; the sum is over the same products.
// Block -> tile map is XCD-aware: XCD x (workgroup i runs on XCD i % 8) takes the M tiles
// congruent to x mod 8 and walks each M tile's N tiles back to back, so an X tile is fetched from
// HBM once and re-read from that XCD's L2.
#include "rp_common.h"

using namespace rpd;

namespace {

constexpr int kDBM = 128, kDBN = 128, kDThreads = 256;
constexpr int kRowBytes = 128;                       // one K step of a row
constexpr int kTileBytes = kDBM * kRowBytes;         // 16 KB per operand per stage

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

template <typename T>
struct DenseStep;

// bf16: K step 64 elements = 4 MFMA k-substeps of 16; lane (r, h) reads chunk 2s + h of its row
template <>
struct DenseStep<uint16_t> {
    static constexpr int kElems = 64;
    __device__ static void compute(const uint4* __restrict__ sA, const uint4* __restrict__ sB, int wm, int wn,
                                   int lane, f32x16 (&acc)[2][2]) {
        const int r = lane & 31, h = lane >> 5;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            bf16x8 a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ra = wm * 64 + i * 32 + r, rb = wn * 64 + i * 32 + r;
                const uint4 va = sA[swz(ra, 2 * s + h)], vb = sB[swz(rb, 2 * s + h)];
                a[i] = __builtin_bit_cast(bf16x8, va);
                b[i] = __builtin_bit_cast(bf16x8, vb);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    }
};

// f32: K step 32 elements = 16 MFMAs of K = 2; MFMA t, lane half h uses k = 16h + t (a permutation
// of the step's K order, the same for A and B): lane (r, h) reads chunks 4h .. 4h + 3 of its row
template <>
struct DenseStep<float> {
    static constexpr int kElems = 32;
    __device__ static void compute(const uint4* __restrict__ sA, const uint4* __restrict__ sB, int wm, int wn,
                                   int lane, f32x16 (&acc)[2][2]) {
        const int r = lane & 31, h = lane >> 5;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float a[2][4], b[2][4];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ra = wm * 64 + i * 32 + r, rb = wn * 64 + i * 32 + r;
                const uint4 va = sA[swz(ra, 4 * h + q)], vb = sB[swz(rb, 4 * h + q)];
                a[i][0] = __uint_as_float(va.x); a[i][1] = __uint_as_float(va.y);
                a[i][2] = __uint_as_float(va.z); a[i][3] = __uint_as_float(va.w);
                b[i][0] = __uint_as_float(vb.x); b[i][1] = __uint_as_float(vb.y);
                b[i][2] = __uint_as_float(vb.z); b[i][3] = __uint_as_float(vb.w);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
        }
    }
};

// One block: rows [m0, m0 + 128) of A x rows [n0, n0 + 128) of B. Rows past M / N are read as
// zeros (clamped loads, masked) and not stored. K must be a multiple of the step (host check).
template <typename T>
__global__ void __launch_bounds__(kDThreads)
dense_nt_kernel(const T* __restrict__ A, const T* __restrict__ B, float* __restrict__ C, int64_t M, int N, int K,
                int64_t ldc, unsigned m_tiles, unsigned n_tiles) {
    __shared__ uint4 lds[2][2][kTileBytes / 16];  // [stage][A|B][128 rows x 8 chunks]: 64 KB
    // XCD-aware tile order (see the file header)
    const unsigned i = blockIdx.x, xcd = i & 7u, j = i >> 3;
    const unsigned mt = (j / n_tiles) * 8u + xcd, nt = j % n_tiles;
    if (mt >= m_tiles) return;  // uniform
    const int64_t m0 = (int64_t)mt * kDBM;
    const int n0 = (int)nt * kDBN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
    constexpr int kE = DenseStep<T>::kElems;
    const int steps = K / kE;
    // staging: thread t moves chunks t + 256 q (q < 4) of each operand: row (t >> 3) + 32 q, chunk t & 7
    const int srow = tid >> 3, sch = tid & 7;
    const char* __restrict__ ga[4];
    const char* __restrict__ gb[4];
    bool va[4], vb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t ra = m0 + srow + 32 * q;
        const int rb = n0 + srow + 32 * q;
        va[q] = ra < M;
        vb[q] = rb < N;
        ga[q] = reinterpret_cast<const char*>(A + (va[q] ? ra : 0) * (int64_t)K) + sch * 16;
        gb[q] = reinterpret_cast<const char*>(B + (int64_t)(vb[q] ? rb : 0) * K) + sch * 16;
    }
    uint4 ra[4], rb[4];
    auto load = [&](int s) {
        const int64_t off = (int64_t)s * kRowBytes;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ra[q] = *reinterpret_cast<const uint4*>(ga[q] + off);
            rb[q] = *reinterpret_cast<const uint4*>(gb[q] + off);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 z = make_uint4(0, 0, 0, 0);
            lds[buf][0][swz(srow + 32 * q, sch)] = va[q] ? ra[q] : z;
            lds[buf][1][swz(srow + 32 * q, sch)] = vb[q] ? rb[q] : z;
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;
    load(0);
    store(0);
    __syncthreads();
    for (int s = 0; s < steps; ++s) {
        const int cur = s & 1;
        if (s + 1 < steps) load(s + 1);  // in flight while this step's MFMAs run
        DenseStep<T>::compute(lds[cur][0], lds[cur][1], wm, wn, lane, acc);
        if (s + 1 < steps) store(cur ^ 1);  // the other buffer: last read before the previous barrier
        __syncthreads();
    }
    // epilogue: 32 x 32 tile (i, j) of the wave; lane holds column lane & 31, rows
    // (e & 3) + 8 (e >> 2) + 4 (lane >> 5) for e < 16
    const int col = lane & 31, rh = 4 * (lane >> 5);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int c = n0 + wn * 64 + b * 32 + col;
            if (c >= N) continue;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t r = m0 + wm * 64 + a * 32 + (e & 3) + 8 * (e >> 2) + rh;
                if (r < M) C[r * ldc + c] = acc[a][b][e];
            }
        }
}

}  // namespace

extern "C" int rp_dense_project_device(int device, const void* X, int32_t dtype, int64_t n, int64_t m,
                                       const void* G, int64_t p, float* Y, int64_t ldy, void* stream) {
    if (!X || !G || !Y) return fail(RP_ERR_INVALID, "NULL operand");
    if (dtype != RP_F32 && dtype != RP_BF16) return fail(RP_ERR_INVALID, "dtype must be RP_F32 or RP_BF16");
    if (n < 0 || m <= 0 || p <= 0 || ldy < p) return fail(RP_ERR_INVALID, "bad shape");
    const int step = dtype == RP_BF16 ? 64 : 32;
    if (m % step) return fail(RP_ERR_UNSUPPORTED, "m=%lld must be a multiple of %d", (long long)m, step);
    if (m > INT32_MAX || p > INT32_MAX) return fail(RP_ERR_UNSUPPORTED, "m or p too large");
    const uintptr_t al = (uintptr_t)X | (uintptr_t)G;
    if (al & 15) return fail(RP_ERR_INVALID, "X and G must be 16-byte aligned");
    if (n == 0) return RP_OK;
    HIP_TRY(hipSetDevice(device));
    const unsigned m_tiles = (unsigned)((n + kDBM - 1) / kDBM), n_tiles = (unsigned)((p + kDBN - 1) / kDBN);
    const uint64_t blocks = (uint64_t)((m_tiles + 7) / 8) * 8ull * n_tiles;
    if (blocks >= (1ull << 31)) return fail(RP_ERR_UNSUPPORTED, "too many rows for one launch");
    hipStream_t st = (hipStream_t)stream;
    if (dtype == RP_BF16)
        hipLaunchKernelGGL(dense_nt_kernel<uint16_t>, dim3((unsigned)blocks), dim3(kDThreads), 0, st,
                           (const uint16_t*)X, (const uint16_t*)G, Y, n, (int)p, (int)m, ldy, m_tiles, n_tiles);
    else
        hipLaunchKernelGGL(dense_nt_kernel<float>, dim3((unsigned)blocks), dim3(kDThreads), 0, st, (const float*)X,
                           (const float*)G, Y, n, (int)p, (int)m, ldy, m_tiles, n_tiles);
    HIP_TRY(hipGetLastError());
    return RP_OK;
}
