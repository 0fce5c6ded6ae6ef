/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from the product
 * (randomprojection_amd/). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may use it, and only as the checker / the timed CPU baseline.
 *
 * Plain-C restatement of the arithmetic the reference's hot path bottoms out in:
 *   code/clustermode/randomProjection.py:46   projected_features = features_matrix.dot(local_csr_matrix)
 *   -> scipy/sparse/_base.py:481-497 (dot) -> _base.py:597-636 (_matmul_dispatch)
 *   -> scipy/sparse/_compressed.py:546-604 (_matmul_sparse)
 *   -> _sparsetools.csr_matmat_maxnnz (_compressed.py:569-574) and csr_matmat (:588-595).
 * scipy's C++ source (sparsetools/csr.h) is not in the container; the semantics restated here are
 * the ones pinned empirically in SURVEY.md §8(a) row a4 and re-pinned by tests/golden fixtures
 * generated with scipy 1.15.3 in this container (tests/golden/make_golden.py):
 *   - Gustavson/SMMP row by row; for each A entry jj in storage order, for each B entry kk of row
 *     Aj[jj] in storage order: sums[k] += Ax[jj] * Bx[kk]   (multiply rounded, then add rounded:
 *     this file is compiled with -ffp-contract=off),
 *   - first touch of k pushes it on a linked list (head insert); emission walks the list, so the
 *     output order of a row is REVERSE first-touch order,
 *   - an entry is emitted iff sums[k] != 0 (+0.0 and -0.0 dropped, NaN kept),
 *   - maxnnz counts distinct k per row before the zero drop (sizes the output).
 * Parity: pinned (tests/test_oracle.py compares against scipy-made golden vectors).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define DEFINE_SMMP(I, T, SFX)                                                                    \
int64_t oracle_maxnnz_##SFX(int64_t n_row, int64_t n_col, const I* Ap, const I* Aj,              \
                            const I* Bp, const I* Bj) {                                          \
    int64_t* mask = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_col > 0 ? n_col : 1));         \
    if (!mask) return -1;                                                                        \
    for (int64_t k = 0; k < n_col; ++k) mask[k] = -1;                                            \
    int64_t nnz = 0;                                                                             \
    for (int64_t i = 0; i < n_row; ++i) {                                                        \
        int64_t row_nnz = 0;                                                                     \
        for (I jj = Ap[i]; jj < Ap[i + 1]; ++jj) {                                               \
            I j = Aj[jj];                                                                        \
            for (I kk = Bp[j]; kk < Bp[j + 1]; ++kk) {                                           \
                I k = Bj[kk];                                                                    \
                if (mask[k] != i) { mask[k] = i; ++row_nnz; }                                    \
            }                                                                                    \
        }                                                                                        \
        nnz += row_nnz;                                                                          \
    }                                                                                            \
    free(mask);                                                                                  \
    return nnz;                                                                                  \
}                                                                                                \
/* Cp[0] is written; Cp[i+1] = running nnz. Returns total nnz, or -1 on allocation failure. */   \
int64_t oracle_matmat_##SFX(int64_t n_row, int64_t n_col, const I* Ap, const I* Aj, const T* Ax, \
                            const I* Bp, const I* Bj, const T* Bx, I* Cp, I* Cj, T* Cx) {        \
    I* next = (I*)malloc(sizeof(I) * (size_t)(n_col > 0 ? n_col : 1));                           \
    T* sums = (T*)malloc(sizeof(T) * (size_t)(n_col > 0 ? n_col : 1));                           \
    if (!next || !sums) { free(next); free(sums); return -1; }                                   \
    for (int64_t k = 0; k < n_col; ++k) { next[k] = -1; sums[k] = 0; }                           \
    int64_t nnz = 0;                                                                             \
    Cp[0] = 0;                                                                                   \
    for (int64_t i = 0; i < n_row; ++i) {                                                        \
        I head = -2;                                                                             \
        I length = 0;                                                                            \
        for (I jj = Ap[i]; jj < Ap[i + 1]; ++jj) {                                               \
            I j = Aj[jj];                                                                        \
            T v = Ax[jj];                                                                        \
            for (I kk = Bp[j]; kk < Bp[j + 1]; ++kk) {                                           \
                I k = Bj[kk];                                                                    \
                T prod = v * Bx[kk];                                                             \
                sums[k] = sums[k] + prod;                                                        \
                if (next[k] == -1) { next[k] = head; head = k; ++length; }                       \
            }                                                                                    \
        }                                                                                        \
        for (I jj = 0; jj < length; ++jj) {                                                      \
            if (sums[head] != 0) { Cj[nnz] = head; Cx[nnz] = sums[head]; ++nnz; }                \
            I temp = head;                                                                       \
            head = next[head];                                                                   \
            next[temp] = -1;                                                                     \
            sums[temp] = 0;                                                                      \
        }                                                                                        \
        Cp[i + 1] = (I)nnz;                                                                      \
    }                                                                                            \
    free(next); free(sums);                                                                      \
    return nnz;                                                                                  \
}

DEFINE_SMMP(int32_t, float, i32_f32)
DEFINE_SMMP(int32_t, double, i32_f64)
DEFINE_SMMP(int64_t, float, i64_f32)
DEFINE_SMMP(int64_t, double, i64_f64)

/*
 * CPU baseline driver (bench.py cpu_baseline leg, kind "port"): the scipy kernel pair
 * (maxnnz, then allocate, then matmat) run on `n_threads` threads over contiguous row blocks —
 * the analogue of SURVEY.md §8(d)(ii) "A_csr @ R_csr on N threads (GIL released)".
 * A is int32-indexed f32 (the recipe's formats). Returns total output nnz or -1.
 */
typedef struct {
    int64_t r0, r1, n_col;
    const int32_t *Ap, *Aj, *Bp, *Bj;
    const float *Ax, *Bx;
    int64_t nnz;
} oracle_job_t;

static void* oracle_job_run(void* arg) {
    oracle_job_t* jb = (oracle_job_t*)arg;
    int64_t n = jb->r1 - jb->r0;
    int32_t base = jb->Ap[jb->r0];
    int32_t* ap = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    if (!ap) { jb->nnz = -1; return NULL; }
    for (int64_t i = 0; i <= n; ++i) ap[i] = jb->Ap[jb->r0 + i] - base;
    const int32_t* aj = jb->Aj + base;
    const float* ax = jb->Ax + base;
    int64_t cap = oracle_maxnnz_i32_f32(n, jb->n_col, ap, aj, jb->Bp, jb->Bj);
    int32_t* cp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    int32_t* cj = (int32_t*)malloc(sizeof(int32_t) * (size_t)(cap > 0 ? cap : 1));
    float* cx = (float*)malloc(sizeof(float) * (size_t)(cap > 0 ? cap : 1));
    if (cap < 0 || !cp || !cj || !cx) { jb->nnz = -1; }
    else jb->nnz = oracle_matmat_i32_f32(n, jb->n_col, ap, aj, ax, jb->Bp, jb->Bj, jb->Bx, cp, cj, cx);
    free(ap); free(cp); free(cj); free(cx);
    return NULL;
}

int64_t oracle_project_mt_i32_f32(int64_t n_row, int64_t n_col, const int32_t* Ap, const int32_t* Aj,
                                  const float* Ax, const int32_t* Bp, const int32_t* Bj,
                                  const float* Bx, int n_threads) {
    if (n_threads < 1) n_threads = 1;
    oracle_job_t* jobs = (oracle_job_t*)calloc((size_t)n_threads, sizeof(oracle_job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -1; }
    for (int t = 0; t < n_threads; ++t) {
        jobs[t].r0 = n_row * t / n_threads;
        jobs[t].r1 = n_row * (t + 1) / n_threads;
        jobs[t].n_col = n_col;
        jobs[t].Ap = Ap; jobs[t].Aj = Aj; jobs[t].Ax = Ax;
        jobs[t].Bp = Bp; jobs[t].Bj = Bj; jobs[t].Bx = Bx;
        pthread_create(&th[t], NULL, oracle_job_run, &jobs[t]);
    }
    int64_t total = 0;
    for (int t = 0; t < n_threads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].nnz < 0) total = -1;
        else if (total >= 0) total += jobs[t].nnz;
    }
    free(jobs); free(th);
    return total;
}
