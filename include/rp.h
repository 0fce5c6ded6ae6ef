/*
 * rp.h — C-ABI of librp.so, the MI355X-native projection step `X_partition @ R` of
 * afcarl/RandomProjection. Plain pointers and sizes only; no exceptions cross the ABI; every
 * entry point returns an rp_status (0 = RP_OK) and rp_last_error() describes the last failure on
 * the calling thread.
 *
 * What each entry point replaces in the reference (paths relative to /root/reference):
 *
 *  rp_projector_create / _create_from_device / _export
 *      R = srp.components_.T.astype(np.float32)          code/clustermode/randomProjection.py:101
 *      sc.broadcast(R)                                   code/clustermode/randomProjection.py:104
 *      (closure capture in localmode)                    code/localmode/randomProjection.py:127,130
 *      other = self.__class__(other)  # CSC->CSR per call  scipy/sparse/_compressed.py:564
 *    R is uploaded once, in a single-magnitude packed layout when it qualifies (every sklearn SRP
 *    matrix does), and stays resident in HBM; _export/_create_from_device let a driver ship the
 *    device image to other GPUs over RCCL (one broadcast) instead of re-packing.
 *
 *  rp_project_device
 *      projected_features = features_matrix.dot(local_csr_matrix)
 *                                                        code/clustermode/randomProjection.py:46
 *      -> scipy _sparsetools.csr_matmat_maxnnz + csr_matmat  scipy/sparse/_compressed.py:569-595
 *    Device-resident CSR in, device-resident CSR out, asynchronous on one stream (when the caller
 *    asks for the nnz, the host also reads a 4-byte verdict of a sampling kernel first). The call runs one of the
 *    kernel pipelines rp_project_plan reports: the row-lane pipeline for short rows over a packed R
 *    (KDD2012: staging choice, then either segment reserves, super-tile partition, bitmap-filtered
 *    gather and the wave kernel, or the direct main kernel; heavy-tile count/write, scan, copy), or
 *    the tile pipeline for long rows / generic R (one look-back kernel + a copy of deferred tiles).
 *    Output equals scipy's bit for bit: same per-row order
 *    (RP_ORDER_SCIPY = reverse first-touch) or ascending (RP_ORDER_SORTED = what pyspark's
 *    SparseVector makes of it, code/clustermode/randomProjection.py:49-50), same zero drop, values
 *    computed with the same separately rounded multiply and add.
 *
 *  rp_project_host_begin / rp_result_fetch / rp_result_free
 *      the same product for host buffers, shaped like scipy's two calls: begin computes C on the
 *      GPU and reports its exact nnz (the role of csr_matmat_maxnnz: size the output), the caller
 *      allocates, fetch fills (the role of csr_matmat). Used by the Python drop-ins
 *      random_project_mappartitions_function (clustermode/randomProjection.py:15-54),
 *      random_project_map_function (localmode/randomProjection.py:15-36) and
 *      SparseRandomProjection.transform (sklearn/random_projection.py:801-824).
 *
 *  rp_project
 *      the same as begin + allocation + fetch in one call (the caller allocates in a callback).
 *
 *  rp_project_stream
 *      the same product for a host matrix of any size, cut into chunks of rows (the recipe's
 *      partitions, code/clustermode/randomProjection.py:107-110, each projected by the partition
 *      function, :28-54) whose upload, projection and download overlap; results go straight into
 *      caller host arrays at their final CSR positions (BASELINE configs[1]: chunked row streaming).
 *
 *  rp_libsvm_parse_device
 *      spark.read.format("libsvm").load(path, numFeatures=m)  code/clustermode/randomProjection.py:71
 *    libsvm text -> CSR on the GPU (Spark MLUtils.parseLibSVMRecord semantics).
 *
 *  rp_synth_rows_device
 *      synthetic KDD2012-shaped rows generated in HBM (benchmarks; the reference downloads
 *      kdd12.tr with code/get_kdd2012_data.sh, not available offline).
 */
#ifndef RP_H
#define RP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    RP_OK = 0,
    RP_ERR_INVALID = 1,      /* bad argument (shape mismatch, bad dtype code, NULL pointer) */
    RP_ERR_HIP = 2,          /* a HIP runtime call failed (no device, launch failure, ...) */
    RP_ERR_CAPACITY = 3,     /* rp_project_device: out->capacity < exact nnz (nnz reported) */
    RP_ERR_UNSUPPORTED = 4,  /* shape outside what the GPU path supports (see rp_last_error) */
    RP_ERR_NOMEM = 5,
    RP_ERR_TIMEOUT = 6       /* a device-side bounded wait expired (should never happen) */
} rp_status;

typedef enum { RP_I32 = 1, RP_I64 = 2, RP_F32 = 3, RP_F64 = 4, RP_BF16 = 5 } rp_dtype;

typedef enum {
    RP_LAYOUT_AUTO = 0,      /* packed when R has one magnitude and p <= 16384, else generic */
    RP_LAYOUT_GENERIC = 1,   /* CSR (int32 indptr, uint16 columns, values) */
    RP_LAYOUT_PACKED = 2     /* require the packed layout; RP_ERR_UNSUPPORTED if R does not fit */
} rp_layout;

typedef enum { RP_ORDER_SCIPY = 0, RP_ORDER_SORTED = 1 } rp_order;

typedef struct rp_projector rp_projector;
typedef struct rp_result rp_result;

/* Static description of a resident R (for logging and for shipping the device image). */
typedef struct {
    int64_t m;               /* rows of R = input features */
    int64_t p;               /* columns of R = output components */
    int64_t nnz;
    int32_t layout;          /* RP_LAYOUT_GENERIC or RP_LAYOUT_PACKED */
    int32_t value_type;      /* RP_F32 / RP_F64: dtype R was given in */
    double magnitude;        /* packed: |value| of every entry; generic: 0 */
    int32_t block_shift;     /* reserved (0) */
    int32_t n_buffers;       /* device buffers making up the image (<= 4) */
    int64_t buffer_bytes[4]; /* packed: W (u64[m]), long-row records (u16), -; generic: Bp, Bj, Bx */
} rp_projector_info;

/* A CSR operand. Host or device memory depending on the call. */
typedef struct {
    int64_t n_rows;
    const void* indptr;      /* n_rows + 1 entries, RP_I32 or RP_I64, indptr[0] may be != 0 */
    int32_t indptr_type;
    const int32_t* indices;  /* int32 feature ids in [0, m) */
    const void* data;        /* RP_F32 or RP_F64 = the compute type (scipy upcast of A and R) */
    int32_t data_type;
    int64_t nnz;             /* indptr[n_rows] - indptr[0] if known (sizes tiles), else -1: the
                                device call then reads it back (one small synchronous copy) */
} rp_csr_in;

/* Device output of rp_project_device (caller-owned device memory). */
typedef struct {
    void* indptr;            /* n_rows + 1 entries */
    int32_t indptr_type;     /* RP_I32 or RP_I64 */
    void* indices;           /* capacity entries */
    int32_t indices_type;    /* RP_I32 or RP_I64 */
    void* data;              /* capacity entries of the compute type */
    int64_t capacity;
} rp_csr_out;

/* Version of this header's signatures. Bumped whenever an exported function's arguments change
 * (6: rp_dense_project_device gained `variant`; rp_project_stream_stats added); bindings compare
 * rp_abi_version() with the value they were written against and refuse a mismatch, since a changed
 * signature under the same symbol name cannot be detected otherwise. */
#define RP_ABI_VERSION 6

const char* rp_last_error(void);
const char* rp_version(void);
int rp_abi_version(void);
/* sha256 prefix (16 hex digits) of the sources the library was built from (build.py); loaders
 * compare it with the sources on disk and refuse a stale binary. No reference counterpart. */
const char* rp_build_id(void);
int rp_device_count(int* count);

int rp_projector_create(int device, int64_t m, int64_t p,
                        const void* indptr, int32_t indptr_type,
                        const void* indices, int32_t indices_type,
                        const void* data, int32_t data_type,
                        int32_t layout, rp_projector** out);
int rp_projector_info_get(const rp_projector* h, rp_projector_info* out);
/* copy device buffer `which` (< info.n_buffers) of the image into caller device memory dst */
int rp_projector_export(const rp_projector* h, int32_t which, void* dst_device, void* stream);
/* build a projector on `device` from an image already in device memory (e.g. after an RCCL
 * broadcast); the buffers are copied, the caller keeps ownership of `buffers` */
int rp_projector_create_from_device(int device, const rp_projector_info* info,
                                    const void* const* buffers, rp_projector** out);
int rp_projector_destroy(rp_projector* h);

/* Host-only (no GPU): build the device image of R that rp_projector_create would upload.
 * Call with buf0..2 == NULL to get the layout and buffer sizes in *info, then again with caller
 * buffers of info->buffer_bytes[i] bytes to receive W/base/records (packed) or Bp/Bj/values
 * (generic). Lets a driver pack once and lets tests check the layout without a device. */
int rp_pack_r_host(int64_t m, int64_t p, const void* indptr, int32_t indptr_type,
                   const void* indices, int32_t indices_type, const void* data, int32_t data_type,
                   int32_t layout, rp_projector_info* info, void* buf0, void* buf1, void* buf2);

/* Workspace bytes rp_project_device needs for n_rows rows holding nnz_a entries: look-back tile
 * states + counters, plus the staged-gather buffers (about 8 bytes per A entry) when the launch
 * would stage. nnz_a < 0 (unknown): the small look-back part for the worst-case tiling only. */
int64_t rp_project_workspace_bytes(const rp_projector* h, int64_t n_rows, int64_t nnz_a);
/* The same for a known compute type (RP_F32 / RP_F64): the value-sized parts (deferred-output pool,
 * row-lane slots) sized for it rather than for float64 (configs[3] at 200M rows: 40 GB, not 66). */
int64_t rp_project_workspace_bytes_for(const rp_projector* h, int64_t n_rows, int64_t nnz_a, int32_t data_type);

/* Staged gather (packed R, m < 2^30): the A entries of each tile are bucketed by feature range and
 * R's descriptors fetched bucket by bucket from an L2-resident slice (one partition pass over A
 * into per-bucket segments with reserves, then one gather, instead of one random 128-B line fill
 * per A entry). mode: -1 auto (large launches over a large R; the device then stages only inputs
 * whose sampled feature ids are near uniform), 0 off, 1 on (the row-lane pipeline still goes
 * direct for the rest of a call whose columns overflow a segment's reserve: far from uniform);
 * bucket_shift: 2^shift features per bucket (0 = auto, 19). Results are identical either way. */
int rp_projector_set_staging(rp_projector* h, int32_t mode, int32_t bucket_shift);

/* Per-projector tuning and test options (the library reads no environment variables). Results are
 * identical under every setting; only the schedule changes. value < default sentinel restores the
 * default.
 *   RP_OPT_PIPELINE      0 auto (default); 1 tile pipeline; 2 row-lane pipeline where it can run
 *   RP_OPT_DEFER_POLLS   tile pipeline: -1 no tile slots (every tile waits for its prefix from a
 *                        decoupled look-back, then writes C itself); any other value (default -2):
 *                        every tile writes its own slot, a scan + copy place the slots (round 6;
 *                        the round-5 look-back deferral it replaced cost configs[3] 65 of 198 ms)
 *   RP_OPT_DEFER_TICKS   accepted and ignored since round 6 (kept for the ABI)
 *   RP_OPT_CHUNK_ROWS    row-lane rows per launch sequence: 0 default (2^27), else rounded up to
 *                        whole 256-row tiles
 *   RP_OPT_HOST_THREADS  helper threads of the host result download: -1 default (min(4, cores));
 *                        0 or 1 plain copies
 * (Options 6 and 7 — the persistent row-lane kernel and the filtered tile pipeline, both measured
 * slower than the defaults — were removed in round 5 and are rejected as unknown.) */
typedef enum {
    RP_OPT_PIPELINE = 1,
    RP_OPT_DEFER_POLLS = 2,
    RP_OPT_DEFER_TICKS = 3,
    RP_OPT_CHUNK_ROWS = 4,
    RP_OPT_HOST_THREADS = 5
} rp_option;
int rp_projector_set_option(rp_projector* h, int32_t option, int64_t value);
int rp_projector_get_option(const rp_projector* h, int32_t option, int64_t* value);

/* The kernel pipeline rp_project_device would run for n_rows rows holding nnz_a entries with the
 * full workspace: *pipeline = RP_PIPE_TILE (one-launch tile SpGEMM with look-back) or
 * RP_PIPE_ROWLANE (row-lane kernel: short rows over a packed R), *staged = 1 if the R descriptors
 * are fetched by the staged gather, 0 if gathered directly, 2 if the device decides per call (auto
 * mode, rp_project_choice), *bucket_shift the staged bucket width (log2 features). Any out
 * pointer may be NULL. For logging and benchmarks; results are identical on every pipeline. */
typedef enum { RP_PIPE_TILE = 0, RP_PIPE_ROWLANE = 1 } rp_pipeline;
int rp_project_plan(const rp_projector* h, int64_t n_rows, int64_t nnz_a, int32_t* pipeline, int32_t* staged,
                    int32_t* bucket_shift);

/* After an rp_project_device call with `workspace` has completed (its stream synchronised by the
 * caller): *staged = 1 if that call used the staged gather, 0 if direct gathers (rp_project_plan's
 * *staged == 2: decided per call from a sample of the input's feature ids taken on the device; and
 * a staged row-lane call whose columns overflowed a segment's reserve finishes direct and reads 0).
 * The call records what actually ran in the workspace header, so a re-planned call (a workspace
 * too small for staging) reads 0. n_rows / nnz_a are unused (kept for the ABI). 4-byte copy. */
int rp_project_choice(const rp_projector* h, int64_t n_rows, int64_t nnz_a, const void* workspace,
                      int32_t* staged);

/* C = A @ R, all device memory, enqueued on `stream` (hipStream_t, NULL = default).
 * workspace: caller device memory of workspace_bytes (>= rp_project_workspace_bytes(h, n, -1);
 * the full rp_project_workspace_bytes(h, n, nnz) also enables deferred tile output (no tile
 * waits on its predecessors) and staging), or NULL to use the projector's own (then calls on one
 * projector must not run concurrently on different streams).
 * total_nnz: if non-NULL the call synchronizes the stream and stores the exact output nnz;
 * RP_ERR_CAPACITY is returned when it exceeds out->capacity (indptr is still complete). In auto
 * staging mode it also reads the sampling kernel's 4-byte verdict on the host and launches only the
 * chosen branch (the staged kernels, or the direct main kernel for far-from-uniform columns).
 * If NULL (with a caller workspace and a->nnz >= 0) the call never waits on the host (timing
 * loops, graph capture): the verdict stays on the device and gates the staged kernels (same bits;
 * the direct case then gathers inside the wave kernel, slower than the host-chosen branch on
 * power-law columns). Under stream capture those three conditions are required (RP_ERR_INVALID). */
int rp_project_device(rp_projector* h, const rp_csr_in* a, const rp_csr_out* c, int32_t order,
                      void* workspace, int64_t workspace_bytes, void* stream, int64_t* total_nnz);

/* Host CSR in -> GPU -> exact nnz. The result stays on the device until fetched. */
int rp_project_host_begin(rp_projector* h, const rp_csr_in* a_host, int32_t order,
                          rp_result** out, int64_t* nnz);
/* Copy into caller host arrays: indptr (n_rows + 1) of indptr_type, indices (nnz) of
 * indices_type, data (nnz) of the compute type. */
int rp_result_fetch(rp_result* r, void* indptr, int32_t indptr_type, void* indices,
                    int32_t indices_type, void* data);
int rp_result_free(rp_result* r);

/* Fused convenience form of begin + fetch: computes C = A @ R for host A, then asks the caller to
 * allocate the output through `alloc` (called once, with the exact n_rows and nnz; it returns 0 and
 * sets host pointers of n_rows + 1 indptr entries and nnz indices/data entries, with their index
 * types, or non-zero to abort with RP_ERR_NOMEM) and fills it. The data type is A's compute type. */
typedef int (*rp_alloc_fn)(void* user, int64_t n_rows, int64_t nnz, void** indptr, int32_t* indptr_type,
                           void** indices, int32_t* indices_type, void** data);
int rp_project(rp_projector* h, const rp_csr_in* a_host, int32_t order, rp_alloc_fn alloc, void* user);

/* Chunked host streaming (boundary 2): C = A @ R for host CSR A of any size into caller host
 * arrays c_host (indptr: n_rows + 1 entries of indptr_type; indices/data: capacity entries; data in
 * the compute type). Rows go in chunks of chunk_rows (0 = 2M): chunk k+1's upload, chunk k's
 * kernels and chunk k-1's download overlap (an upload thread, a download thread, a compute
 * stream; device output offsets chained on the device). Host arrays may be pageable or pinned
 * (rp_host_alloc: the copies then run without blocking their threads); pageable destinations
 * should already be faulted in (first-touch faults cost more than the copy). *total_nnz = exact
 * nnz; RP_ERR_CAPACITY if it exceeds c_host->capacity (indptr complete, the entries that fit
 * written) or an RP_I32 indptr cannot hold it. Input indptr monotonicity and column range are
 * checked on the device (RP_ERR_INVALID). Serialised per projector. */
int rp_project_stream(rp_projector* h, const rp_csr_in* a_host, int32_t order, int64_t chunk_rows,
                      const rp_csr_out* c_host, int64_t* total_nnz);
/* What the last rp_project_stream / rp_libsvm_project_stream call on this projector did: *chunks
 * = chunks streamed; *recomputed = chunks whose output outgrew their device slot and were projected
 * again alone after the pipeline drained (0 in the steady state: slot capacities follow the
 * measured output per entry of the chunks already downloaded); *regrown = slot capacities raised
 * from that measurement. Any out pointer may be NULL. No reference counterpart (diagnostics). */
int rp_project_stream_stats(rp_projector* h, int64_t* chunks, int64_t* recomputed, int64_t* regrown);
/* Page-locked host memory (hipHostMalloc) / its release. */
int rp_host_alloc(int64_t bytes, void** out);
int rp_host_free(void* p);

/* Synthetic rows on the device: per-row nnz = 1 + Poisson(mean_extra), or exactly -mean_extra
 * when mean_extra < 0 (capped at max_row_nnz),
 * distinct ascending columns in [0, m) — uniform (dist 0) or power-law Zipf(s) over a fixed
 * permutation without replacement (dist 1) — values 1.0f. Two calls: first with indices == NULL
 * to fill indptr (int32 or int64) and get the nnz, then with indices/data of that size. */
int rp_synth_rows_device(int device, int64_t n_rows, int64_t m, double mean_extra,
                         int32_t max_row_nnz, int32_t dist, double zipf_s, uint64_t seed,
                         void* indptr, int32_t indptr_type, int32_t* indices, float* data,
                         void* stream, int64_t* nnz);

/* libsvm text -> CSR, both in device memory (replaces spark.read.format("libsvm").load(path,
 * numFeatures=m), code/clustermode/randomProjection.py:71; Spark MLUtils.parseLibSVMRecord):
 * lines trimmed, blank and '#' lines skipped, "label i:v i:v ..." split on single spaces,
 * i 1-based -> 0-based, strictly ascending and < num_features, v parsed as double and stored as
 * float32 (the partition function's astype(np.float32), clustermode:38), label kept as double.
 * `text` must be 16-byte aligned. With indices == NULL only *n_rows and *nnz are computed;
 * otherwise labels (cap_rows), indptr (cap_rows + 1), indices/data (cap_nnz) are filled.
 * A malformed line gives RP_ERR_INVALID and *err_line = its 0-based line number. */
int rp_libsvm_parse_device(int device, const char* text, int64_t n_bytes, int64_t num_features,
                           double* labels, void* indptr, int32_t indptr_type, int32_t* indices,
                           float* data, int64_t cap_rows, int64_t cap_nnz, void* stream,
                           int64_t* n_rows, int64_t* nnz, int64_t* err_line);

/* Boundary 3, chunked: libsvm text in host memory -> GPU parse -> projection -> host CSR.
 * Replaces spark.read.format("libsvm").load(...) followed by the partition function's projection
 * (code/clustermode/randomProjection.py:71-72 then :46 inside mapPartitions, :107-110). The text is
 * cut into chunks of whole lines of about chunk_bytes (0 = 64 MB, a Spark text partition); chunk
 * k+1's upload, chunk k's parse + projection and chunk k-1's download overlap (an upload thread, a
 * compute stream, a download thread). Parsing follows rp_libsvm_parse_device (float32 values, so R
 * must be float32: the recipe's astype). Outputs: labels[cap_rows] (f64), c_host = the projected CSR
 * (indptr cap_rows + 1 entries, indices/data capacity entries, data float32), *n_rows, *total_nnz.
 * RP_ERR_CAPACITY when rows exceed cap_rows or entries exceed capacity (then *n_rows / *total_nnz
 * report what was needed as far as known); RP_ERR_INVALID with *err_line = 0-based line of the file
 * for a malformed line. Host arrays may be pinned (rp_host_alloc) or pageable. */
int rp_libsvm_project_stream(rp_projector* h, const char* text, int64_t n_bytes, int32_t order, int64_t chunk_bytes,
                             double* labels, int64_t cap_rows, const rp_csr_out* c_host, int64_t* n_rows,
                             int64_t* total_nnz, int64_t* err_line);

/* Synthetic libsvm text on the device (benchmarks of boundary 3): row i of a device CSR (int64
 * indptr, int32 indices) as "<0|1> <j+1>:<value> ..." with decimal values of 6-17 significant
 * digits. line_offsets: device int64[n_rows + 1], filled with each line's start (and the total).
 * With text == NULL only *n_bytes is computed; then text (cap_bytes, device) is written. */
int rp_synth_libsvm_device(int device, int64_t n_rows, const int64_t* indptr, const int32_t* indices, uint64_t seed,
                           int64_t* line_offsets, char* text, int64_t cap_bytes, void* stream, int64_t* n_bytes);

/* Dense Gaussian projection (BASELINE configs[4]): Y[n x p] (row stride ldy) = X[n x m] . G[p x m]^T
 * for device arrays X and G of dtype RP_BF16 (bf16 operands, f32 accumulate, Y f32), RP_F32 (exact-f32
 * MFMA products, f32 accumulate, Y f32) or RP_F64 (f64 MFMA, Y f64), both row-major, 16-byte aligned,
 * m a multiple of 64 (bf16) / 32 (f32) / 16 (f64). Replaces sklearn GaussianRandomProjection.transform's
 * X @ components_.T (sklearn/random_projection.py:569-612), computed in X's dtype as sklearn does,
 * with hand-written MFMA GEMMs. Asynchronous on `stream`. variant: -1 = the default kernel; 0..11 pick
 * another measured tile variant for this call only (A/B measurements; rp_dense.hip lists them). */
int rp_dense_project_device(int device, const void* X, int32_t dtype, int64_t n, int64_t m, const void* G,
                            int64_t p, void* Y, int64_t ldy, void* stream, int32_t variant);

#ifdef __cplusplus
}
#endif

#endif /* RP_H */
