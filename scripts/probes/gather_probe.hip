// Diagnostic probe (not part of librp): random 2-byte gathers from a table of S bytes, to measure
// the request rate the memory side sustains vs table size (L2 / Infinity Cache / HBM), optionally
// beside a streaming read of a large buffer (the A stream of the SpGEMM).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

template <int K>
__global__ void gather(const uint16_t* __restrict__ t, uint32_t n, uint32_t iters, uint32_t* out,
                       const uint4* __restrict__ stream, uint64_t stream_n) {
    uint32_t acc = 0;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = hash32(gid * 2654435761u + 12345u);
    uint64_t sp = gid;
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t idx[K];
#pragma unroll
        for (int k = 0; k < K; ++k) { h = hash32(h + k); idx[k] = (uint32_t)(((uint64_t)h * n) >> 32); }
        uint32_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = t[idx[k]];
#pragma unroll
        for (int k = 0; k < K; ++k) acc += v[k];
        if (stream_n) {
            uint4 s = stream[sp % stream_n];
            acc += s.x;
            sp += (uint64_t)gridDim.x * blockDim.x;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const int grid = 256 * 16, block = 256;
    const uint32_t iters = 64;
    uint16_t* t; uint32_t* out; uint4* stream;
    const size_t max_bytes = (size_t)2 << 30;
    hipMalloc(&t, max_bytes); hipMemset(t, 1, max_bytes);
    hipMalloc(&out, 64);
    const size_t sbytes = (size_t)8 << 30;
    hipMalloc(&stream, sbytes); hipMemset(stream, 2, sbytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const size_t sizes_mb[] = {2, 8, 32, 64, 109, 160, 220, 300, 512, 2048};
    printf("{\"probe\":\"random u16 gathers\",\"threads\":%d,\"gathers_per_thread\":%u,\"results\":[\n", grid * block, iters * 8);
    bool first = true;
    for (int with_stream = 0; with_stream < 2; ++with_stream)
        for (size_t mb : sizes_mb) {
            const uint32_t n = (uint32_t)((mb << 20) / 2);
            const uint64_t sn = with_stream ? sbytes / 16 : 0;
            hipLaunchKernelGGL(gather<8>, grid, block, 0, 0, t, n, iters, out, stream, sn);
            hipEventRecord(e0);
            const int reps = 5;
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(gather<8>, grid, block, 0, 0, t, n, iters, out, stream, sn);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); ms /= reps;
            const double reqs = (double)grid * block * iters * 8;
            const double sgb = with_stream ? (double)grid * block * iters * 16 / 1e9 : 0;
            printf("%s {\"table_MB\":%zu,\"stream\":%d,\"ms\":%.3f,\"Greq_per_s\":%.2f,\"stream_GBps\":%.1f}\n",
                   first ? "" : ",", mb, with_stream, ms, reqs / ms / 1e6, sgb / ms * 1e3);
            first = false;
        }
    printf("]}\n");
    return 0;
}
