// Diagnostic probe 2 (not part of librp): random gathers by load flavour and width, to see whether
// any load form raises the random-request rate (smaller fabric requests, different L2 policy).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

template <int MODE, typename W>
__global__ void gather(const W* __restrict__ t, uint32_t n, uint32_t iters, uint32_t* out) {
    uint32_t acc = 0;
    uint32_t h = hash32((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u + 777u);
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t idx[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { h = hash32(h + k); idx[k] = (uint32_t)(((uint64_t)h * n) >> 32); }
        W v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (MODE == 0) v[k] = t[idx[k]];
            else if (MODE == 1) v[k] = __builtin_nontemporal_load(&t[idx[k]]);
            else v[k] = __hip_atomic_load(&t[idx[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += (uint32_t)v[k];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int MODE, typename W>
void run(const char* name, void* t, size_t table_bytes, uint32_t* out, bool& first) {
    const int grid = 256 * 16, block = 256;
    const uint32_t iters = 64;
    const uint32_t n = (uint32_t)(table_bytes / sizeof(W));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((gather<MODE, W>), grid, block, 0, 0, (const W*)t, n, iters, out);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((gather<MODE, W>), grid, block, 0, 0, (const W*)t, n, iters, out);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    printf("%s {\"mode\":\"%s\",\"width\":%zu,\"table_MB\":%zu,\"ms\":%.3f,\"Greq_per_s\":%.2f}\n", first ? "" : ",", name,
           sizeof(W), table_bytes >> 20, ms, (double)grid * block * iters * 8 / ms / 1e6);
    first = false;
}

int main() {
    void* t; uint32_t* out;
    const size_t bytes = (size_t)512 << 20;
    hipMalloc(&t, bytes); hipMemset(t, 1, bytes); hipMalloc(&out, 64);
    bool first = true;
    printf("[\n");
    for (size_t mb : {(size_t)128, (size_t)512}) {
        const size_t b = mb << 20;
        run<0, uint16_t>("plain", t, b, out, first);
        run<1, uint16_t>("nontemporal", t, b, out, first);
        run<0, uint64_t>("plain", t, b, out, first);
        run<1, uint64_t>("nontemporal", t, b, out, first);
        run<2, uint64_t>("atomic_agent", t, b, out, first);
        
    }
    printf("]\n");
    return 0;
}
