// Diagnostic probe 3 (not part of librp): random gathers from tables allocated with different HIP
// memory flavours (default coarse-grained, uncached, fine-grained) -- does any of them fetch less
// than a 128-B line per random miss and so sustain more random requests per second?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

__global__ void gather(const uint64_t* __restrict__ t, uint32_t n, uint32_t iters, uint32_t* out) {
    uint32_t acc = 0;
    uint32_t h = hash32((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u + 777u);
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t idx[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { h = hash32(h + k); idx[k] = (uint32_t)(((uint64_t)h * n) >> 32); }
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = t[idx[k]];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += (uint32_t)v[k];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = (size_t)512 << 20;
    uint32_t* out;
    hipMalloc(&out, 64);
    struct { const char* name; unsigned flag; int kind; } kinds[] = {
        {"default", 0, 0}, {"uncached", hipDeviceMallocUncached, 1}, {"finegrained", hipDeviceMallocFinegrained, 1}};
    printf("[\n");
    bool first = true;
    for (auto& k : kinds) {
        void* t = nullptr;
        hipError_t e = k.kind == 0 ? hipMalloc(&t, bytes) : hipExtMallocWithFlags(&t, bytes, k.flag);
        if (e != hipSuccess) { printf("%s {\"alloc\":\"%s\",\"error\":\"%s\"}\n", first ? "" : ",", k.name, hipGetErrorString(e)); first = false; continue; }
        hipMemset(t, 1, bytes);
        const int grid = 256 * 16, block = 256;
        const uint32_t iters = 32, n = (uint32_t)(bytes / 8);
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipLaunchKernelGGL(gather, grid, block, 0, 0, (const uint64_t*)t, n, iters, out);
        hipEventRecord(e0);
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(gather, grid, block, 0, 0, (const uint64_t*)t, n, iters, out);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
        printf("%s {\"alloc\":\"%s\",\"ms\":%.3f,\"Greq_per_s\":%.2f}\n", first ? "" : ",", k.name, ms,
               (double)grid * block * iters * 8 / ms / 1e6);
        first = false;
        hipFree(t);
    }
    printf("]\n");
    return 0;
}
