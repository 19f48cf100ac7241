// Cost of the bucket scatter's store pattern: 4.2M 8-B keys written to random slots of a 34 MB array
// (each slot exactly once) vs coalesced, and 4-B variants.  Indices are a host-made permutation, so every
// store is in bounds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <numeric>
#include <algorithm>

__global__ void k_scatter8(const unsigned *perm, unsigned n, unsigned long long *out) {
    unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[perm[i]] = ((unsigned long long)i << 32) | i;
}
__global__ void k_scatter4(const unsigned *perm, unsigned n, unsigned *out) {
    unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[perm[i]] = i;
}
__global__ void k_linear8(const unsigned *perm, unsigned n, unsigned long long *out) {
    unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = ((unsigned long long)perm[i] << 32) | i;
}
__global__ void k_gather8(const unsigned *perm, unsigned n, const unsigned long long *in, unsigned long long *out) {
    unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[perm[i]];
}

int main() {
    const unsigned n = 4200000;
    std::vector<unsigned> h(n);
    std::iota(h.begin(), h.end(), 0u);
    std::mt19937 rng(1);
    std::shuffle(h.begin(), h.end(), rng);
    // "bucketed" permutation: slots grouped in runs of 2 consecutive indices (the walk's ~2 instances per
    // (block, tile) run)
    std::vector<unsigned> h2(n);
    {
        std::vector<unsigned> runs(n / 2);
        std::iota(runs.begin(), runs.end(), 0u);
        std::shuffle(runs.begin(), runs.end(), rng);
        for (unsigned r = 0; r < n / 2; r++) { h2[2 * r] = 2 * runs[r]; h2[2 * r + 1] = 2 * runs[r] + 1; }
    }
    unsigned *d_perm, *d_perm2, *d_o4;
    unsigned long long *d_o8, *d_i8;
    hipMalloc(&d_perm, n * 4); hipMalloc(&d_perm2, n * 4); hipMalloc(&d_o4, n * 4);
    hipMalloc(&d_o8, n * 8); hipMalloc(&d_i8, n * 8);
    hipMemcpy(d_perm, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_perm2, h2.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(d_i8, 0, n * 8);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const unsigned g = (n + 255) / 256;
    auto time = [&](const char *name, auto fn) {
        for (int w = 0; w < 3; w++) fn();
        hipEventRecord(a);
        for (int r = 0; r < 20; r++) fn();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("%-28s %8.1f us\n", name, ms * 1000 / 20);
    };
    time("linear 8B", [&] { k_linear8<<<g, 256>>>(d_perm, n, d_o8); });
    time("scatter 8B random", [&] { k_scatter8<<<g, 256>>>(d_perm, n, d_o8); });
    time("scatter 8B runs of 2", [&] { k_scatter8<<<g, 256>>>(d_perm2, n, d_o8); });
    time("scatter 4B random", [&] { k_scatter4<<<g, 256>>>(d_perm, n, d_o4); });
    time("gather 8B random", [&] { k_gather8<<<g, 256>>>(d_perm, n, d_i8, d_o8); });
    return 0;
}
