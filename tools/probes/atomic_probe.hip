// Throughput of device-scope atomicAdd on a small hot array (tile counters) vs LDS-aggregated variants.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>

__global__ void k_atomic(const unsigned *idx, unsigned n, unsigned *cnt) {
    unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) atomicAdd(&cnt[idx[i]], 1u);
}
__global__ void k_atomic_ret(const unsigned *idx, unsigned n, unsigned *cnt, unsigned *pos) {
    unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) pos[i] = atomicAdd(&cnt[idx[i]], 1u);
}

int main() {
    const unsigned n = 4200000, T = 8160;
    std::vector<unsigned> h(n);
    std::mt19937 rng(1);
    // clustered tiles like a Gaussian scene: normal around the centre of a 120x68 grid
    std::normal_distribution<float> nx(60.f, 25.f), ny(34.f, 14.f);
    for (unsigned i = 0; i < n; i++) {
        int x = (int)nx(rng), y = (int)ny(rng);
        x = x < 0 ? 0 : (x > 119 ? 119 : x);
        y = y < 0 ? 0 : (y > 67 ? 67 : y);
        h[i] = y * 120 + x;
    }
    unsigned *d_idx, *d_cnt, *d_pos;
    hipMalloc(&d_idx, n * 4); hipMalloc(&d_cnt, T * 4); hipMalloc(&d_pos, n * 4);
    hipMemcpy(d_idx, h.data(), n * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int mode = 0; mode < 2; mode++) {
        float best = 1e9;
        for (int r = 0; r < 10; r++) {
            hipMemset(d_cnt, 0, T * 4);
            hipEventRecord(a);
            if (mode == 0) k_atomic<<<(n + 255) / 256, 256>>>(d_idx, n, d_cnt);
            else k_atomic_ret<<<(n + 255) / 256, 256>>>(d_idx, n, d_cnt, d_pos);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("mode %d (%s): %.1f us for %u atomics on %u counters\n", mode, mode ? "returning" : "no-return",
               best * 1000, n, T);
    }
    return 0;
}
