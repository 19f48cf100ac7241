// FETCH_SIZE / WRITE_SIZE calibration for the rasterizer's access patterns.
//
// MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE only for wide coalesced streaming reads (it reports half of their
// bytes).  The composite passes, the expansion and the bucket scatter instead gather 4-B words and 48-B records from
// random places, and scatter 4-/8-B words.  Each kernel below reads or writes a KNOWN number of bytes and distinct
// 128-B lines, all from a 2 GiB table (far beyond the 256 MiB Infinity Cache), each line touched at most once per
// launch.  Run under `rocprofv3 --pmc FETCH_SIZE` (and a separate `--pmc WRITE_SIZE` pass); tools/pmc_gather_calib.py
// divides the counted bytes by the known ones per pattern.  Timing (hipEvents) is printed as a cross-check: a pattern
// whose counter undercounts shows up as a byte rate above what the same lines cost in the streaming kernel.
//
//   stream16      coalesced 16 B per lane, every byte of the table read once                  (known: bytes)
//   line_full     random 128-B lines, 8 lanes x 16 B cover a line (full line used)             (known: lines x 128)
//   gather4       one 4-B word per random line                                                 (known: lines)
//   gather16      one 16-B word per random line                                                (known: lines)
//   rec48         one 48-B record (3 x 16 B) per lane, random records of a 48-B-record table  (known: records)
//   scatter4/8    one 4-/8-B store per random line                                             (WRITE_SIZE pass)
//   runs8x2       8-B stores in runs of 2 consecutive slots, runs at random (the bucket scatter's ~2 per tile)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr size_t TABLE = 2ull << 30;  // 2 GiB
constexpr unsigned LINES = TABLE / 128;  // 2^24 lines
constexpr unsigned N = 4u << 20;  // gathers per launch (4 Mi: the cfg 3 instance count)

// a bijection on [0, 2^24) (odd multiplier mod 2^24), so every launch touches N distinct lines, scattered
__device__ __forceinline__ unsigned line_of(unsigned i) { return (i * 2654435761u) & (LINES - 1); }

__global__ void stream16(const float4 *__restrict__ t, size_t n4, float *__restrict__ sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 v = t[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 123.f) sink[0] = acc;
}
__global__ void line_full(const float4 *__restrict__ t, float *__restrict__ sink, unsigned salt) {
    const unsigned g = blockIdx.x * 256 + threadIdx.x;  // 8 lanes per line
    const unsigned l = line_of((g >> 3) + salt);
    const float4 v = t[(size_t)l * 8 + (g & 7)];
    if (v.x + v.y + v.z + v.w == 123.f) sink[0] = 1.f;
}
__global__ void gather4(const float *__restrict__ t, float *__restrict__ sink, unsigned salt) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x + salt;
    const float v = t[(size_t)line_of(i) * 32 + (i & 31)];
    if (v == 123.f) sink[0] = 1.f;
}
__global__ void gather16(const float4 *__restrict__ t, float *__restrict__ sink, unsigned salt) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x + salt;
    const float4 v = t[(size_t)line_of(i) * 8 + (i & 7)];
    if (v.x + v.y + v.z + v.w == 123.f) sink[0] = 1.f;
}
struct Rec48 { float4 a, b, c; };
__global__ void rec48(const Rec48 *__restrict__ t, unsigned nrec, float *__restrict__ sink, unsigned salt) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x + salt;
    const unsigned r = (unsigned)(((unsigned long long)line_of(i) * nrec) >> 24);  // random record, spread over the table
    const Rec48 v = t[r];
    if (v.a.x + v.b.y + v.c.z == 123.f) sink[0] = 1.f;
}
__global__ void scatter4(unsigned *__restrict__ t, unsigned salt) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x + salt;
    t[(size_t)line_of(i) * 32 + (i & 31)] = i;
}
__global__ void scatter8(unsigned long long *__restrict__ t, unsigned salt) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x + salt;
    t[(size_t)line_of(i) * 16 + (i & 15)] = i;
}
__global__ void runs8x2(unsigned long long *__restrict__ t, unsigned salt) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x + salt;
    // pairs of consecutive 8-B slots, at a random 16-B-aligned place of a random line
    t[(size_t)line_of(i >> 1) * 16 + ((i >> 1) & 7) * 2 + (i & 1)] = i;
}

int main() {
    void *tab;
    float *sink;
    if (hipMalloc(&tab, TABLE) != hipSuccess || hipMalloc(&sink, 256) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    hipMemset(tab, 0, TABLE);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const unsigned g = N / 256;
    const unsigned nrec = (unsigned)(TABLE / sizeof(Rec48));
    // the warm launch uses other lines (salt 0 / N) than the timed one, so the timed one is not served by the
    // Infinity Cache
    auto run = [&](const char *name, double bytes, double lines, auto fn) {
        fn(0u);  // warm
        hipDeviceSynchronize();
        hipEventRecord(e0);
        fn(N);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-10s known_bytes %12.0f lines %10.0f  %8.1f us  %7.2f TB/s of known bytes  %7.2f TB/s of lines x 128\n",
               name, bytes, lines, ms * 1e3, bytes / (ms * 1e-3) / 1e12, lines * 128 / (ms * 1e-3) / 1e12);
    };
    // each kernel runs twice (warm + timed): the PMC tool divides its per-kernel counter total by the dispatches
    run("stream16", (double)TABLE / 4, (double)LINES / 4, [&](unsigned s) {
        stream16<<<4096, 256>>>((const float4 *)tab + (s ? TABLE / 16 / 2 : 0), TABLE / 16 / 4, sink);  // 512 MiB
    });
    run("line_full", (double)N * 16, (double)N / 8, [&](unsigned s) { line_full<<<g, 256>>>((const float4 *)tab, sink, s); });
    run("gather4", (double)N * 4, (double)N, [&](unsigned s) { gather4<<<g, 256>>>((const float *)tab, sink, s); });
    run("gather16", (double)N * 16, (double)N, [&](unsigned s) { gather16<<<g, 256>>>((const float4 *)tab, sink, s); });
    run("rec48", (double)N * 48, (double)N * 1.375, [&](unsigned s) { rec48<<<g, 256>>>((const Rec48 *)tab, nrec, sink, s); });
    run("scatter4", (double)N * 4, (double)N, [&](unsigned s) { scatter4<<<g, 256>>>((unsigned *)tab, s); });
    run("scatter8", (double)N * 8, (double)N, [&](unsigned s) { scatter8<<<g, 256>>>((unsigned long long *)tab, s); });
    run("runs8x2", (double)N * 8, (double)N / 2, [&](unsigned s) { runs8x2<<<g, 256>>>((unsigned long long *)tab, s); });
    hipDeviceSynchronize();
    hipFree(tab);
    hipFree(sink);
    printf("done\n");
    return 0;
}
