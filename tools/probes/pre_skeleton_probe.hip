// The preprocess kernel's memory pattern without its arithmetic (is 3 TB/s its access pattern's
// ceiling?).  Per Gaussian the preprocess reads 44 B of geometry (mean 12, opacity 4, rotation 16 as four 4-B loads,
// scale 12) and a 192-B coefficient row, and writes radius, tile count, depth key (4 B each), clamp byte, the 40-B render
// record (16 + 16 + 8 B at a 40-B stride), the 16-B expansion record and the 9-plane direction Jacobian.  Each
// kernel below does those memory operations (or a subset) with a trivial reduction in place of the arithmetic, over
// two alternating buffer sets (together beyond the 256 MiB Infinity Cache), timed with hipEvents.
//
//   hipcc --offload-arch=gfx950 -O3 tools/probes/pre_skeleton_probe.hip -o tools/probes/bin/pre_skeleton_probe
//   tools/probes/bin/pre_skeleton_probe [P]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct Rec {
    float4 a, b;
    float2 c;
};
struct Bufs {
    float *mean, *opac, *rot, *scale, *sh;
    int *radii;
    unsigned *tiles, *dkey;
    unsigned char *clamped;
    Rec *rec;
    uint4 *exp;
    float *jac;
};

enum : int { LD_GEOM = 1, LD_SH = 2, LD_SH_COAL = 4, ST_GEOM = 8, ST_JAC = 16, ST_ONCE = 32 };

template <int F>
__global__ __launch_bounds__(256) void skeleton(Bufs b, int P) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int ic = min(i, P - 1);
    float acc = 0.f;
    if (F & LD_GEOM) {
        acc += b.mean[3 * ic] + b.mean[3 * ic + 1] + b.mean[3 * ic + 2] + b.opac[ic];
        acc += b.rot[4 * ic] * b.rot[4 * ic + 1] + b.rot[4 * ic + 2] * b.rot[4 * ic + 3];
        acc += b.scale[3 * ic] + b.scale[3 * ic + 1] * b.scale[3 * ic + 2];
    }
    if (F & LD_SH) {
        const float4 *row = reinterpret_cast<const float4 *>(b.sh) + (size_t)ic * 12;
        float4 v[12];
#pragma unroll
        for (int k = 0; k < 12; k++) v[k] = row[k];
#pragma unroll
        for (int k = 0; k < 12; k++) acc += v[k].x * v[k].y + v[k].z * v[k].w;
    }
    if (F & LD_SH_COAL) {  // the wave's 64 rows (12 KB) as 12 coalesced 1-KB loads
        const int w0 = (i & ~63);
        const float4 *blk = reinterpret_cast<const float4 *>(b.sh) + (size_t)min(w0, P - 64) * 12;
        float4 v[12];
#pragma unroll
        for (int k = 0; k < 12; k++) v[k] = blk[k * 64 + lane];
#pragma unroll
        for (int k = 0; k < 12; k++) acc += v[k].x * v[k].y + v[k].z * v[k].w;
    }
    if (i >= P) return;
    if (F & ST_GEOM) {
        if (!(F & ST_ONCE)) {  // the preprocess's early defaults, overwritten below
            b.radii[i] = 0;
            b.tiles[i] = 0;
            b.dkey[i] = 0xffffffffu;
            b.clamped[i] = 0;
        }
        b.rec[i].a = make_float4(acc, acc + 1.f, acc + 2.f, acc + 3.f);
        b.rec[i].b = make_float4(acc + 4.f, acc + 5.f, acc + 6.f, acc + 7.f);
        b.rec[i].c = make_float2(acc + 8.f, acc + 9.f);
        b.radii[i] = (int)acc;
        b.exp[i] = make_uint4(__float_as_uint(acc), 1u, 2u, 3u);
        b.tiles[i] = (unsigned)acc + 1u;
        b.dkey[i] = __float_as_uint(acc);
        b.clamped[i] = (unsigned char)acc;
    }
    if (F & ST_JAC) {
#pragma unroll
        for (int k = 0; k < 9; k++) b.jac[(size_t)k * P + i] = acc + (float)k;
    }
}

static Bufs alloc(int P) {
    Bufs b;
    hipMalloc(&b.mean, 12ull * P);
    hipMalloc(&b.opac, 4ull * P);
    hipMalloc(&b.rot, 16ull * P);
    hipMalloc(&b.scale, 12ull * P);
    hipMalloc(&b.sh, 192ull * P);
    hipMalloc(&b.radii, 4ull * P);
    hipMalloc(&b.tiles, 4ull * P);
    hipMalloc(&b.dkey, 4ull * P);
    hipMalloc(&b.clamped, 1ull * P);
    hipMalloc(&b.rec, sizeof(Rec) * (size_t)P);
    hipMalloc(&b.exp, 16ull * P);
    hipMalloc(&b.jac, 36ull * P);
    hipMemset(b.sh, 0, 192ull * P);
    hipMemset(b.mean, 0, 12ull * P);
    hipMemset(b.rot, 0, 16ull * P);
    hipMemset(b.scale, 0, 12ull * P);
    hipMemset(b.opac, 0, 4ull * P);
    return b;
}

template <int F>
static void run(const char *name, Bufs *sets, int P, double bytes) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = (P + 255) / 256;
    for (int w = 0; w < 4; w++) skeleton<F><<<grid, 256>>>(sets[w & 1], P);
    std::vector<float> ms;
    for (int r = 0; r < 20; r++) {
        hipEventRecord(e0);
        skeleton<F><<<grid, 256>>>(sets[r & 1], P);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float t = 0.f;
        hipEventElapsedTime(&t, e0, e1);
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    printf("%-28s %8.4f ms  %6.2f TB/s  (%.0f MB)\n", name, med, bytes / (med * 1e-3) / 1e12, bytes / 1e6);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main(int argc, char **argv) {
    const int P = argc > 1 ? atoi(argv[1]) : 1000000;
    Bufs sets[2] = {alloc(P), alloc(P)};
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("allocation failed\n");
        return 1;
    }
    const double g = 44.0 * P, sh = 192.0 * P, sg = (4 + 4 + 4 + 1 + 40 + 16) * (double)P, sj = 36.0 * P;
    printf("P = %d\n", P);
    run<LD_GEOM | LD_SH | ST_GEOM | ST_JAC>("full (row loads)", sets, P, g + sh + sg + sj);
    run<LD_GEOM | LD_SH_COAL | ST_GEOM | ST_JAC>("full (coalesced sh)", sets, P, g + sh + sg + sj);
    run<LD_GEOM | LD_SH | ST_GEOM | ST_JAC | ST_ONCE>("full, stores once", sets, P, g + sh + sg + sj);
    run<LD_GEOM | ST_GEOM>("geometry only", sets, P, g + sg);
    run<LD_GEOM | LD_SH>("loads only (row)", sets, P, g + sh);
    run<LD_GEOM | LD_SH_COAL>("loads only (coalesced sh)", sets, P, g + sh);
    run<ST_GEOM | ST_JAC>("stores only", sets, P, sg + sj);
    run<LD_SH_COAL>("sh coalesced only", sets, P, sh);
    run<LD_SH>("sh rows only", sets, P, sh);
    return 0;
}
