// Issue rate of the f32 VALU forms the composite kernels are built from, on one SIMD with 1..8 waves:
// v_fma_f32, v_pk_fma_f32 (two f32 FMAs per lane), v_exp_f32, v_rcp_f32, and an fma/exp mix.  Each wave runs
// 8 independent dependency chains (SALU: s_add_u32 chains; the shader clock is s_memtime / s_memrealtime) (so latency is hidden) for ITER iterations; the cycle count is taken with
// s_memtime around the loop.  Prints cycles per wave-instruction per SIMD (= cycles / (waves x instructions)).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/valu_rate_probe.hip -o tools/probes/valu_rate_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;

template <int OP>
__global__ __launch_bounds__(256) void probe(float *out, unsigned long long *cyc, float seed, unsigned useed) {
    float a[8];
    unsigned sc[8];
    unsigned long long m64 = ((unsigned long long)useed << 32) | useed, m64b = ~0ull ^ useed;
    f2 p[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a[i] = seed + threadIdx.x * 1e-3f + i;
        p[i] = f2{a[i], a[i] + 0.5f};
        sc[i] = useed + i;
    }
    const float b = 0.999f, c = 1e-3f;
    const f2 b2 = f2{b, b}, c2 = f2{c, c};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(b2), "v"(c2));
            if (OP == 2) asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
            if (OP == 3) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[i]));
            if (OP == 4) {  // 3 fma : 1 exp
                if (i & 3) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                else asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
            }
            if (OP == 5) {  // 3 pk_fma : 1 exp
                if (i & 3) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(b2), "v"(c2));
                else asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
            }
            if (OP == 6) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(b2));
            if (OP == 7) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 9) asm volatile("s_add_u32 %0, %0, 3" : "+s"(sc[i]) : : "scc");
            if (OP == 10) {  // alternating v_fma / s_add
                if (i & 1) asm volatile("s_add_u32 %0, %0, 3" : "+s"(sc[i]) : : "scc");
                else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            }
            if (OP == 11) {  // 3 v_fma : 1 s_add (the composite backward's VALU : SALU mix)
                if ((i & 3) == 3) asm volatile("s_add_u32 %0, %0, 3" : "+s"(sc[i]) : : "scc");
                else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            }
            if (OP == 12) {  // 1 v_fma : 1 s_and_b64 (64-bit mask logic, as the exec-mask control uses)
                if (i & 1) asm volatile("s_and_b64 %0, %0, %1" : "+s"(m64) : "s"(m64b) : "scc");
                else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            }
            if (OP == 13) asm volatile("v_mov_b32 %0, 0" : "=v"(a[i]));  // zeroing (the backward's accumulator init)
            if (OP == 14) asm volatile("v_mov_b64 %0, 0" : "=v"(p[i]));  // two zeroed registers per instruction
            if (OP == 15) {  // 1 v_fma : 1 v_mov_b64
                if (i & 1) asm volatile("v_mov_b64 %0, 0" : "=v"(p[i]));
                else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            }
            if (OP == 8) {  // alternating v_fma / v_pk_fma
                if (i & 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(b2), "v"(c2));
                else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i] + p[i].x + p[i].y + (float)sc[i];
    s += (float)(unsigned)m64;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) {
        cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
        if (blockIdx.x == 0 && threadIdx.x == 0) cyc[256 * 32] = r1 - r0;  // 100 MHz ticks of wave 0
    }
}

template <int OP>
static void run(const char *name, float *out, unsigned long long *cyc) {
    // 4-wave workgroups (one wave per SIMD), W workgroups per CU (256 CUs) -> W waves per SIMD
    for (int w : {1, 2, 4, 8}) {
        const int waves = 4, blocks = 256 * w;
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        probe<OP><<<blocks, 64 * waves>>>(out, cyc, 1.0f, 7u);
        (void)hipEventRecord(e1);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            printf("launch failed\n");
            return;
        }
        static unsigned long long h[256 * 32];
        for (auto &x : h) x = 0;
        if (hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks * waves, hipMemcpyDeviceToHost) != hipSuccess) return;
        double mx = 0;
        for (int i = 0; i < blocks * waves; i++) mx = h[i] > mx ? h[i] : mx;
        // s_memtime counts at the shader clock (MI355X_MICROARCH.md constants table)
        const double per = mx / (double(w) * ITER * 8);
        unsigned long long rt = 0, c0 = 0;
        (void)hipMemcpy(&rt, cyc + 256 * 32, sizeof(rt), hipMemcpyDeviceToHost);
        c0 = h[0];
        const double ghz = rt ? (double)c0 / (double)rt * 0.1 : 0.0;  // s_memtime ticks per 10 ns
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        // kernel-wide: wave-instructions per SIMD over the event time at the 2.4 GHz shader clock
        const double per_ev = ms * 2.4e6 / (double(blocks) * waves * ITER * 8 / 1024.0);
        printf("%-22s waves/SIMD %d: %.2f cyc/instr/SIMD (s_memtime)  %.2f (events @2.4GHz, %.3f ms)  clock %.2f GHz  "
               "%.3f ns/instr/SIMD\n", name, w, per, per_ev, ms, ghz,
               ms * 1e6 / (double(blocks) * waves * ITER * 8 / 1024.0));
    }
}

int main() {
    float *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, 256 * 8 * 256 * sizeof(float)) != hipSuccess) return 1;
    if (hipMalloc(&cyc, (256 * 32 + 1) * sizeof(unsigned long long)) != hipSuccess) return 1;
    run<0>("v_fma_f32", out, cyc);
    run<7>("v_mul_f32", out, cyc);
    run<1>("v_pk_fma_f32", out, cyc);
    run<6>("v_pk_mul_f32", out, cyc);
    run<2>("v_exp_f32", out, cyc);
    run<3>("v_rcp_f32", out, cyc);
    run<4>("3 fma : 1 exp", out, cyc);
    run<5>("3 pk_fma : 1 exp", out, cyc);
    run<8>("fma / pk_fma alt", out, cyc);
    run<9>("s_add_u32", out, cyc);
    run<10>("fma / s_add alt", out, cyc);
    run<11>("3 fma : 1 s_add", out, cyc);
    run<12>("fma / s_and_b64 alt", out, cyc);
    run<13>("v_mov_b32 0", out, cyc);
    run<14>("v_mov_b64 0", out, cyc);
    run<15>("fma / v_mov_b64 alt", out, cyc);
    return 0;
}
