// Prints the lane mapping of gfx950's v_permlane32_swap / v_permlane16_swap (as exposed by the clang
// builtins) so the wave reductions in gsr_backward.hip can rely on a measured, not assumed, semantics.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned *out) {
    const unsigned l = threadIdx.x;
    const unsigned x = l, y = 100 + l;
    auto a = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    auto b = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    out[l] = a[0];
    out[64 + l] = a[1];
    out[128 + l] = b[0];
    out[192 + l] = b[1];
}

int main() {
    unsigned *d, h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    probe<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *names[4] = {"swap32.x", "swap32.y", "swap16.x", "swap16.y"};
    for (int t = 0; t < 4; t++) {
        printf("%s:", names[t]);
        for (int l = 0; l < 64; l++) printf(" %u", h[64 * t + l]);
        printf("\n");
    }
    return hipFree(d) == hipSuccess ? 0 : 1;
}
