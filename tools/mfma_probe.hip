// Lane-map probe of the f32 MFMA forms the SubNet uses (exact integer data): for each B lane l0, B = one-hot
// at l0 and A[l] = l + 1, so D[lane][r] = (the A lane whose value reached output (lane, r) with B lane l0) + 1,
// or 0.  Prints, per form, every nonzero (B lane, D lane, reg) -> A lane triple, compactly.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
template <int FORM>
__global__ void k(float* d, int l0) {
    const int l = threadIdx.x;
    const float a = float(l + 1), b = (l == l0) ? 1.f : 0.f;
    f4 c = {0.f, 0.f, 0.f, 0.f};
    if constexpr (FORM == 0) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    else c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}
int main() {
    float* d;
    hipMalloc(&d, 256 * 4);
    float h[256];
    for (int form = 0; form < 2; ++form) {
        printf("form %s: (Blane: Dlane.reg<-Alane ...)\n", form ? "16x16x4" : "4x4x1_16b");
        for (int l0 = 0; l0 < 64; ++l0) {
            if (form == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, d, l0);
            else hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, d, l0);
            hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
            printf("B%02d:", l0);
            for (int i = 0; i < 256; ++i)
                if (h[i] != 0.f) printf(" %d.%d<-%d", i / 4, i % 4, int(h[i]) - 1);
            printf("\n");
        }
    }
    return 0;
}
