// Timing + phase trace of the Poisson two-pass kernels at 256^2 (no torch): pass A k_gal_reg<256, true>
// and pass B k_pois_b<256> on random state (timing only: the values are not a real forward).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DGD_FUSED_TRACE=1] -o tools/kbench_pois tools/kbench_pois.hip
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
__global__ void k_fillp(float* p, size_t n, unsigned seed, float lo, float hi) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u + seed;
        x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
        p[i] = lo + (hi - lo) * ((x & 0xffffff) / float(0x1000000));
    }
}
template <typename F>
float time_ms(F&& f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}
int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096, reps = argc > 2 ? atoi(argv[2]) : 10;
    constexpr int L = 256, K = L / 2 + 1;
    const size_t img = (size_t)N * L * L, spec = (size_t)N * K * L;
    float *z, *zin, *y, *w, *par; float2* st;
    CK(hipMalloc(&z, img * 4)); CK(hipMalloc(&zin, img * 4)); CK(hipMalloc(&y, img * 4)); CK(hipMalloc(&w, img * 4));
    const size_t pad = getenv("KB_PAD") ? (size_t)atoll(getenv("KB_PAD")) / 8 : 0;  // float2 between the state slots
    CK(hipMalloc(&st, 5 * spec * 8 + 4 * pad * 8)); CK(hipMalloc(&par, N * 4));
    hipLaunchKernelGGL(k_fillp, dim3(4096), dim3(256), 0, 0, z, img, 1u, 0.f, 1.f);
    hipLaunchKernelGGL(k_fillp, dim3(4096), dim3(256), 0, 0, y, img, 2u, 10.f, 100.f);
    hipLaunchKernelGGL(k_fillp, dim3(4096), dim3(256), 0, 0, w, img, 3u, 0.f, 1.f);
    hipLaunchKernelGGL(k_fillp, dim3(4096), dim3(256), 0, 0, (float*)st, 10 * spec, 4u, 0.f, 1.f);
    hipLaunchKernelGGL(k_fillp, dim3(64), dim3(256), 0, 0, par, (size_t)N, 5u, 0.5f, 1.5f);
    CK(hipDeviceSynchronize());
#if GD_FUSED_TRACE
    unsigned long long* tr;
    CK(hipMalloc(&tr, (size_t)N * 16 * 8)); CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_fused_trace), &tr, sizeof(tr)));
#endif
    Args a; memset(&a, 0, sizeof(a));
    a.N = N; a.llh = GD_LLH_POISSON;
    a.s_hh = (float*)st; float2* c = st + spec / 2 + pad;
    a.s_g = c; a.s_u1 = c + spec + pad; a.s_w = c + 2 * (spec + pad); a.s_x = c + 3 * (spec + pad);
    a.a0 = z; a.o0 = zin; a.y = y; a.o1 = w;
    a.alpha = a.rho1 = a.rho2 = a.rho2n = GalScalar{par, 1};
    const double imgb = L * L * 4.0, halfb = K * L * 8.0;
    const double ga = N * (2 * imgb + 4.5 * halfb) / 1e9, gbb = N * (3 * imgb + 3 * halfb) / 1e9;
    const float ta = time_ms([&] { hipLaunchKernelGGL((k_gal_reg<L, true>), dim3(N), dim3(512), 0, 0, a); }, reps);
    const float tb = time_ms([&] { hipLaunchKernelGGL((k_pois_b<L>), dim3(N), dim3(512), 0, 0, a, 0); }, reps);
    CK(hipGetLastError());
    printf("pass A k_gal_reg<256,POIS> MID N=%d %.3f ms %.2f TB/s (%.2f GB)\n", N, ta, ga / ta, ga);
    printf("pass B k_pois_b<256>       N=%d %.3f ms %.2f TB/s (%.2f GB, + the OTF re-read)\n", N, tb, gbb / tb, gbb);
#if GD_FUSED_TRACE
    CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
    hipLaunchKernelGGL((k_pois_b<L>), dim3(N), dim3(512), 0, 0, a, 0);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)N * 16);
    CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
    const char* names[] = {"C1 (H X, column IFFTs)", "I half 0 (V step, F rows)", "I half 1", "W slice A", "W slice B"};
    double tot = 0;
    for (int k = 0; k < 5; ++k) {
        double s = 0;
        for (int i = 0; i < N; ++i) s += (double)(h[i * 16 + k + 1] - h[i * 16 + k]);
        s = s / N / 100.0; tot += s;
        printf("  %-28s %7.2f us\n", names[k], s);
    }
    printf("  %-28s %7.2f us\n", "pass B workgroup", tot);
#endif
    return 0;
}
