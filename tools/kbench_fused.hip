// Standalone microbenchmark of the fused Gaussian iteration k_gal_iter<256> (no torch): kernel time
// per variant and, built with -DGD_FUSED_TRACE=1, per-phase durations from s_memrealtime stamps
// (100 MHz) taken by thread 0 of every workgroup at the phase barriers.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGD_FUSED_TRACE=1 -o tools/kbench_fused tools/kbench_fused.hip
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"

#include <algorithm>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_fill(float* p, size_t n, unsigned seed, float lo, float hi) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u + seed;
        x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
        p[i] = lo + (hi - lo) * ((x & 0xffffff) / float(0x1000000));
    }
}

template <typename F>
float time_ms(F&& f, int reps = 10) {
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
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int variant = argc > 2 ? atoi(argv[2]) : 1;  // 1: k_gal_iter (parking), 2: k_gal_iter2 (register transpose)
    constexpr int L = 256, K = L / 2 + 1;
    const size_t img = (size_t)N * L * L, spec = (size_t)N * K * L;
    float *z, *zin, *par;
    float2* state;
    CK(hipMalloc(&z, img * 4)); CK(hipMalloc(&zin, img * 4));
    CK(hipMalloc(&state, 4 * spec * 8)); CK(hipMalloc(&par, N * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, z, img, 1u, 0.f, 1.f);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)state, 8 * spec, 2u, 0.f, 1.f);
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, par, (size_t)N, 3u, 0.5f, 1.5f);
    CK(hipDeviceSynchronize());
    Args a;
    memset(&a, 0, sizeof(a));
    a.N = N; a.s_hh = (float*)state; a.s_g = state + spec / 2; a.s_u1 = a.s_g + spec; a.s_w = a.s_g + 2 * spec;
    a.a0 = z; a.o0 = zin;
    a.alpha = a.rho1 = a.rho2 = a.rho2n = GalScalar{par, 1};
    a.llh = GD_LLH_GAUSSIAN;
#if GD_FUSED_TRACE
    unsigned long long* tr;  // stamps are written on every launch: set the buffer before any
    CK(hipMalloc(&tr, (size_t)N * 16 * 8));
    CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_fused_trace), &tr, sizeof(tr)));
#endif
    const double img_b = L * L * 4.0, half_b = K * L * 8.0;
    const double gb_mid = N * (2 * img_b + 5.5 * half_b) / 1e9;
    auto launch = [&] {
        if (variant == 2)
            hipLaunchKernelGGL((k_gal_iter2<L, false, false>), dim3(N), dim3(1024), 0, 0, a);
        else
            hipLaunchKernelGGL((k_gal_iter<L, false, false>), dim3(N), dim3(1024), 0, 0, a);
    };
    float t = time_ms(launch);
    printf("%s<256,MID>  %.3f ms  %.2f TB/s algorithmic (%.2f GB)\n", variant == 2 ? "k_gal_iter2" : "k_gal_iter", t,
           gb_mid / t, gb_mid);
#if GD_FUSED_TRACE
    launch();
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)N * 16);
    CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
    const char* names1[] = {"start -> z loaded", "row FFTs + park B bins", "slice A bins -> LDS", "gather A",
                           "column A (+ Nyquist) + park A", "unpark B, bins -> LDS", "gather B",
                           "column B + I half 0", "I half 1"};
    const char* names2[] = {"start -> z loaded", "row FFTs", "slice A bins -> LDS + gather A",
                            "slice B bins -> LDS", "column A (+ Nyquist), regs", "gather B",
                            "A rows half 0 + column B", "I half 0", "I half 1"};
    const char** names = variant == 2 ? names2 : names1;
    const int NP = 10;
    double sum[NP] = {0};
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int g = 0; g < N; ++g) {
        for (int k = 1; k < NP; ++k) sum[k - 1] += (h[g * 16 + k] - h[g * 16 + k - 1]) * 0.01;  // us
        t0 = std::min(t0, h[g * 16]);
        t1 = std::max(t1, h[g * 16 + 9]);
    }
    double tot = 0;
    for (int k = 0; k < NP - 1; ++k) {
        printf("  %-36s %7.2f us\n", names[k], sum[k] / N);
        tot += sum[k] / N;
    }
    printf("  %-36s %7.2f us per workgroup; first start -> last stamp %.3f ms\n", "total", tot, (t1 - t0) * 1e-5);
#endif
    return 0;
}
