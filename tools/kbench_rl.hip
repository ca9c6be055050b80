// Timing + phase trace of the fused Richardson-Lucy kernel k_rl_reg<256> (no torch).  Synthetic y >= 0
// and a positive Gaussian-like PSF per galaxy; the OTF through the engine's gd_psf_to_otf.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DGD_FUSED_TRACE=1] -o tools/kbench_rl tools/kbench_rl.hip
//   tools/kbench_rl [N=4096] [n_iters=100] [reps=3]
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"

#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_img(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u + seed;
        x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
        p[i] = 10.f + 100.f * ((x & 0xffffff) / float(0x1000000));
    }
}
__global__ void k_psf(float* p, int N, int h) {
    const int g = blockIdx.x;
    for (int i = threadIdx.x; i < h * h; i += blockDim.x) {
        const float dy = (i / h) - h / 2 + 0.5f, dx = (i % h) - h / 2 + 0.5f, s = 2.0f + (g % 7) * 0.3f;
        p[(size_t)g * h * h + i] = __expf(-(dx * dx + dy * dy) / (2 * s * s)) / (2 * 3.14159265f * s * s * 16.f);
    }
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096, n = argc > 2 ? atoi(argv[2]) : 100, reps = argc > 3 ? atoi(argv[3]) : 3;
    constexpr int L = 256, h = 48;
    float *y, *x, *psf; void *otf, *ws;
    // placement experiment: KB_XPAD bytes in front of x (the output / iterate), KB_OPAD in front of the OTF
    const size_t xpad = getenv("KB_XPAD") ? (size_t)atoll(getenv("KB_XPAD")) / 4 : 0;
    const size_t opad = getenv("KB_OPAD") ? (size_t)atoll(getenv("KB_OPAD")) : 0;
    CK(hipMalloc(&y, (size_t)N * L * L * 4)); CK(hipMalloc(&x, ((size_t)N * L * L + xpad) * 4));
    x += xpad;
    CK(hipMalloc(&psf, (size_t)N * h * h * 4));
    CK(hipMalloc(&otf, gd_otf_bytes(N, L, L) + opad)); CK(hipMalloc(&ws, gd_workspace_bytes(N, L, L)));
    otf = (char*)otf + opad;
    hipLaunchKernelGGL(k_img, dim3(4096), dim3(256), 0, 0, y, (size_t)N * L * L, 1u);
    hipLaunchKernelGGL(k_psf, dim3(N), dim3(256), 0, 0, psf, N, h);
    if (gd_psf_to_otf(psf, h * h, h, h, N, L, L, otf, ws, nullptr) != GD_OK) { printf("otf: %s\n", gd_last_error()); return 1; }
    CK(hipDeviceSynchronize());
#if GD_FUSED_TRACE
    unsigned long long* tr;
    CK(hipMalloc(&tr, (size_t)N * 16 * 8));
    CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_fused_trace), &tr, sizeof(tr)));
#endif
    Args a;
    memset(&a, 0, sizeof(a));
    a.N = N; a.y = y; a.o0 = x; a.otf = reinterpret_cast<float2*>(otf);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_rl_reg<L>), dim3(N), dim3(512), 0, 0, a, n);
    CK(hipGetLastError()); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_rl_reg<L>), dim3(N), dim3(512), 0, 0, a, n);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("k_rl_reg<256> N=%d n_iters=%d  %.3f ms  %.0f gal/s  %.2f us per galaxy-iteration-round\n", N, n, ms,
           N / (ms * 1e-3), ms * 1e3 / (n * ((N + 255) / 256)));
    std::vector<float> hx(L * L);
    CK(hipMemcpy(hx.data(), x, L * L * 4, hipMemcpyDeviceToHost));
    double s = 0; bool fin = true;
    for (float v : hx) { s += v; fin = fin && std::isfinite(v); }
    printf("galaxy 0: sum %.6e finite %d\n", s, (int)fin);
    {  // FNV-1a over the first min(N, 64) galaxies' outputs (bitwise comparison across builds)
        const size_t cnt = (size_t)(N < 64 ? N : 64) * L * L;
        std::vector<unsigned> hb(cnt);
        CK(hipMemcpy(hb.data(), x, cnt * 4, hipMemcpyDeviceToHost));
        unsigned long long hsh = 1469598103934665603ull;
        for (unsigned v : hb) { hsh ^= v; hsh *= 1099511628211ull; }
        printf("output fnv %016llx (first %zu galaxies)\n", hsh, cnt / (L * L));
    }
#if GD_FUSED_TRACE
    std::vector<unsigned long long> t((size_t)N * 16);
    CK(hipMemcpy(t.data(), tr, t.size() * 8, hipMemcpyDeviceToHost));
    const char* names[] = {"start -> x0 row FFTs", "it0 cols * H", "it0 rows ratio", "it0 cols * conj H", "it0 rows update", "iterations 1.. + end"};
    double tot = 0;
    for (int k = 0; k < 6; ++k) {
        double acc = 0;
        for (int i = 0; i < N; ++i) acc += (double)(t[i * 16 + k + 1] - t[i * 16 + k]);
        acc = acc / N / 100.0;
        tot += acc;
        printf("  %-24s %9.2f us\n", names[k], acc);
    }
    printf("  %-24s %9.2f us\n", "whole workgroup", tot);
#endif
    return 0;
}
