// Timing + phase trace of the SubNet kernels (no torch): k_subnet_features_psf at batch N and
// k_subnet_rhos_psf (one fused launch) at batch Nr, synthetic 48 x 48 PSFs and seeded random weights.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DGD_SN_TRACE=1] -o tools/kbench_subnet tools/kbench_subnet.hip
//   tools/kbench_subnet [N=4096] [Nr=256] [reps=20]
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"

#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_psf(float* p, int N, int h) {
    const int g = blockIdx.x;
    for (int i = threadIdx.x; i < h * h; i += blockDim.x) {
        const float dy = (i / h) - h / 2 + 0.5f, dx = (i % h) - h / 2 + 0.5f, s = 2.0f + (g % 7) * 0.3f;
        p[(size_t)g * h * h + i] = __expf(-(dx * dx + dy * dy) / (2 * s * s)) / (2 * 3.14159265f * s * s);
    }
}

static std::vector<float> rnd(size_t n, float scale, unsigned seed) {
    std::vector<float> v(n);
    unsigned x = seed;
    for (auto& e : v) {
        x = x * 1664525u + 1013904223u;
        e = scale * (((x >> 8) & 0xffff) / 32768.f - 1.f);
    }
    return v;
}

static const char* kPhase[13] = {"start", "PSF rows+cols FFT", "|H|^2 pool", "conv0 1->4 @64",
                                 "conv1 4->4 @64+pool", "conv2 4->8 @32", "conv3 8->8 @32+pool",
                                 "conv4 8->16 @16", "conv5 16->16 @16+pool", "conv6 16->16 @8",
                                 "conv7 16->16 @8", "MLP (layer 1)", "MLP layers 2-3"};

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096, Nr = argc > 2 ? atoi(argv[2]) : 256,
              reps = argc > 3 ? atoi(argv[3]) : 20;
    constexpr int h = 48, n_out = 16;
    const int NM = N > Nr ? N : Nr;
    float *psf, *params, *mlp, *alpha, *feat, *rhos;
    CK(hipMalloc(&psf, (size_t)NM * h * h * 4));
    CK(hipMalloc(&params, gd::subnet::kParams * 4));
    const int nm = gd::subnet::mlp_param_count(n_out);
    CK(hipMalloc(&mlp, (size_t)nm * 4));
    CK(hipMalloc(&alpha, (size_t)NM * 4));
    CK(hipMalloc(&feat, (size_t)NM * 1024 * 4));
    CK(hipMalloc(&rhos, (size_t)NM * n_out * 4));
    hipLaunchKernelGGL(k_psf, dim3(NM), dim3(256), 0, 0, psf, NM, h);
    auto hp = rnd(gd::subnet::kParams, 0.3f, 7u), hm = rnd(nm, 0.05f, 9u), ha = rnd(NM, 0.5f, 11u);
    for (auto& e : ha) e += 1.f;
    CK(hipMemcpy(params, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(mlp, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(alpha, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
#if GD_SN_TRACE
    unsigned long long* tr;
    CK(hipMalloc(&tr, (size_t)NM * 16 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(gd::subnet::g_sn_trace), &tr, sizeof(tr)));
#endif
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto feats = [&](int n) {
        hipLaunchKernelGGL(gd::subnet::k_subnet_features_psf, dim3(n), dim3(gd::subnet::kThreads), 0, 0, psf,
                           (long long)h * h, h, params, feat, n);
    };
    auto fused = [&](int n) {
        hipLaunchKernelGGL(gd::subnet::k_subnet_rhos_psf, dim3(n), dim3(gd::subnet::kThreads), 0, 0, psf,
                           (long long)h * h, h, params, mlp, alpha, 1LL, rhos, n_out, n);
    };
    auto timeit = [&](auto launch, int n, const char* name) {
        launch(n);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch(n);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-24s N=%5d  %8.1f us per launch\n", name, n, ms * 1e3 / reps);
#if GD_SN_TRACE
        std::vector<unsigned long long> t((size_t)n * 16);
        CK(hipMemset(tr, 0, (size_t)n * 16 * 8));
        launch(n);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(t.data(), tr, t.size() * 8, hipMemcpyDeviceToHost));
        printf("  phase trace (mean us per workgroup, 100 MHz clock):\n");
        for (int k = 1; k < 13; ++k) {
            double s = 0;
            int c = 0;
            for (int g = 0; g < n; ++g)
                if (t[g * 16 + k] && t[g * 16 + k - 1]) {
                    s += double(t[g * 16 + k] - t[g * 16 + k - 1]);
                    ++c;
                }
            if (c) printf("    %-24s %8.2f\n", kPhase[k], s / c * 1e-2);
        }
        double s = 0;
        for (int g = 0; g < n; ++g) s += double(t[g * 16 + (t[g * 16 + 12] ? 12 : t[g * 16 + 11] ? 11 : 10)] - t[g * 16]);
        printf("    %-24s %8.2f\n", "whole workgroup", s / n * 1e-2);
#endif
    };
    timeit(feats, N, "k_subnet_features_psf");
    // the batched MLP on those features: k_subnet_mlp (VALU) and k_subnet_mlp_mfma, both into rhosb
    float* rhosb;
    CK(hipMalloc(&rhosb, (size_t)NM * n_out * 4));
    auto mlp_valu = [&](int n) {
        hipLaunchKernelGGL(gd::subnet::k_subnet_mlp, dim3((n + gd::subnet::kMlpG - 1) / gd::subnet::kMlpG),
                           dim3(gd::subnet::kMlpThreads), 0, 0, feat, mlp, alpha, 1LL, rhosb, n_out, n);
    };
    auto mlp_mfma = [&](int n) {
        hipLaunchKernelGGL(gd::subnet::k_subnet_mlp_mfma, dim3((n + gd::subnet::kMG - 1) / gd::subnet::kMG),
                           dim3(gd::subnet::kMlpThreads), 0, 0, feat, mlp, alpha, 1LL, rhosb, n_out, n);
    };
    auto rfnv = [&](int n) {
        std::vector<float> v((size_t)n * n_out);
        CK(hipMemcpy(v.data(), rhosb, v.size() * 4, hipMemcpyDeviceToHost));
        unsigned long long h = 1469598103934665603ull;
        for (float f : v) { unsigned u; memcpy(&u, &f, 4); h = (h ^ u) * 1099511628211ull; }
        return h;
    };
    timeit(mlp_valu, N, "k_subnet_mlp");
    const unsigned long long h_valu = rfnv(N), h_valu_r = rfnv(Nr);
    timeit(mlp_mfma, N, "k_subnet_mlp_mfma");
    printf("batched rhos fnv: k_subnet_mlp %016llx  k_subnet_mlp_mfma %016llx  (first %d: %016llx / %016llx)\n", h_valu,
           rfnv(N), Nr, h_valu_r, rfnv(Nr));
    timeit(fused, Nr, "k_subnet_rhos_psf");
    std::vector<float> hr(n_out);
    CK(hipMemcpy(hr.data(), rhos, n_out * 4, hipMemcpyDeviceToHost));
    printf("rhos[0][:4] = %g %g %g %g\n", hr[0], hr[1], hr[2], hr[3]);
    // bitwise fingerprints of every feature (batched kernel, N) and every rho (fused kernel, Nr): variants that
    // must be bit-identical print the same hashes
    auto fnv = [](const std::vector<float>& v) {
        unsigned long long h = 1469598103934665603ull;
        for (float f : v) { unsigned u; memcpy(&u, &f, 4); h = (h ^ u) * 1099511628211ull; }
        return h;
    };
    std::vector<float> hf((size_t)N * 1024), hra((size_t)Nr * n_out);
    CK(hipMemcpy(hf.data(), feat, hf.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hra.data(), rhos, hra.size() * 4, hipMemcpyDeviceToHost));
    printf("features fnv %016llx  rhos fnv %016llx\n", fnv(hf), fnv(hra));
    return 0;
}
