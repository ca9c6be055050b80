// Timing + phase trace of the small-image Gaussian engine at configs[1] (256 x 48^2, n_iters = 8), no
// torch: the fused init (k_gal_small_init), one middle iteration (k_gal_small) launched back to back,
// and a hipGraph of the whole spectral forward (init + 8 iterations, identity denoiser) replayed.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DGD_FUSED_TRACE=1] -o tools/kbench_small tools/kbench_small.hip
//   tools/kbench_small [N=256] [L=48] [reps=200]
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"

#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define GK(x) do { int r_ = (x); if (r_ != GD_OK) { printf("engine error %d (%s) at %d\n", r_, gd_last_error(), __LINE__); exit(1); } } while (0)

__global__ void k_img(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u + seed;
        x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
        p[i] = 0.01f * ((x & 0xffffff) / float(0x1000000)) - 0.002f;
    }
}
__global__ void k_psf(float* p, int N, int h) {
    const int g = blockIdx.x;
    for (int i = threadIdx.x; i < h * h; i += blockDim.x) {
        const float dy = (i / h) - h / 2 + 0.5f, dx = (i % h) - h / 2 + 0.5f, s = 2.0f + (g % 7) * 0.3f;
        p[(size_t)g * h * h + i] = __expf(-(dx * dx + dy * dy) / (2 * s * s)) / (2 * 3.14159265f * s * s);
    }
}
__global__ void k_const(float* p, int n, float base, float step) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = base + step * (i % 13);
}

// Workgroup placement probe: 2N workgroups of 512 threads and 80 KiB of LDS (k_subnet_rhos_init's shape),
// each holding its CU for ~20 us, record (XCC, SE, SH, CU) from the hardware-id registers.
__global__ __launch_bounds__(512) void k_place(unsigned* out) {
    __shared__ float pad[20480];
    pad[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc + (pad[(blockIdx.x * 7) & 511] < 0.f ? 1u : 0u);
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(2);
}
static void placement(int N) {
    unsigned* d; CK(hipMalloc(&d, (size_t)4 * N * 4));
    hipLaunchKernelGGL(k_place, dim3(2 * N), dim3(512), 0, 0, d);
    CK(hipDeviceSynchronize());
    std::vector<unsigned> h((size_t)4 * N);
    CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    auto key = [&](int b) {
        const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 15;
        return (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
    };
    for (int part = 0; part < 3; ++part) {
        const int b0 = part == 2 ? 0 : part * N, b1 = part == 0 ? N : 2 * N;
        std::vector<std::pair<unsigned, int>> cnt;
        for (int b = b0; b < b1; ++b) {
            const unsigned k = key(b);
            bool f = false;
            for (auto& c : cnt) if (c.first == k) { ++c.second; f = true; }
            if (!f) cnt.push_back({k, 1});
        }
        int mx = 0;
        for (auto& c : cnt) mx = c.second > mx ? c.second : mx;
        printf("placement blocks [%d, %d): %zu distinct CUs, max %d blocks per CU\n", b0, b1, cnt.size(), mx);
    }
    printf("first 16 blocks (xcc se sh cu):");
    for (int b = 0; b < 16; ++b) { const unsigned k = key(b); printf(" %u.%u.%u.%u", k >> 16, (k >> 8) & 7, (k >> 4) & 1, k & 15); }
    printf("\n");
    CK(hipFree(d));
}

#if GD_FUSED_TRACE
static void print_trace(unsigned long long* tr, int N, int nph, const char** names) {
    std::vector<unsigned long long> t((size_t)N * 16);
    CK(hipMemcpy(t.data(), tr, t.size() * 8, hipMemcpyDeviceToHost));
    double tot = 0;
    for (int k = 0; k < nph; ++k) {
        double acc = 0;
        for (int i = 0; i < N; ++i) acc += (double)(t[i * 16 + k + 1] - t[i * 16 + k]);
        acc = acc / N / 100.0;  // s_memrealtime: 100 MHz
        tot += acc;
        printf("    %-28s %8.2f us\n", names[k], acc);
    }
    printf("    %-28s %8.2f us\n", "whole workgroup", tot);
}
#endif

// FNV-1a over the bits of n device floats: variants that must be bit-identical print the same value
static unsigned long long fnv_dev(const float* p, size_t n) {
    std::vector<float> v(n);
    CK(hipMemcpy(v.data(), p, n * 4, hipMemcpyDeviceToHost));
    unsigned long long h = 1469598103934665603ull;
    for (float f : v) { unsigned u; memcpy(&u, &f, 4); h = (h ^ u) * 1099511628211ull; }
    return h;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 256, L = argc > 2 ? atoi(argv[2]) : 48, reps = argc > 3 ? atoi(argv[3]) : 200;
    const int h = L < 48 ? L : 48, n_it = 8;
    if (argc > 4 && atoi(argv[4]) == 1) { placement(N); return 0; }
    float *y, *psf, *alpha, *rho1, *rho2, *zin, *out; void *state, *ws;
    CK(hipMalloc(&y, (size_t)N * L * L * 4)); CK(hipMalloc(&zin, (size_t)N * L * L * 4));
    CK(hipMalloc(&out, (size_t)N * L * L * 4));
    CK(hipMalloc(&psf, (size_t)N * h * h * 4));
    CK(hipMalloc(&alpha, N * 4)); CK(hipMalloc(&rho1, (size_t)N * n_it * 4)); CK(hipMalloc(&rho2, (size_t)N * n_it * 4));
    CK(hipMalloc(&state, gd_admm_state_bytes(N, L, L, GD_LLH_GAUSSIAN)));
    CK(hipMalloc(&ws, gd_workspace_bytes(N, L, L) + 16));
    hipLaunchKernelGGL(k_img, dim3(1024), dim3(256), 0, 0, y, (size_t)N * L * L, 1u);
    hipLaunchKernelGGL(k_psf, dim3(N), dim3(256), 0, 0, psf, N, h);
    hipLaunchKernelGGL(k_const, dim3(4), dim3(256), 0, 0, alpha, N, 0.004f, 0.0003f);
    hipLaunchKernelGGL(k_const, dim3(8), dim3(256), 0, 0, rho1, N * n_it, 0.7f, 0.05f);
    hipLaunchKernelGGL(k_const, dim3(8), dim3(256), 0, 0, rho2, N * n_it, 0.9f, 0.04f);
    CK(hipDeviceSynchronize());
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
#if GD_FUSED_TRACE
    unsigned long long* tr;
    CK(hipMalloc(&tr, (size_t)N * 16 * 8));
    CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_fused_trace), &tr, sizeof(tr)));
#endif
    auto init = [&]() {
        GK(gd_admm_init(y, psf, (long long)h * h, h, h, alpha, 1, nullptr, 0, GD_LLH_GAUSSIAN, N, L, L, state, zin, ws, st));
    };
    auto iter = [&](int it) {
        const bool last = it == n_it - 1;
        GK(gd_admm_iter(y, zin, last ? out : zin, alpha, 1, rho1 + it, n_it, rho2 + it, n_it, last ? nullptr : rho2 + it + 1,
                        n_it, GD_LLH_GAUSSIAN, it, last, N, L, L, state, ws, st));
    };
    auto forward = [&]() {
        init();
        for (int it = 0; it < n_it; ++it) iter(it);
    };
    forward();
    CK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char* what, auto&& f, int r) {
        f();
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < r; ++i) f();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-40s %9.2f us per call\n", what, ms * 1e3 / r);
    };
    {   // SubNet alone and the fused init + SubNet launch (synthetic weights: timing only)
        float *prm, *mlp, *rh;
        const int n_out = 2 * n_it;
        CK(hipMalloc(&prm, gd::subnet::kParams * 4)); CK(hipMalloc(&mlp, gd::subnet::mlp_param_count(n_out) * 4));
        CK(hipMalloc(&rh, (size_t)N * n_out * 4));
        hipLaunchKernelGGL(k_const, dim3(16), dim3(256), 0, 0, prm, gd::subnet::kParams, -0.02f, 0.005f);
        hipLaunchKernelGGL(k_const, dim3(64), dim3(256), 0, 0, mlp, gd::subnet::mlp_param_count(n_out), -0.003f, 0.0005f);
        CK(hipDeviceSynchronize());
        float* feat; CK(hipMalloc(&feat, (size_t)N * 1024 * 4));
        timeit("SubNet (gd_subnet_rhos_psf)", [&]() {
            GK(gd_subnet_rhos_psf(psf, (long long)h * h, h, prm, mlp, alpha, 1, feat, rh, n_out, N, st)); }, reps);
        if (gd_admm_init_subnet_supported(N, L, L, h, h, GD_LLH_GAUSSIAN, n_out)) {
            for (int map = 0; map < 3; ++map) {
                g_sri_map = map;
                char name[64];
                snprintf(name, sizeof name, "init + SubNet, one launch (map %d)", map);
                timeit(name, [&]() {
                    GK(gd_admm_init_subnet(y, psf, (long long)h * h, h, h, alpha, 1, GD_LLH_GAUSSIAN, N, L, L, state, zin,
                                           prm, mlp, rh, n_out, ws, st)); }, reps);
            }
        }
        CK(hipStreamSynchronize(st));
        printf("rhos fnv %016llx  init zin fnv %016llx\n", fnv_dev(rh, (size_t)N * n_out), fnv_dev(zin, (size_t)N * L * L));
    }
    timeit("init (back to back)", init, reps);
    timeit("middle iteration (back to back)", [&]() { iter(3); }, reps);
    // the whole spectral forward as one graph
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    forward();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    timeit("forward (hipGraph: init + 8 iterations)", [&]() { CK(hipGraphLaunch(ge, st)); }, reps / 4 + 1);
    std::vector<float> ho((size_t)L * L);
    CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
    double s = 0;
    for (float v : ho) s += v;
    printf("galaxy 0 output sum %.6e  output fnv %016llx\n", s, fnv_dev(out, (size_t)N * L * L));
#if GD_FUSED_TRACE
    const char* names[] = {"twiddles + state prefetch", "R: row FFTs", "C: columns + update", "I: inverse rows + store"};
    CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
    iter(3);
    CK(hipStreamSynchronize(st));
    printf("k_gal_small<%d> middle iteration phase trace (mean per workgroup):\n", L);
    print_trace(tr, N, 4, names);
#endif
    return 0;
}
