// Standalone check + timing of the fused Gaussian iteration k_gal_reg<256> (no torch): checked against the
// engine's chained three-kernel path (Ops<256>::admm_iter_gauss with g_fused = 0: RF_ONE -> C_G_ITER* -> RI_OUT1
// through the workspace) on the same 256^2 state layout (sidx_c / sidx_h).  The per-bin arithmetic is the same
// (gauss_math_rt); the transforms' rounding differs, so results agree to rounding (max |d| <= 1e-6 max |x| over
// zin and the U1 / W~ state is the bar; the tool exits non-zero otherwise).  Then k_gal_reg is timed over the batch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/kbench_reg tools/kbench_reg.hip
//   tools/kbench_reg [N=4096] [reps=20] [noparity]  (noparity: time layout experiments that break the comparison)
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"

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

constexpr int L = 256, K = L / 2 + 1;

struct Bufs {
    float *z, *zin;
    float2* state;  // |H|^2 (K L floats, padded to K L float2) | G | U1 | W~
    float2* ws;     // the chained path's workspace
    Args a;
};

Bufs make(int N, float* par, bool placed = false) {
    const size_t img = (size_t)N * L * L, spec = (size_t)N * K * L;
    Bufs b;
    // placement experiment: KB_PAD bytes between the state slots, KB_ZPAD bytes in front of z and zin (multiples of 16)
    // (the timing buffers only; the parity buffers keep the engine's contiguous slots)
    const size_t pad = placed && getenv("KB_PAD") ? (size_t)atoll(getenv("KB_PAD")) / 16 * 2 : 0;    // in float2
    const size_t zpad = placed && getenv("KB_ZPAD") ? (size_t)atoll(getenv("KB_ZPAD")) / 16 * 4 : 0; // in floats
    // KB_LAYOUT=1: the engine's Gaussian layout (bind_state: |H|^2 takes half a slot); KB_ALIAS=1: z == zin (the
    // identity denoiser's in-place iteration)
    const bool eng = placed && getenv("KB_LAYOUT") && atoi(getenv("KB_LAYOUT")) == 1;
    const bool alias = placed && getenv("KB_ALIAS") && atoi(getenv("KB_ALIAS")) == 1;
    CK(hipMalloc(&b.z, (img + zpad) * 4)); CK(hipMalloc(&b.zin, (img + zpad) * 4));
    CK(hipMalloc(&b.state, (4 * spec + 3 * pad) * 8));
    CK(hipMalloc(&b.ws, 2 * spec * 8));
    memset(&b.a, 0, sizeof(b.a));
    b.a.T = b.ws;
    b.a.N = N; b.a.gH = b.a.gW = L; b.a.s_hh = (float*)b.state;
    b.a.s_g = b.state + (eng ? (spec + 1) / 2 : spec) + pad; b.a.s_u1 = b.a.s_g + spec + pad;
    b.a.s_w = b.a.s_u1 + spec + pad;
    b.z += zpad; b.zin += zpad;
    if (alias) b.zin = b.z;
    b.a.a0 = b.z; b.a.o0 = b.zin;
    b.a.alpha = b.a.rho1 = b.a.rho2 = b.a.rho2n = GalScalar{par, 1};
    b.a.llh = GD_LLH_GAUSSIAN;
    return b;
}

void seed(Bufs& b, int N) {
    const size_t img = (size_t)N * L * L, spec = (size_t)N * K * L;
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, b.z, img, 1u, 0.f, 1.f);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)b.state, 8 * spec, 2u, 0.f, 1.f);
    CK(hipMemset(b.zin, 0, img * 4));
    CK(hipDeviceSynchronize());
}

// Streaming ceiling for one galaxy's MID traffic (z, |H|^2, G, U1, W~ in; U1, W~, zin out), float4 per
// lane, no phases: what the memory system gives this read/write mix with one T-thread workgroup per CU
// (LDS sized like k_gal_reg's so the residency matches).
template <int T>
__global__ __launch_bounds__(T) void k_stream(Args a) {
    __shared__ float pad[35000];
    const int g = blockIdx.x, tid = threadIdx.x;
    const size_t img = (size_t)L * L, spec = (size_t)K * L;
    const f4v* z = reinterpret_cast<const f4v*>(a.a0 + g * img);
    f4v* zin = reinterpret_cast<f4v*>(a.o0 + g * img);
    const f4v* hh = reinterpret_cast<const f4v*>(a.s_hh + g * spec);
    const f4v* G = reinterpret_cast<const f4v*>(a.s_g + g * spec);
    f4v* U = reinterpret_cast<f4v*>(a.s_u1 + g * spec);
    f4v* W = reinterpret_cast<f4v*>(a.s_w + g * spec);
    if (tid == 0) pad[0] = 0.f;
    for (int i = tid; i < (int)(img / 4); i += T) zin[i] = z[i] * 1.5f;
    for (int i = tid; i < (int)(spec / 2); i += T) {
        const f4v h = hh[i / 2];
        const f4v gg = G[i], u = U[i], w = W[i];
        U[i] = u + gg * h;
        W[i] = w - gg;
    }
}

// variant 0: the chained three-kernel path (the reference), 1: k_gal_reg; fl: 0 MID, 1 FIRST, 2 LAST, 3 FIRST_LAST
void launch_v(int variant, int fl, Args a) {
    a.first = fl & 1;
    a.last = fl >> 1;
    if (variant == 0) {
        const int old = g_fused;
        g_fused = 0;
        if (Ops<L>::admm_iter_gauss(a, 0) != GD_OK) { printf("chain failed: %s\n", g_last_error.c_str()); exit(1); }
        g_fused = old;
    } else {
        hipLaunchKernelGGL((k_gal_reg<L>), dim3(a.N), dim3(512), 0, 0, a);
    }
}

double diff(const void* x, const void* y, size_t bytes) {
    std::vector<float> hx(bytes / 4), hy(bytes / 4);
    CK(hipMemcpy(hx.data(), x, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hy.data(), y, bytes, hipMemcpyDeviceToHost));
    long long n = 0, first = -1;
    double md = 0, mx = 0;
    for (size_t i = 0; i < hx.size(); ++i) {
        if (memcmp(&hx[i], &hy[i], 4)) { ++n; if (first < 0) first = (long long)i; }
        md = fmax(md, fabs((double)hx[i] - hy[i]));
        mx = fmax(mx, fabs((double)hx[i]));
    }
    if (n) printf("   max|d| %.3e  max|x| %.3e  first differing word %lld (%g vs %g)\n", md, mx, first, hx[first], hy[first]);
    return mx > 0 ? md / mx : md;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    float* par;
    CK(hipMalloc(&par, N * 4));
#if GD_FUSED_TRACE
    unsigned long long* tr;  // every launch of a traced build writes stamps: set the buffer before any
    CK(hipMalloc(&tr, (size_t)N * 16 * 8));
    CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_fused_trace), &tr, sizeof(tr)));
#endif
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, par, (size_t)N, 3u, 0.5f, 1.5f);
    // parity on a small batch: every variant (FIRST, MID, LAST, FIRST_LAST), all outputs, on a consistent
    // (Hermitian) state: the engine's init from random y and PSFs, then the iterations in order with the identity
    // denoiser (random spectra are not the spectra of real images: the two paths drop their non-Hermitian parts
    // differently)
    const int Nc = N < 64 ? N : 64;
    const size_t img = (size_t)Nc * L * L, spec = (size_t)Nc * K * L;
    Bufs x = make(Nc, par), y = make(Nc, par);
    float2* state0;
    CK(hipMalloc(&state0, 4 * spec * 8));
    {
        float *yi, *psf;
        const int h = 48;
        CK(hipMalloc(&yi, img * 4)); CK(hipMalloc(&psf, (size_t)Nc * h * h * 4));
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, yi, img, 11u, -0.1f, 1.f);
        hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, psf, (size_t)Nc * h * h, 12u, 0.f, 1e-3f);
        CK(hipMemset(x.state, 0, 4 * spec * 8));
        Args b = x.a;
        b.y = yi; b.psf = psf; b.psf_gstride = h * h; b.h = h; b.o2 = x.zin;
        if (Ops<L>::admm_init_gauss(b, 0) != GD_OK) { printf("init failed: %s\n", g_last_error.c_str()); return 1; }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(state0, x.state, 4 * spec * 8, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(x.z, x.zin, img * 4, hipMemcpyDeviceToDevice));  // z0 = x0 (identity denoiser)
    }
    float* z0;
    CK(hipMalloc(&z0, img * 4));
    CK(hipMemcpy(z0, x.z, img * 4, hipMemcpyDeviceToDevice));
    int bad = 0;
    const char* fln[] = {"MID", "FIRST", "LAST", "FIRST_LAST"};
    for (int fl : {1, 0, 2, 3}) {  // FIRST, MID, LAST continue from the previous step; FIRST_LAST from the init
        if (fl == 3) {
            CK(hipMemcpy(x.state, state0, 4 * spec * 8, hipMemcpyDeviceToDevice));
            CK(hipMemcpy(x.z, z0, img * 4, hipMemcpyDeviceToDevice));
        }
        CK(hipMemcpy(y.state, x.state, 4 * spec * 8, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(y.z, x.z, img * 4, hipMemcpyDeviceToDevice));
        launch_v(0, fl, x.a);
        launch_v(1, fl, y.a);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        const double dz = diff(x.zin, y.zin, img * 4), ds = diff(x.state, y.state, 4 * spec * 8);
        printf("parity %-10s zin max|d|/max|x| %.2e, state %.2e\n", fln[fl], dz, ds);
        bad += !(dz <= 1e-6) || !(ds <= 1e-6);
        CK(hipMemcpy(x.z, x.zin, img * 4, hipMemcpyDeviceToDevice));  // the next step's z
    }
    if (bad && !(argc > 3 && !strcmp(argv[3], "noparity"))) {
        printf("FAIL: k_gal_reg differs from the chained path\n");
        return 1;
    }
    Bufs t = make(N, par, true);
    seed(t, N);
    const double img_b = L * L * 4.0, half_b = K * L * 8.0;
    const double gb[4] = {N * (2 * img_b + 5.5 * half_b) / 1e9, N * (2 * img_b + 4.5 * half_b) / 1e9,
                          N * (2 * img_b + 2.5 * half_b) / 1e9, N * (2 * img_b + 1.5 * half_b) / 1e9};
    {
        const float m5 = time_ms([&] { hipLaunchKernelGGL(k_stream<512>, dim3(N), dim3(512), 0, 0, t.a); }, reps);
        const float m10 = time_ms([&] { hipLaunchKernelGGL(k_stream<1024>, dim3(N), dim3(1024), 0, 0, t.a); }, reps);
        CK(hipGetLastError());
        printf("k_stream<512>  (MID bytes) N=%d  %.3f ms  %.2f TB/s\n", N, m5, gb[0] / m5);
        printf("k_stream<1024> (MID bytes) N=%d  %.3f ms  %.2f TB/s\n", N, m10, gb[0] / m10);
    }
    // KB_REV=1: consecutive launches alternate the galaxy order (Args::rev), as gd_admm_iter does
    const bool alt = getenv("KB_REV") && atoi(getenv("KB_REV"));
    for (int fl = 0; fl < 3; ++fl) {
        const float ms = time_ms([&] { if (alt) t.a.rev ^= 1; launch_v(1, fl, t.a); }, reps);
        CK(hipGetLastError());
        printf("k_gal_reg<256,%-5s> N=%d  %.3f ms  %.2f TB/s algorithmic (%.2f GB)\n", fln[fl], N, ms, gb[fl] / ms, gb[fl]);
    }
#if GD_FUSED_TRACE
    // per-phase durations of k_gal_reg<MID> (thread 0's s_memrealtime stamps, 100 MHz) at several batch sizes
    const char* names[] = {"start -> z loaded", "row FFTs", "slice A -> S + gather", "column A FFT + update",
                           "column A IFFT", "slice B -> S + gather", "column B", "I half 0", "I half 1 + drain"};
    for (int n : {32, 256, N}) {
        Args b = t.a;
        b.N = n;
        for (int v = 0; v < 2; ++v) {  // warm, then the traced launch
            CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
            hipLaunchKernelGGL((k_gal_reg<L>), dim3(n), dim3(512), 0, 0, b);
            CK(hipDeviceSynchronize());
        }
        std::vector<unsigned long long> h((size_t)n * 16);
        CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
        if (n == N) {  // raw stamps of the full batch for offline analysis
            FILE* f = fopen("gpurun_out/kreg_trace.bin", "wb");
            if (f) { fwrite(h.data(), 8, h.size(), f); fclose(f); }
        }
        printf("phase trace N=%d (mean us per workgroup):\n", n);
        double tot = 0;
        for (int k = 0; k < 9; ++k) {
            double s = 0;
            for (int i = 0; i < n; ++i) s += (double)(h[i * 16 + k + 1] - h[i * 16 + k]);
            s = s / n / 100.0;
            tot += s;
            printf("  %-26s %7.2f\n", names[k], s);
        }
        printf("  %-26s %7.2f\n", "whole workgroup", tot);
    }
#endif
    // the fused init (k_psf_rows<STATE> must have run: PSF compact rows in the U1 slot)
    {
        float* psf;
        const int h = 48;
        CK(hipMalloc(&psf, (size_t)N * h * h * 4));
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, psf, (size_t)N * h * h, 5u, 0.f, 1e-3f);
        Args b = t.a;
        b.y = t.z; b.psf = psf; b.psf_gstride = h * h; b.h = h; b.o2 = t.zin;
        const int bpg = (h / 2 + Geo<L>::LPB - 1) / Geo<L>::LPB;
        auto rows = [&] { hipLaunchKernelGGL((k_psf_rows<L, true>), dim3(N * bpg), dim3(256), 0, 0, b); };
        const float mr = time_ms(rows, reps);
        const float mi = time_ms([&] { rows(); hipLaunchKernelGGL((k_gal_reg_init<L>), dim3(N), dim3(512), 0, 0, b); }, reps);
        CK(hipGetLastError());
        const double gi = N * (2 * img_b + 2.5 * half_b + 2.0 * h * K * 8) / 1e9;
        printf("k_psf_rows<STATE> N=%d  %.3f ms; + k_gal_reg_init %.3f ms  %.2f TB/s algorithmic (%.2f GB)\n", N, mr, mi, gi / mi, gi);
        {  // FNV-1a of the init's outputs (zin, W~, G) over the first min(N, 64) galaxies: bitwise comparison across builds
            CK(hipDeviceSynchronize());
            const int ng = N < 64 ? N : 64;
            unsigned long long hsh = 1469598103934665603ull;
            auto fold = [&](const void* p, size_t words) {
                std::vector<unsigned> hb(words);
                CK(hipMemcpy(hb.data(), p, words * 4, hipMemcpyDeviceToHost));
                for (unsigned v : hb) { hsh ^= v; hsh *= 1099511628211ull; }
            };
            fold(b.o2, (size_t)ng * L * L);
            fold(b.s_w, (size_t)ng * K * L * 2);
            fold(b.s_g, (size_t)ng * K * L * 2);
            printf("init outputs fnv %016llx (first %d galaxies)\n", hsh, ng);
        }
#if GD_FUSED_TRACE
        const char* inames[] = {"start -> y loaded", "row FFTs", "A gather + park", "A: Y, OTF cols, update, IFFT",
                                "B gather", "B: Y, OTF cols, update, IFFT", "I half 0", "I half 1 (+ x0 row FFTs)",
                                "W: A gather + park", "W: A cols -> F(x0)", "W: B gather", "W: B cols -> F(x0)"};
        const int order[] = {0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11, 12};
        for (int n : {32, N}) {
            b.N = n;
            for (int v = 0; v < 2; ++v) {
                CK(hipMemset(tr, 0, (size_t)N * 16 * 8));
                rows();
                hipLaunchKernelGGL((k_gal_reg_init<L>), dim3(n), dim3(512), 0, 0, b);
                CK(hipDeviceSynchronize());
            }
            std::vector<unsigned long long> h2((size_t)n * 16);
            CK(hipMemcpy(h2.data(), tr, h2.size() * 8, hipMemcpyDeviceToHost));
            printf("init phase trace N=%d (mean us per workgroup):\n", n);
            // stamps: 0 start, 1 y, 2..5 INIT slices (TB = 2), 6, 7 I halves, 8 I end, 9..12 W slices, 13 end
            const int st[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13};
            double tot = 0;
            for (int k = 0; k < 13; ++k) {
                double s = 0;
                for (int i = 0; i < n; ++i) s += (double)(h2[i * 16 + st[k + 1]] - h2[i * 16 + st[k]]);
                s = s / n / 100.0;
                tot += s;
                const char* nm = k == 8 ? "I end -> W" : inames[k < 8 ? k : k - 1];
                printf("  %-30s %7.2f\n", nm, s);
            }
            printf("  %-30s %7.2f\n", "whole workgroup", tot);
            (void)order;
        }
#endif
    }
    return 0;
}
