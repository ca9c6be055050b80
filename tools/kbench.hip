// Standalone kernel microbenchmark (no torch): times engine kernels and variants on synthetic
// buffers of the benchmark shape (4096 x 256^2) with hipEvents, next to plain streaming kernels
// that calibrate the achievable HBM rate for the same byte counts and access widths.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kbench tools/kbench.hip && ./kbench
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"

#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_fill(float* p, size_t n, unsigned seed) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u + seed;
        x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
        p[i] = (x & 0xffffff) / float(0x1000000) - 0.5f;
    }
}

// streaming reference: read R arrays, write W arrays, float4 per lane, fully coalesced
template <int R, int Wn>
__global__ __launch_bounds__(256) void k_stream4(const float4* __restrict__ in, float4* __restrict__ out, size_t n4) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n4; i += stride) {
        float4 acc = make_float4(0, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            float4 v = in[r * n4 + i];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
#pragma unroll
        for (int w = 0; w < Wn; ++w) out[w * n4 + i] = acc;
    }
}

// copy variants for the achievable-bandwidth ceiling
typedef float f4v __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_u(const f4v* __restrict__ in, f4v* __restrict__ out, size_t n4) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n4) v[u] = NT ? __builtin_nontemporal_load(in + i) : in[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n4) {
            if (NT) __builtin_nontemporal_store(v[u], out + i);
            else out[i] = v[u];
        }
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
    constexpr int L = 256, K = L / 2 + 1;
    const size_t img = (size_t)N * L * L, spec = (size_t)N * K * L;
    float *y, *z, *zin;
    float2 *T, *state;
    CK(hipMalloc(&y, img * 4)); CK(hipMalloc(&z, img * 4)); CK(hipMalloc(&zin, img * 4));
    CK(hipMalloc(&T, 2 * spec * 8)); CK(hipMalloc(&state, 4 * spec * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, z, img, 1u);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)T, 4 * spec, 2u);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)state, 8 * spec, 3u);
    std::vector<float> ones(N, 1.0f);
    float* par;
    CK(hipMalloc(&par, N * 4));
    CK(hipMemcpy(par, ones.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());

    Args a;
    memset(&a, 0, sizeof(a));
    a.N = N; a.T = T; a.s_hh = (float*)state; a.s_g = state + spec / 2; a.s_u1 = a.s_g + spec; a.s_w = a.s_g + 2 * spec;
    a.y = y; a.a0 = z; a.o0 = zin;
    a.alpha = a.rho1 = a.rho2 = a.rho2n = GalScalar{par, 1};
    a.llh = GD_LLH_GAUSSIAN; a.first = 0; a.last = 0;
    using Gm = Geo<L>;
    const int cgrid = (N * K + Gm::LPB - 1) / Gm::LPB;
    const double half_gb = spec * 8 / 1e9, img_gb = img * 4 / 1e9;

    auto col = [&](auto var) {
        constexpr int V = decltype(var)::value;
        return time_ms([&] { hipLaunchKernelGGL((k_col<L, C_G_ITER, V>), dim3(cgrid), dim3(256), 0, 0, a); });
    };
    float t0 = col(std::integral_constant<int, 0>{});
    float t1 = col(std::integral_constant<int, 1>{});
    float t2 = col(std::integral_constant<int, 2>{});
    const double colgb = 8 * half_gb;
    printf("k_col<G_ITER>  prod %.3f ms (%.2f TB/s) | no-FFT %.3f ms (%.2f) | prefetch H,W %.3f ms (%.2f)\n",
           t0, colgb / t0, t1, colgb / t1, t2, colgb / t2);

    auto rows = [&](auto rbx) {
        constexpr int RBX = decltype(rbx)::value;
        using R = RowGeo<L, 1, RBX>;
        const int grid = N * (L / R::RB);
        float tf = time_ms([&] { hipLaunchKernelGGL((k_row_fwd<L, RF_ONE, RBX>), dim3(grid), dim3(R::THREADS), 0, 0, a); });
        float ti = time_ms([&] { hipLaunchKernelGGL((k_row_inv<L, RI_OUT1, RBX>), dim3(grid), dim3(R::THREADS), 0, 0, a); });
        printf("rows/block %3d (%4d thr, LDS %6d B): k_row_fwd<ONE> %.3f ms (%.2f TB/s) | k_row_inv<OUT1> %.3f ms (%.2f TB/s)\n",
               R::RB, R::THREADS, R::LDS * 8, tf, (img_gb + half_gb) / tf, ti, (img_gb + half_gb) / ti);
    };
    rows(std::integral_constant<int, 16>{});
    rows(std::integral_constant<int, 0>{});
    rows(std::integral_constant<int, 64>{});

    // calibration: same bytes as k_col (5 reads + 3 writes of a half spectrum) as float4 streams
    const size_t n4 = spec * 8 / 16;
    float ts = time_ms([&] { hipLaunchKernelGGL((k_stream4<5, 3>), dim3(8192), dim3(256), 0, 0,
                                                (const float4*)state, (float4*)T, n4 / 2); });
    printf("stream4 5R+3W (%.2f GB) %.3f ms (%.2f TB/s)\n", colgb / 2, ts, colgb / 2 / ts);
    float tc = time_ms([&] { hipLaunchKernelGGL((k_stream4<1, 1>), dim3(8192), dim3(256), 0, 0,
                                                (const float4*)state, (float4*)T, n4 * 2); });
    printf("copy float4 (%.2f GB) %.3f ms (%.2f TB/s)\n", 4 * half_gb, tc, 4 * half_gb / tc);
    // ---- full Gaussian iteration RF(z) -> C -> RI(zin): one pass over the batch vs chunks on S streams
    {
        const int rg1 = RowGeo<L, 1>::RB;
        auto launch_iter = [&](const Args& b, float2* Tb, hipStream_t st) {
            Args c = b;
            c.T = Tb;
            hipLaunchKernelGGL((k_row_fwd<L, RF_ONE>), dim3(c.N * (L / rg1)), dim3(RowGeo<L, 1>::THREADS), 0, st, c);
            hipLaunchKernelGGL((k_col<L, C_G_ITER>), dim3((c.N * K + Gm::LPB - 1) / Gm::LPB), dim3(256), 0, st, c);
            hipLaunchKernelGGL((k_row_inv<L, RI_OUT1>), dim3(c.N * (L / rg1)), dim3(RowGeo<L, 1>::THREADS), 0, st, c);
        };
        const double iter_gb = N * (2.0 * (L * L * 4) + 11.5 * (K * L * 8)) / 1e9;
        float tfull = time_ms([&] { launch_iter(a, T, 0); });
        printf("iteration, one pass   : %.3f ms (%.2f TB/s algorithmic)\n", tfull, iter_gb / tfull);
        const int SMAX = 4;
        hipStream_t str[SMAX];
        for (int i = 0; i < SMAX; ++i) CK(hipStreamCreateWithFlags(&str[i], hipStreamNonBlocking));
        hipEvent_t ev0, evs[SMAX];
        CK(hipEventCreateWithFlags(&ev0, hipEventDisableTiming));
        for (int i = 0; i < SMAX; ++i) CK(hipEventCreateWithFlags(&evs[i], hipEventDisableTiming));
        for (int S : {2, 3, 4})
            for (int G : {64, 96, 128, 160, 192}) {
                if ((size_t)S * G > (size_t)N) continue;
                float t = time_ms([&] {
                    CK(hipEventRecord(ev0, 0));
                    for (int i = 0; i < S; ++i) CK(hipStreamWaitEvent(str[i], ev0, 0));
                    for (int g0 = 0, c = 0; g0 < N; g0 += G, ++c) {
                        const int n = N - g0 < G ? N - g0 : G;
                        Args b = offset_args(a, g0, n, L);
                        launch_iter(b, T + (size_t)(c % S) * 2 * G * K * L, str[c % S]);
                    }
                    for (int i = 0; i < S; ++i) {
                        CK(hipEventRecord(evs[i], str[i]));
                        CK(hipStreamWaitEvent(0, evs[i], 0));
                    }
                });
                printf("iteration, chunks of %4d on %d streams: %.3f ms (%.2f TB/s algorithmic)\n", G, S, t, iter_gb / t);
            }
    }

    auto cu = [&](auto u, auto nt) {
        constexpr int U = decltype(u)::value;
        constexpr bool NT = decltype(nt)::value;
        const size_t n = n4 * 2;
        const int grid = (int)((n + 256 * U - 1) / (256 * U));
        float t = time_ms([&] { hipLaunchKernelGGL((k_copy_u<U, NT>), dim3(grid), dim3(256), 0, 0,
                                                   (const f4v*)state, (f4v*)T, n); });
        printf("copy x%d %s (%.2f GB) %.3f ms (%.2f TB/s)\n", U, NT ? "nt" : "  ", 4 * half_gb, t, 4 * half_gb / t);
    };
    cu(std::integral_constant<int, 1>{}, std::false_type{});
    cu(std::integral_constant<int, 4>{}, std::false_type{});
    cu(std::integral_constant<int, 8>{}, std::false_type{});
    cu(std::integral_constant<int, 4>{}, std::true_type{});
    return 0;
}
