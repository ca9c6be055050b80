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
    a.N = N; a.T = T; a.otf = state; a.s_yal = state + spec; a.s_u1 = state + 2 * spec; a.s_w = state + 3 * spec;
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

    const int rg1 = N * (L / RowGeo<L, 1>::RB);
    float tf = time_ms([&] { hipLaunchKernelGGL((k_row_fwd<L, RF_ONE>), dim3(rg1), dim3(RowGeo<L, 1>::THREADS), 0, 0, a); });
    float ti = time_ms([&] { hipLaunchKernelGGL((k_row_inv<L, RI_OUT1>), dim3(rg1), dim3(RowGeo<L, 1>::THREADS), 0, 0, a); });
    printf("k_row_fwd<ONE> %.3f ms (%.2f TB/s) | k_row_inv<OUT1> %.3f ms (%.2f TB/s)\n",
           tf, (img_gb + half_gb) / tf, ti, (img_gb + half_gb) / ti);

    // calibration: same bytes as k_col (5 reads + 3 writes of a half spectrum) as float4 streams
    const size_t n4 = spec * 8 / 16;
    float ts = time_ms([&] { hipLaunchKernelGGL((k_stream4<5, 3>), dim3(8192), dim3(256), 0, 0,
                                                (const float4*)state, (float4*)T, n4 / 2); });
    printf("stream4 5R+3W (%.2f GB) %.3f ms (%.2f TB/s)\n", colgb / 2, ts, colgb / 2 / ts);
    float tc = time_ms([&] { hipLaunchKernelGGL((k_stream4<1, 1>), dim3(8192), dim3(256), 0, 0,
                                                (const float4*)state, (float4*)T, n4 * 2); });
    printf("copy float4 (%.2f GB) %.3f ms (%.2f TB/s)\n", 4 * half_gb, tc, 4 * half_gb / tc);
    return 0;
}
