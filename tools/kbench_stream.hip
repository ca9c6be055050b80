// Streaming ceiling of the fused iteration's per-galaxy byte mix (z, |H|^2, G, U1, W~ in; U1, W~, zin out:
// 1,977,344 B per galaxy at 256^2) for one workgroup per CU (LDS padded like k_gal_reg), as a function of
// the 16-byte loads each thread keeps in flight (U) and the workgroup size (T), and for a pure copy.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/kbench_stream tools/kbench_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int L = 256, K = L / 2 + 1;
constexpr size_t IMG = (size_t)L * L, SPEC = (size_t)K * L;

template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void k_mix(const float* z, float* zin, const float* hh, const float2* G, float2* Uu,
                                           float2* W, int N) {
    __shared__ float pad[35000];
    if (threadIdx.x == 0) pad[0] = 0.f;
    for (int g = blockIdx.x; g < N; g += gridDim.x) {
        const f4v* zs = reinterpret_cast<const f4v*>(z + g * IMG);
        f4v* zo = reinterpret_cast<f4v*>(zin + g * IMG);
        constexpr int NZ = IMG / 4;
        static_assert(NZ % (T * U) == 0, "image loop is exact");
        for (int i0 = threadIdx.x; i0 < NZ; i0 += T * U) {
            f4v v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = zs[i0 + u * T];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (NT) __builtin_nontemporal_store(v[u] * 1.5f, zo + i0 + u * T);
                else zo[i0 + u * T] = v[u] * 1.5f;
            }
        }
        const f4v* h4 = reinterpret_cast<const f4v*>(hh + g * SPEC);
        const f4v* g4 = reinterpret_cast<const f4v*>(G + g * SPEC);
        f4v* u4 = reinterpret_cast<f4v*>(Uu + g * SPEC);
        f4v* w4 = reinterpret_cast<f4v*>(W + g * SPEC);
        constexpr int NS = SPEC / 4;  // 4-bin groups: 1 f4v of |H|^2, 2 f4v each of G, U1, W~
        constexpr int UU = U / 4 > 0 ? U / 4 : 1;
        for (int i0 = threadIdx.x; i0 < NS; i0 += T * UU) {
            f4v h[UU], gg[UU][2], uu[UU][2], ww[UU][2];
#pragma unroll
            for (int u = 0; u < UU; ++u) {
                const int i = i0 + u * T < NS ? i0 + u * T : NS - 1;  // clamped: the tail re-reads, no write below
                h[u] = h4[i];
                gg[u][0] = g4[2 * i]; gg[u][1] = g4[2 * i + 1];
                uu[u][0] = u4[2 * i]; uu[u][1] = u4[2 * i + 1];
                ww[u][0] = w4[2 * i]; ww[u][1] = w4[2 * i + 1];
            }
#pragma unroll
            for (int u = 0; u < UU; ++u) {
                const int i = i0 + u * T;
                if (i >= NS) break;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const f4v a = uu[u][e] + gg[u][e] * h[u].x, b = ww[u][e] - gg[u][e];
                    if (NT) { __builtin_nontemporal_store(a, u4 + 2 * i + e); __builtin_nontemporal_store(b, w4 + 2 * i + e); }
                    else { u4[2 * i + e] = a; w4[2 * i + e] = b; }
                }
            }
        }
    }
}
template <int T, int U>
__global__ __launch_bounds__(T) void k_copy(const f4v* a, f4v* b, size_t n) {
    for (size_t i0 = (size_t)blockIdx.x * T * U + threadIdx.x; i0 < n; i0 += (size_t)gridDim.x * T * U) {
        f4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i0 + u * T < n ? a[i0 + u * T] : f4v{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) if (i0 + u * T < n) b[i0 + u * T] = v[u] + 1.f;
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
    const int N = argc > 1 ? atoi(argv[1]) : 4096, reps = 20;
    float *z, *zin, *hh; float2 *G, *Uu, *W;
    CK(hipMalloc(&z, N * IMG * 4)); CK(hipMalloc(&zin, N * IMG * 4)); CK(hipMalloc(&hh, N * SPEC * 4));
    CK(hipMalloc(&G, N * SPEC * 8)); CK(hipMalloc(&Uu, N * SPEC * 8)); CK(hipMalloc(&W, N * SPEC * 8));
    CK(hipMemset(z, 0, N * IMG * 4)); CK(hipMemset(hh, 0, N * SPEC * 4)); CK(hipMemset(G, 0, N * SPEC * 8));
    CK(hipMemset(Uu, 0, N * SPEC * 8)); CK(hipMemset(W, 0, N * SPEC * 8));
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double gb = N * (2.0 * IMG * 4 + 5.5 * SPEC * 8) / 1e9;
#define RUN(T, U, NT, grid)                                                                               \
    {                                                                                                     \
        const float ms = time_ms([&] { hipLaunchKernelGGL((k_mix<T, U, NT>), dim3(grid), dim3(T), 0, 0, z, zin, hh, G, Uu, W, N); }, reps); \
        CK(hipGetLastError());                                                                           \
        printf("mix T=%4d U=%2d nt=%d grid=%5d  %.3f ms  %.2f TB/s\n", T, U, NT, grid, ms, gb / ms);        \
    }
    RUN(512, 4, false, N) RUN(512, 8, false, N) RUN(512, 16, false, N)
    RUN(512, 4, false, cus) RUN(512, 8, false, cus) RUN(512, 16, false, cus)
    RUN(512, 8, true, cus) RUN(512, 16, true, cus)
    RUN(1024, 8, false, cus) RUN(1024, 16, false, cus)
    RUN(256, 16, false, cus)
    {
        const size_t n = N * IMG / 4 * 4;  // 4 images' worth
        f4v *a, *b;
        CK(hipMalloc(&a, n * 16)); CK(hipMalloc(&b, n * 16)); CK(hipMemset(a, 0, n * 16));
        for (int grid : {cus, cus * 4, 8192}) {
            const float ms = time_ms([&] { hipLaunchKernelGGL((k_copy<256, 8>), dim3(grid), dim3(256), 0, 0, a, b, n); }, reps);
            printf("copy T=256 U=8 grid=%5d  %.3f ms  %.2f TB/s (read+write)\n", grid, ms, 2.0 * n * 16 / 1e9 / ms);
        }
    }
    return 0;
}
