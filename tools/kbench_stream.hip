// Streaming ceilings on MI355X (round 5 rewrite).  Two questions:
//  (1) what a plain HBM stream reaches with this build and this box: copy / read-only / write-only, 16-byte
//      accesses per lane, workgroup size T, loads in flight per thread U, grid (persistent multiples of the CU
//      count or one pass over the data), default or non-temporal (nt) loads and stores, random data;
//  (2) what the fused 256^2 iteration's per-galaxy byte mix reaches (z, |H|^2, G, U1, W~ in; U1, W~, zin out:
//      1,977,344 B per galaxy, 2 img + 5.5 half spectra), one workgroup per galaxy with k_gal_reg's LDS
//      footprint (one workgroup per CU), for the state in the engine's layout (four arrays, SoA) and in an
//      interleaved layout (a column's |H|^2, G, U1, W~ in one contiguous record, AoS), with the z read and
//      zin write either in their own phases (as k_gal_reg: z first, zin last) or spread over the galaxy.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/kbench_stream tools/kbench_stream.hip
//   tools/kbench_stream [N=4096] [reps=20]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int L = 256, K = L / 2 + 1;
constexpr size_t IMG = (size_t)L * L, SPEC = (size_t)K * L;

__global__ void k_fill(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u + seed;
        x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
        p[i] = (x & 0xffffff) / float(0x1000000);
    }
}

template <bool NT>
__device__ __forceinline__ f4v ld(const f4v* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4v* p, f4v v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// ---- (1) plain streams, grid-stride over n float4
template <int T, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(T) void k_copy(const f4v* a, f4v* b, size_t n) {
    for (size_t i0 = (size_t)blockIdx.x * T * U + threadIdx.x; i0 < n; i0 += (size_t)gridDim.x * T * U) {
        f4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i0 + u * T < n ? ld<NTL>(a + i0 + u * T) : f4v{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * T < n) st<NTS>(b + i0 + u * T, v[u] + 1.f);
    }
}
template <int T, int U, bool NTL>
__global__ __launch_bounds__(T) void k_read(const f4v* a, f4v* sink, size_t n) {
    f4v acc = {0, 0, 0, 0};
    for (size_t i0 = (size_t)blockIdx.x * T * U + threadIdx.x; i0 < n; i0 += (size_t)gridDim.x * T * U) {
        f4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i0 + u * T < n ? ld<NTL>(a + i0 + u * T) : f4v{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc.x == -1.f) sink[threadIdx.x] = acc;  // never true on the [0, 1) data: keeps the loads
}
template <int T, int U, bool NTS>
__global__ __launch_bounds__(T) void k_write(f4v* b, size_t n) {
    const f4v v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    for (size_t i0 = (size_t)blockIdx.x * T * U + threadIdx.x; i0 < n; i0 += (size_t)gridDim.x * T * U) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * T < n) st<NTS>(b + i0 + u * T, v);
    }
}

// ---- (2) the fused iteration's byte mix, one 512-thread workgroup per galaxy, k_gal_reg's LDS footprint.
// SoA: |H|^2 [N][K L] floats, G / U1 / W~ [N][K L] float2 (the engine's layout).
// AoS: per galaxy and 4-bin group b (b < K L / 4) one 112-byte record {|H|^2 x4, G x4, U1 x4, W~ x4}
//      = 7 float4; U1 / W~ rewritten in place.
// PH = 1: z loaded before the state, zin stored after it (k_gal_reg's phase order); PH = 0: interleaved.
template <bool AOS, bool NTS, int D>
__device__ __forceinline__ void mix_state(const f4v* hh, const f4v* G, f4v* Uu, f4v* W, f4v* rec, int tid) {
    constexpr int NS = SPEC / 4;  // 4-bin groups per galaxy
    constexpr int T = 512;
    static_assert(NS % T == 64, "tail");
    for (int i0 = tid; i0 < NS; i0 += T * D) {
        f4v h[D], g0[D], g1[D], u0[D], u1[D], w0[D], w1[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int i = min(i0 + d * T, NS - 1);
            if constexpr (AOS) {
                const f4v* r = rec + (size_t)i * 7;
                h[d] = r[0]; g0[d] = r[1]; g1[d] = r[2]; u0[d] = r[3]; u1[d] = r[4]; w0[d] = r[5]; w1[d] = r[6];
            } else {
                h[d] = hh[i]; g0[d] = G[2 * i]; g1[d] = G[2 * i + 1];
                u0[d] = Uu[2 * i]; u1[d] = Uu[2 * i + 1]; w0[d] = W[2 * i]; w1[d] = W[2 * i + 1];
            }
        }
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int i = i0 + d * T;
            if (i >= NS) break;
            const f4v a0 = u0[d] + g0[d] * h[d].x, a1 = u1[d] + g1[d] * h[d].y, b0 = w0[d] - g0[d], b1 = w1[d] - g1[d];
            if constexpr (AOS) {
                f4v* r = rec + (size_t)i * 7;
                st<NTS>(r + 3, a0); st<NTS>(r + 4, a1); st<NTS>(r + 5, b0); st<NTS>(r + 6, b1);
            } else {
                st<NTS>(Uu + 2 * i, a0); st<NTS>(Uu + 2 * i + 1, a1); st<NTS>(W + 2 * i, b0); st<NTS>(W + 2 * i + 1, b1);
            }
        }
    }
}
template <bool AOS, bool NTS, int D, bool PH>
__global__ __launch_bounds__(512) void k_mix(const float* z, float* zin, const float* hh, const float2* G, float2* Uu,
                                             float2* W, float* rec, int N) {
    __shared__ float pad[36000];  // 144 KB: one workgroup per CU, as k_gal_reg
    const int g = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) pad[g & 1023] = 0.f;
    const f4v* zs = reinterpret_cast<const f4v*>(z + g * IMG);
    f4v* zo = reinterpret_cast<f4v*>(zin + g * IMG);
    const f4v* h4 = reinterpret_cast<const f4v*>(hh + g * SPEC);
    const f4v* g4 = reinterpret_cast<const f4v*>(G + g * SPEC);
    f4v* u4 = reinterpret_cast<f4v*>(Uu + g * SPEC);
    f4v* w4 = reinterpret_cast<f4v*>(W + g * SPEC);
    f4v* r4 = reinterpret_cast<f4v*>(rec + g * SPEC * 7);
    constexpr int NZ = IMG / 4, PER = NZ / 512;  // 32 float4 per thread
    if constexpr (PH) {
        f4v v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) v[u] = zs[tid + 512 * u];
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < PER; ++u) s += v[u].x + v[u].w;
        pad[tid] = s;  // "row FFTs"
        mix_state<AOS, NTS, D>(h4, g4, u4, w4, r4, tid);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PER; ++u) st<NTS>(zo + tid + 512 * u, v[u] * pad[(tid + u) & 511]);
    } else {
        for (int u0 = 0; u0 < PER; u0 += 8) {
            f4v v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = zs[tid + 512 * (u0 + u)];
#pragma unroll
            for (int u = 0; u < 8; ++u) st<NTS>(zo + tid + 512 * (u0 + u), v[u] * 1.5f);
        }
        mix_state<AOS, NTS, D>(h4, g4, u4, w4, r4, tid);
    }
}

// ---- (3) k_gal_reg's own access pattern with no compute: 512 threads = 32 lines of 16 lanes, 4 lines per wave.
//   z: pair p = line + 32 q (q < 4), lane j loads rows 2p, 2p + 1 at j + 16 r (4-byte loads, 64 B per line and
//      instruction); zin stored the same way (phase I), after the state;
//   state: slice A (columns line + 32 u, u < 2) then slice B (64 + ...), per column 4 groups q of 4 bins x 16 lanes,
//      one 16-byte |H|^2 load and two each of G, U1, W~ per group, D groups in flight (fused_update4x's order);
//   LAYOUT 0: the engine's [kx][256] columns (soff_c / soff_h); 1: columns interleaved in quads of 4 (kx >> 2):
//      the 4 columns a wave holds (lines 4w .. 4w + 3) are adjacent per 256-byte group, so one wave instruction
//      reads 1 KiB contiguous.
template <int LAYOUT>
__device__ __forceinline__ int qoff_c(int kx, int m, int j) {  // float2 units, bins j + 16 (2m + e)
    if constexpr (LAYOUT == 0) return kx * 256 + 32 * m + 2 * j;
    else return (kx >> 2) * 1024 + 128 * m + 32 * (kx & 3) + 2 * j;
}
template <int LAYOUT>
__device__ __forceinline__ int qoff_h(int kx, int q, int j) {  // floats, bins j + 16 (4q + e)
    if constexpr (LAYOUT == 0) return kx * 256 + 64 * q + 4 * j;
    else return (kx >> 2) * 1024 + 256 * q + 64 * (kx & 3) + 4 * j;
}
template <int LAYOUT, int D, bool Z16>
__global__ __launch_bounds__(512) void k_regpat(const float* z, float* zin, const float* hh, const float2* G, float2* Uu,
                                                float2* W, int N) {
    __shared__ float pad[36000];
    const int g = blockIdx.x, tid = threadIdx.x, line = tid >> 4, j = tid & 15;
    if (tid == 0) pad[g & 1023] = 0.f;
    const float* zg = z + g * IMG;
    float* og = zin + g * IMG;
    float2 X[4][16];
    if constexpr (Z16) {  // the same bytes per thread as 16-byte loads (1 KiB per wave instruction)
        const f4v* z4 = reinterpret_cast<const f4v*>(zg);
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const f4v v = z4[tid + 512 * u];
            X[u >> 3][2 * (u & 7)] = make_float2(v[0], v[1]);
            X[u >> 3][2 * (u & 7) + 1] = make_float2(v[2], v[3]);
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float* r0 = zg + (size_t)(2 * (line + 32 * q)) * 256 + j;
#pragma unroll
            for (int r = 0; r < 16; ++r) X[q][r] = make_float2(r0[16 * r], r0[256 + 16 * r]);
        }
    }
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc += X[q][r].x - X[q][r].y;
    pad[tid] = acc;
    const size_t gb = (size_t)g * SPEC;
    const float* hg = hh + gb;
    const float2 *Gg = G + gb;
    float2 *Ug = Uu + gb, *Wg = W + gb;
    for (int slice = 0; slice < 2; ++slice) {
        __syncthreads();
        constexpr int NG = 8;  // 2 columns x 4 groups
        f4v h[NG], g0[NG], g1[NG], u0[NG], u1[NG], w0[NG], w1[NG];
        auto load = [&](int t) {
            const int kx = 64 * slice + line + 32 * (t >> 2), q = t & 3;
            h[t] = *reinterpret_cast<const f4v*>(hg + qoff_h<LAYOUT>(kx, q, j));
            g0[t] = *reinterpret_cast<const f4v*>(Gg + qoff_c<LAYOUT>(kx, 2 * q, j));
            g1[t] = *reinterpret_cast<const f4v*>(Gg + qoff_c<LAYOUT>(kx, 2 * q + 1, j));
            u0[t] = *reinterpret_cast<const f4v*>(Ug + qoff_c<LAYOUT>(kx, 2 * q, j));
            u1[t] = *reinterpret_cast<const f4v*>(Ug + qoff_c<LAYOUT>(kx, 2 * q + 1, j));
            w0[t] = *reinterpret_cast<const f4v*>(Wg + qoff_c<LAYOUT>(kx, 2 * q, j));
            w1[t] = *reinterpret_cast<const f4v*>(Wg + qoff_c<LAYOUT>(kx, 2 * q + 1, j));
        };
#pragma unroll
        for (int t = 0; t < D; ++t) load(t);
#pragma unroll
        for (int t = 0; t < NG; ++t) {
            const int kx = 64 * slice + line + 32 * (t >> 2), q = t & 3;
            st<true>(reinterpret_cast<f4v*>(Ug + qoff_c<LAYOUT>(kx, 2 * q, j)), u0[t] + g0[t] * h[t].x);
            st<true>(reinterpret_cast<f4v*>(Ug + qoff_c<LAYOUT>(kx, 2 * q + 1, j)), u1[t] + g1[t] * h[t].y);
            st<true>(reinterpret_cast<f4v*>(Wg + qoff_c<LAYOUT>(kx, 2 * q, j)), w0[t] - g0[t]);
            st<true>(reinterpret_cast<f4v*>(Wg + qoff_c<LAYOUT>(kx, 2 * q + 1, j)), w1[t] - g1[t]);
            if (t + D < NG) load(t + D);
        }
    }
    __syncthreads();
    const float s = pad[(tid + 1) & 511];
    if constexpr (Z16) {
        f4v* o4 = reinterpret_cast<f4v*>(og);
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const float2 a = X[u >> 3][2 * (u & 7)], b = X[u >> 3][2 * (u & 7) + 1];
            st<true>(o4 + tid + 512 * u, f4v{a.x * s, a.y * s, b.x * s, b.y * s});
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float* o = og + (size_t)(2 * (line + 32 * q)) * 256 + j;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                __builtin_nontemporal_store(X[q][r].x * s, o + 16 * r);
                __builtin_nontemporal_store(X[q][r].y * s, o + 256 + 16 * r);
            }
        }
    }
}

// ---- timing: median of 5 timed blocks of reps launches each
template <typename F>
float time_ms(F&& f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int k = 0; k < 5; ++k) {
        CK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i) f();
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        v.push_back(ms / reps);
    }
    std::sort(v.begin(), v.end());
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
    return v[2];
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096, reps = argc > 2 ? atoi(argv[2]) : 20;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // (1) plain streams over 4 GiB per buffer
    {
        const size_t n = (size_t)1 << 28;  // float4 = 4 GiB
        f4v *a, *b, *sink;
        CK(hipMalloc(&a, n * 16)); CK(hipMalloc(&b, n * 16)); CK(hipMalloc(&sink, 1 << 16));
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (float*)a, n * 4, 1u);
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (float*)b, n * 4, 2u);
        CK(hipDeviceSynchronize());
        const double gb1 = n * 16 / 1e9;
#define COPY(T, U, NTL, NTS, grid)                                                                                   \
    {                                                                                                                \
        const int gr = (grid) > 0 ? (grid) : (int)((n + (size_t)T * U - 1) / ((size_t)T * U));                       \
        const float ms = time_ms([&] { hipLaunchKernelGGL((k_copy<T, U, NTL, NTS>), dim3(gr), dim3(T), 0, 0, a, b, n); }, reps); \
        CK(hipGetLastError());                                                                                       \
        printf("copy  T=%4d U=%2d ntl=%d nts=%d grid=%7d  %.3f ms  %.3f TB/s (read+write)\n", T, U, NTL, NTS, gr, ms, 2 * gb1 / ms); \
    }
#define READ(T, U, NTL, grid)                                                                                        \
    {                                                                                                                \
        const int gr = (grid) > 0 ? (grid) : (int)((n + (size_t)T * U - 1) / ((size_t)T * U));                       \
        const float ms = time_ms([&] { hipLaunchKernelGGL((k_read<T, U, NTL>), dim3(gr), dim3(T), 0, 0, a, sink, n); }, reps); \
        CK(hipGetLastError());                                                                                       \
        printf("read  T=%4d U=%2d ntl=%d       grid=%7d  %.3f ms  %.3f TB/s\n", T, U, NTL, gr, ms, gb1 / ms);      \
    }
#define WRITE(T, U, NTS, grid)                                                                                       \
    {                                                                                                                \
        const int gr = (grid) > 0 ? (grid) : (int)((n + (size_t)T * U - 1) / ((size_t)T * U));                       \
        const float ms = time_ms([&] { hipLaunchKernelGGL((k_write<T, U, NTS>), dim3(gr), dim3(T), 0, 0, b, n); }, reps); \
        CK(hipGetLastError());                                                                                       \
        printf("write T=%4d U=%2d       nts=%d grid=%7d  %.3f ms  %.3f TB/s\n", T, U, NTS, gr, ms, gb1 / ms);      \
    }
        const int r1 = reps / 4 > 2 ? reps / 4 : 2;
        (void)r1;
        COPY(256, 4, false, false, 0) COPY(256, 8, false, false, 0) COPY(256, 16, false, false, 0)
        COPY(512, 4, false, false, 0) COPY(1024, 4, false, false, 0)
        COPY(256, 4, false, false, cus) COPY(256, 8, false, false, cus) COPY(256, 8, false, false, 2 * cus)
        COPY(256, 8, false, false, 4 * cus) COPY(256, 8, false, false, 8 * cus) COPY(512, 8, false, false, 4 * cus)
        COPY(1024, 8, false, false, 2 * cus) COPY(1024, 16, false, false, cus)
        COPY(256, 4, false, true, 0) COPY(256, 8, false, true, 0) COPY(256, 8, false, true, 4 * cus)
        COPY(256, 4, true, true, 0) COPY(256, 8, true, true, 4 * cus) COPY(256, 4, true, false, 0)
        READ(256, 4, false, 0) READ(256, 8, false, 0) READ(256, 8, false, 4 * cus) READ(512, 8, false, 4 * cus)
        READ(256, 16, false, 2 * cus) READ(256, 8, true, 0) READ(256, 8, true, 4 * cus)
        WRITE(256, 4, false, 0) WRITE(256, 8, false, 0) WRITE(256, 8, false, 4 * cus) WRITE(256, 4, true, 0)
        WRITE(256, 8, true, 4 * cus)
        CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(sink));
    }
    // (2) the fused iteration's byte mix
    {
        float *z, *zin, *hh, *rec;
        float2 *G, *Uu, *W;
        CK(hipMalloc(&z, N * IMG * 4)); CK(hipMalloc(&zin, N * IMG * 4)); CK(hipMalloc(&hh, N * SPEC * 4));
        CK(hipMalloc(&G, N * SPEC * 8)); CK(hipMalloc(&Uu, N * SPEC * 8)); CK(hipMalloc(&W, N * SPEC * 8));
        CK(hipMalloc(&rec, N * SPEC * 7 * 4 + 64));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, z, N * IMG, 3u);
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, hh, N * SPEC, 4u);
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)G, N * SPEC * 2, 5u);
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)Uu, N * SPEC * 2, 6u);
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)W, N * SPEC * 2, 7u);
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, rec, N * SPEC * 7, 8u);
        CK(hipDeviceSynchronize());
        const double gb = N * (2.0 * IMG * 4 + 5.5 * SPEC * 8) / 1e9;
#define MIX(AOS, NTS, D, PH)                                                                                         \
    {                                                                                                                \
        const float ms = time_ms([&] { hipLaunchKernelGGL((k_mix<AOS, NTS, D, PH>), dim3(N), dim3(512), 0, 0, z, zin, hh, G, Uu, W, rec, N); }, reps); \
        CK(hipGetLastError());                                                                                       \
        printf("mix aos=%d nts=%d D=%d phased=%d N=%d  %.3f ms  %.3f TB/s (%.3f GB)\n", AOS, NTS, D, PH, N, ms, gb / ms, gb); \
    }
        MIX(false, false, 1, true) MIX(false, false, 2, true) MIX(false, false, 4, true)
        MIX(false, true, 1, true) MIX(false, true, 2, true) MIX(false, true, 4, true)
        MIX(true, false, 2, true) MIX(true, true, 1, true) MIX(true, true, 2, true) MIX(true, true, 4, true)
        MIX(false, true, 2, false) MIX(true, true, 2, false)
#define REGPAT(LAY, D, Z16)                                                                                          \
    {                                                                                                                \
        const float ms = time_ms([&] { hipLaunchKernelGGL((k_regpat<LAY, D, Z16>), dim3(N), dim3(512), 0, 0, z, zin, hh, G, Uu, W, N); }, reps); \
        CK(hipGetLastError());                                                                                       \
        printf("k_gal_reg pattern layout=%d D=%d z16=%d N=%d  %.3f ms  %.3f TB/s (%.3f GB)\n", LAY, D, Z16, N, ms, gb / ms, gb); \
    }
        REGPAT(0, 2, false) REGPAT(0, 4, false) REGPAT(1, 2, false) REGPAT(1, 4, false) REGPAT(0, 2, true) REGPAT(1, 2, true)
        REGPAT(1, 8, true)
    }
    return 0;
}
