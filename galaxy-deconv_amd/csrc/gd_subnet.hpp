// SubNet feature extractor (models/Unrolled_ADMM.py:77-84) as ONE kernel, one workgroup per galaxy.
//
//   |FFT2(pad128(psf))|^2 -> MaxPool2 -> [conv3x3+BN+ReLU] x2 -> MaxPool2 -> ... (4 Down blocks)
//   -> 16 x 8 x 8 = 1024 features (channel-major, the reference's .view(N, 1, 16*8*8) order)
//
// Input is the engine's half-spectrum OTF of the PSF at 128x128 (gd_psf_to_otf): a circular shift
// only changes phases, so |OTF|^2 equals |FFT2(F.pad(psf))|^2 of :79-83; the full 128 x 128 map is
// read through Hermitian symmetry |H(ky,kx)|^2 = |H(-ky,-kx)|^2.  BatchNorm (eval) is folded into
// the conv weights on the host.  Activations live in LDS (80 KiB: two workgroups per CU); a thread
// owns a 2 x 2 block of output pixels (one pixel in the 8 x 8 layers) and a block of its output
// channels in registers, so each input value is read once per channel block and the weights are
// wave-uniform (scalar loads, tap-major so channel pairs are SGPR pairs).
#pragma once
#include <hip/hip_runtime.h>

namespace gd {
namespace subnet {

// conv layer table: (cin, cout, spatial side)
constexpr int kCin[8] = {1, 4, 4, 8, 8, 16, 16, 16};
constexpr int kCout[8] = {4, 4, 8, 8, 16, 16, 16, 16};
constexpr int woff(int l) {  // offset of layer l's weights in the packed [w | b] array
    int o = 0;
    for (int i = 0; i < l; ++i) o += kCout[i] * kCin[i] * 9 + kCout[i];
    return o;
}
constexpr int kParams = woff(8);  // 9,196 floats
#ifndef GD_SN_THREADS
#define GD_SN_THREADS 512  // measured: 256 -> 512 threads per galaxy: 119 -> 74 us at 256 x 48^2, 927 -> 659 us at 4096
#endif
constexpr int kThreads = GD_SN_THREADS;
// Optional per-workgroup phase timestamps (tools/kbench_subnet.hip builds with GD_SN_TRACE=1).
#if GD_SN_TRACE
__device__ unsigned long long* g_sn_trace;
#define SN_TRACE(k) \
    if (tid == 0) g_sn_trace[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define SN_TRACE(k)
#endif
#ifndef GD_SN_QUAD
#define GD_SN_QUAD 1  // the non-pooled layers 0, 2, 4 in 2 x 2 blocks (0: one pixel per work item)
#endif
// Output-channel split of the 16-channel layers at 16^2 / 8^2 (layers 5, 6, 7: 64 work items per channel
// group).  Batched launches (two workgroups per CU, many rounds) cap it at 4 groups of 4 channels: half
// the waves idle in those layers, but each window read feeds twice the FMAs and the other workgroup
// fills the CU (features at 4096: 417 -> 393 us).  One round of workgroups (k_subnet_rhos_psf, <= 256
// galaxies, latency-bound) keeps 8 groups of 2 (42.8 -> 41.7 us at 256).  profiles/r02z_ksubnet_cs.txt
#ifndef GD_SN_CS_BATCHED
#define GD_SN_CS_BATCHED 4
#endif
constexpr int kCSBatched = GD_SN_CS_BATCHED, kCSOneRound = 64;
#ifndef GD_SN_CS4
#define GD_SN_CS4 4   // the same cap for layer 4 (8 -> 16 at 16^2) in the batched kernel: 400 -> 389 us
#endif
#ifndef GD_SN_CS23
#define GD_SN_CS23 64  // experiment: cap for layers 2, 3 (at 32^2) in the batched kernel
#endif
#ifndef GD_SN_UNROLL_PX
#define GD_SN_UNROLL_PX 2  // input channels per unrolled step: per-pixel layers
#endif
#ifndef GD_SN_UNROLL_Q
#define GD_SN_UNROLL_Q 2   // 2 x 2-block layers
#endif
// Row stride of the 16^2 stage's activations (layers 3 -> 4 -> 5).  A wave's 64 items are the 8 x 8 blocks
// of 2 x 2 outputs; with rows of 16 floats the 4 block rows in a 32-lane half start 32 floats apart, so
// their 4 x 4 window reads (ds_read_b32, bank (a/4) mod 32) hit the same 16 banks: 4-way conflicts.  A
// stride of 24 puts block rows 16 banks apart: 2-way window reads (the floor for same-parity word reads)
// and conflict-free float2 stores of layer 4 (rows 2 oy, 2 oy + 1 of a 16-lane group on disjoint banks).
// One-launch SubNet 41.4-42.0 -> 39.6-39.8 us at 256, batched features 384-387 -> 369-370 us at 4096
// (20: 40.1-40.3 / 373-375 us), rhos bit-identical (profiles/r03w_subnet_rowstride_ab.txt).
#ifndef GD_SN_RS16
#define GD_SN_RS16 24
#endif
constexpr int kRS16 = GD_SN_RS16;
#ifndef GD_SN_RS8P
#define GD_SN_RS8P 12  // row stride of the zero-haloed 8^2 stage (10 rows of 10 + pad) on the MFMA path
#endif
constexpr int kRS8P = GD_SN_RS8P;
constexpr int kRegionA = 16 * 16 * 16;  // floats: 64x64x1 input, then pooled stage outputs
constexpr int kRegionB = 4 * 64 * 64;   // floats: first conv of each stage

// Output channels are split over CS thread groups when a layer has fewer than 256 output pixels;
// a group is 64 consecutive work items, i.e. one wave, so its channel offset is wave-uniform and the
// weights come through scalar loads.
constexpr int csplit(int npix, int cout, int cmax = 64) {
    int c = 1;
    while (npix * c < kThreads && c < cout && c < cmax) c *= 2;
    return c;
}

// Weights are tap-major, [cin][3][3][cout] (then bias [cout]): the CPT output channels of one tap are
// contiguous, so one scalar load brings them and channel pairs feed packed FMAs straight from SGPR pairs
// (with the [cout][cin][3][3] layout the pairs were 9 floats apart: SGPR spills to VGPR lanes and moves).
__device__ __forceinline__ constexpr int wtap(int ci, int dy, int dx, int cout) { return ((ci * 3 + dy) * 3 + dx) * cout; }

// acc[k] = b[c0+k] + sum_ci,dy,dx w[ci][dy][dx][c0+k] in[ci][y+dy-1][x+dx-1]   (zero padding)
template <int CIN, int COUT, int CPT, int S, int RSI = S>
__device__ __forceinline__ void conv_pixel(const float* in, const float* __restrict__ w,
                                           const float* __restrict__ b, int c0, int y, int x, float (&acc)[CPT]) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) acc[k] = b[c0 + k];
#pragma unroll GD_SN_UNROLL_PX
    for (int ci = 0; ci < CIN; ++ci) {
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
            const int yy = y + dy - 1;
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                const int xx = x + dx - 1;
                const float v = (yy >= 0 && yy < S && xx >= 0 && xx < S) ? in[(ci * S + yy) * RSI + xx] : 0.f;
#pragma unroll
                for (int k = 0; k < CPT; ++k) acc[k] = fmaf(w[wtap(ci, dy, dx, COUT) + c0 + k], v, acc[k]);
            }
        }
    }
}

// conv3x3 + bias + ReLU (+ MaxPool2d(2) when POOL, i.e. the pool that opens the next Down block):
// in [CIN][S][S] -> out [COUT][S'][S'] (S' = S or S/2), LDS or global.  QUAD (always when POOL): a work
// item computes the 2 x 2 conv outputs of one block from one 4 x 4 input window, 16 LDS reads per input
// channel instead of 4 x 9 and 4 CPT independent accumulators.  Every output's fma order (bias, then
// ci, dy, dx) is conv_pixel's in both forms, so the features do not depend on the form.
// RSI / RSO: row strides of the input / output activations in LDS (>= S / S'), [c][y][RS]
template <int CIN, int COUT, int S, bool POOL, bool QUAD = POOL, int CMAX = 64, int RSI = S, int RSO = (POOL ? S / 2 : S),
          bool PADO = false>
__device__ __forceinline__ void conv_layer(const float* in, float* out, const float* __restrict__ w,
                                           const float* __restrict__ b, int tid) {
    static_assert(QUAD || !POOL, "the pooled layers compute 2 x 2 blocks");
    constexpr int SO = POOL ? S / 2 : S;
    static_assert(RSI >= S && RSO >= SO && RSO % 2 == 0, "row strides");
    constexpr int SI = QUAD ? S / 2 : S;  // work items per row
    constexpr int NITEM = SI * SI;
    constexpr int CS = csplit(NITEM, COUT, CMAX), CPT = COUT / CS;
    for (int it = tid; it < NITEM * CS; it += kThreads) {
        const int grp = it / NITEM, p = it - grp * NITEM;
        const int c0 = __builtin_amdgcn_readfirstlane(grp * CPT);
        const int oy = p / SI, ox = p - oy * SI;
        if constexpr (QUAD) {
            float acc[4][CPT];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < CPT; ++k) acc[q][k] = b[c0 + k];
            const int y0 = 2 * oy - 1, x0 = 2 * ox - 1;
#pragma unroll GD_SN_UNROLL_Q
            for (int ci = 0; ci < CIN; ++ci) {
                float win[4][4];
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const int yy = y0 + r, xx = x0 + c;
                        win[r][c] = (yy >= 0 && yy < S && xx >= 0 && xx < S) ? in[(ci * S + yy) * RSI + xx] : 0.f;
                    }
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                        for (int q = 0; q < 4; ++q)
#pragma unroll
                            for (int k = 0; k < CPT; ++k)
                                acc[q][k] = fmaf(w[wtap(ci, dy, dx, COUT) + c0 + k], win[(q >> 1) + dy][(q & 1) + dx],
                                                 acc[q][k]);
            }
            if constexpr (POOL) {
#pragma unroll
                for (int k = 0; k < CPT; ++k)  // ReLU outputs are >= 0
                    out[PADO ? ((c0 + k) * (SO + 2) + oy + 1) * RSO + ox + 1 : ((c0 + k) * SO + oy) * RSO + ox] =
                        fmaxf(fmaxf(fmaxf(0.f, acc[0][k]), fmaxf(0.f, acc[1][k])),
                              fmaxf(fmaxf(0.f, acc[2][k]), fmaxf(0.f, acc[3][k])));
            } else {
#pragma unroll
                for (int k = 0; k < CPT; ++k)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        *reinterpret_cast<float2*>(out + ((c0 + k) * S + 2 * oy + h) * RSO + 2 * ox) =
                            make_float2(fmaxf(acc[2 * h][k], 0.f), fmaxf(acc[2 * h + 1][k], 0.f));
            }
        } else {
            float res[CPT];
            conv_pixel<CIN, COUT, CPT, S, RSI>(in, w, b, c0, oy, ox, res);
#pragma unroll
            for (int k = 0; k < CPT; ++k) out[((c0 + k) * SO + oy) * RSO + ox] = fmaxf(res[k], 0.f);
        }
    }
}

// ---- the 16-output-channel layers (4, 5, 6, 7) on the matrix cores: v_mfma_f32_16x16x4_f32, an implicit GEMM
// D[pixel][cout] = bias + sum_k A[pixel][k] W[k][cout] with k = (ci, dy, dx) in conv_pixel's order.  The f32 MFMA
// is bit for bit a k-ordered fmaf chain (one rounding per product, cdna_hip_programming.md 'FP32-input MFMA'),
// so every output equals the VALU form's fma(w, v, acc) chain from the bias: the features, and the rhos, are
// bit-identical to conv_layer's (tests: test_subnet_fused_launch_bit_identical and the rhos against the PyTorch
// SubNet).  A 16-pixel tile is 4 blocks of 2 x 2 outputs; lane l (q = l >> 4, i = l & 15) holds A[i][4s + q]
// = the input at pixel i's window offset of k = 4s + q, and W[4s + q][l & 15] (the tap-major weights ARE
// W[k][cout]: one coalesced load per k-step); its accumulators D[4q + r][l & 15], r < 4, are block q's 2 x 2
// outputs of channel l & 15, so the 2 x 2 MaxPool is a max over the lane's own registers.  Inputs carry a
// one-pixel zero halo ([c][S + 2][RSI], interior at (y + 1, x + 1)): no bounds test per tap.  One k-step is
// one address add, one ds_read_b32 and one MFMA (the VALU form: 16 exec-masked window reads and scalar weight
// loads per input channel, waited with lgkmcnt(0)).
#ifndef GD_SN_MFMA
#define GD_SN_MFMA 1  // 0: the VALU conv_layer for layers 4-7 (bit-identical features; profiles/r04b_ksubnet_mfma_ab.txt)
#endif
typedef float sn_f4 __attribute__((ext_vector_type(4)));
template <int C, int S, int RS>
__device__ __forceinline__ void zero_halo(float* buf, int tid) {  // [C][S + 2][RS]: rows 0, S + 1 and columns 0, S + 1
    constexpr int PER = 4 * S + 4;
    for (int e = tid; e < C * PER; e += kThreads) {
        const int c = e / PER, u = e - c * PER;
        int y, x;
        if (u < S + 2) { y = 0; x = u; }
        else if (u < 2 * (S + 2)) { y = S + 1; x = u - (S + 2); }
        else { const int v = u - 2 * (S + 2); y = 1 + (v >> 1); x = (v & 1) ? S + 1 : 0; }
        buf[(c * (S + 2) + y) * RS + x] = 0.f;
    }
}
// in: [CIN][S + 2][RSI] (zero halo) -> conv3x3 + bias + ReLU (+ MaxPool2d(2) when POOL) ->
//   OUTF == 0: [16][SO + 2][RSO] with zero halo (SO = S or S / 2; the halo is written here too);
//   OUTF == 1: the feature vector [16][S][S] (the reference's .view(N, 1, 16 * 8 * 8) order)
template <int CIN, int S, bool POOL, int RSI, int RSO, int OUTF>
__device__ __forceinline__ void conv_mfma(const float* in, float* out, const float* __restrict__ w,
                                          const float* __restrict__ b, int tid) {
    constexpr int COUT = 16, K = CIN * 9, NS = K / 4, CHI = (S + 2) * RSI, SO = POOL ? S / 2 : S;
    constexpr int BPR = S / 2, NT = S * S / 16, NW = kThreads / 64, NC = NS / 9;
    static_assert(CIN % 4 == 0 && (S * S) % 16 == 0, "k-steps of 4 in chunks of 9 (4 input channels), tiles of 16 pixels");
    const int wave = tid >> 6, lane = tid & 63, q = lane >> 4, col = lane & 15;
    if constexpr (OUTF == 0) zero_halo<COUT, SO, RSO>(out, tid);  // disjoint from the interior written below
    if (wave >= NT) return;  // 8^2 layers: 4 tiles, waves 4-7 idle (no barrier inside)
    // k = 4 s + q: the (ci, dy, dx) pattern repeats every 9 k-steps (36 taps = 4 input channels), so a lane
    // keeps 9 window offsets and step s reads at off9[s % 9] + 4 CHI (s / 9) (the second term an immediate)
    int off9[9];
#pragma unroll
    for (int s = 0; s < 9; ++s) {
        const int k = 4 * s + q, ci = k / 9, r = k - 9 * ci, dy = r / 3, dx = r - 3 * dy;
        off9[s] = ci * CHI + dy * RSI + dx;
    }
    float bw[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) bw[s] = w[(4 * s + q) * COUT + col];
    const float bias = b[col];
    for (int t = wave; t < NT; t += NW) {
        // A row of this lane: pixel ia = lane & 15 of tile t (block ia >> 2, position ia & 3)
        const int ia = lane & 15, blk = 4 * t + (ia >> 2), by = blk / BPR, bx = blk - by * BPR;
        const int y = 2 * by + ((ia >> 1) & 1), x = 2 * bx + (ia & 1);
        const float* src = in + y * RSI + x;  // window origin in padded coordinates
        sn_f4 acc = {bias, bias, bias, bias};
        // software-pipelined: chunk c + 1's 9 reads are in flight while chunk c's 9 MFMAs issue
        float av[2][9];
#pragma unroll
        for (int s = 0; s < 9; ++s) av[0][s] = src[off9[s]];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c + 1 < NC) {
#pragma unroll
                for (int s = 0; s < 9; ++s) av[(c + 1) & 1][s] = src[off9[s] + 4 * CHI * (c + 1)];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < 9; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[c & 1][s], bw[9 * c + s], acc, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        // this lane's results: block (t, q), positions r = 0..3 (D row 4q + r), channel col
        const int ob = 4 * t + q, oby = ob / BPR, obx = ob - oby * BPR;
        if constexpr (POOL) {
            const float m = fmaxf(fmaxf(fmaxf(0.f, acc[0]), fmaxf(0.f, acc[1])), fmaxf(fmaxf(0.f, acc[2]), fmaxf(0.f, acc[3])));
            if constexpr (OUTF == 0) out[(col * (SO + 2) + oby + 1) * RSO + obx + 1] = m;
            else out[(col * SO + oby) * SO + obx] = m;
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int yy = 2 * oby + (r >> 1), xx = 2 * obx + (r & 1);
                const float v = fmaxf(acc[r], 0.f);
                if constexpr (OUTF == 0) out[(col * (SO + 2) + yy + 1) * RSO + xx + 1] = v;
                else out[(col * SO + yy) * SO + xx] = v;
            }
        }
    }
}

__device__ __forceinline__ float mag2(const float2* __restrict__ otf, int ky, int kx) {
    // otf: [65][128] half spectrum (kx-major); |H(ky,kx)|^2 for any kx via Hermitian symmetry
    if (kx > 64) {
        kx = 128 - kx;
        ky = (128 - ky) & 127;
    }
    const float2 h = otf[kx * 128 + ky];
    return h.x * h.x + h.y * h.y;
}

// The conv stack of galaxy g; the last layer writes the 1024 features to `out` (LDS or global).
// C5 / C67: caps on the output-channel split of layer 5 and layers 6, 7 (kCSBatched / kCSOneRound)
template <int C5, int C67>
__device__ __forceinline__ void conv_layers(const float* __restrict__ params, float* out, float* A, float* B, int tid);
__device__ __forceinline__ void conv_stack(const float2* __restrict__ otf128, const float* __restrict__ params,
                                           float* out, float* A, float* B, int g, int tid) {
    const float2* otf = otf128 + (size_t)g * 65 * 128;
    // Down(1,4): MaxPool2d(2) of |H|^2 (128x128) -> A[64][64]; pooled[i][j] = max |H|^2 over
    // rows ky = 2i, 2i+1 and columns kx = 2j, 2j+1.  Lanes take consecutive i (coalesced ky pairs).
    for (int p = tid; p < 64 * 64; p += kThreads) {
        const int j = p >> 6, i = p & 63;
        const float m = fmaxf(fmaxf(mag2(otf, 2 * i, 2 * j), mag2(otf, 2 * i + 1, 2 * j)),
                              fmaxf(mag2(otf, 2 * i, 2 * j + 1), mag2(otf, 2 * i + 1, 2 * j + 1)));
        A[i * 64 + j] = m;
    }
    __syncthreads();
    conv_layers<kCSBatched, kCSBatched>(params, out, A, B, tid);
}
// the four Down blocks from the pooled |H|^2 in A[64][64]
template <int C5, int C67>
__device__ __forceinline__ void conv_layers(const float* __restrict__ params, float* out, float* A, float* B, int tid) {
    const float* P = params;
#define GD_SN_LAYER(l, CI, CO, S, POOL, QUAD, IN, OUT, CMAX, RSI, RSO)                             \
    conv_layer<CI, CO, S, POOL, QUAD, CMAX, RSI, RSO>(IN, OUT, P + woff(l), P + woff(l) + CO * CI * 9, tid); \
    __syncthreads();                                                                             \
    SN_TRACE(3 + l);
    constexpr int R16 = kRS16;
    GD_SN_LAYER(0, 1, 4, 64, false, GD_SN_QUAD, A, B, 64, 64, 64)   // B[4][64][64]
    GD_SN_LAYER(1, 4, 4, 64, true, true, B, A, 64, 64, 32)          // A[4][32][32]   (+ MaxPool of Down(4,8))
    GD_SN_LAYER(2, 4, 8, 32, false, GD_SN_QUAD, A, B, (C5 < 64 ? GD_SN_CS23 : 64), 32, 32)   // B[8][32][32]
#if GD_SN_MFMA
    // layer 3 writes the 16^2 stage with a zero halo; layers 4-7 on the matrix cores (conv_mfma)
    constexpr int P16 = R16, P8 = kRS8P;
    static_assert(16 * 18 * P16 <= kRegionB && 8 * 18 * P16 <= kRegionA && 16 * 10 * P8 <= kRegionA, "padded stages");
    zero_halo<8, 16, P16>(A, tid);
    conv_layer<8, 8, 32, true, true, (C5 < 64 ? GD_SN_CS23 : 64), 32, P16, true>(B, A, P + woff(3), P + woff(3) + 8 * 8 * 9, tid);
    __syncthreads();
    SN_TRACE(6);
    conv_mfma<8, 16, false, P16, P16, 0>(A, B, P + woff(4), P + woff(4) + 16 * 8 * 9, tid);   // B[16][18][P16]
    __syncthreads();
    SN_TRACE(7);
    conv_mfma<16, 16, true, P16, P8, 0>(B, A, P + woff(5), P + woff(5) + 16 * 16 * 9, tid);   // A[16][10][P8]
    __syncthreads();
    SN_TRACE(8);
    conv_mfma<16, 8, false, P8, P8, 0>(A, B, P + woff(6), P + woff(6) + 16 * 16 * 9, tid);     // B[16][10][P8]
    __syncthreads();
    SN_TRACE(9);
    conv_mfma<16, 8, false, P8, P8, 1>(B, out, P + woff(7), P + woff(7) + 16 * 16 * 9, tid);   // features
    SN_TRACE(10);
#else
    GD_SN_LAYER(3, 8, 8, 32, true, true, B, A, (C5 < 64 ? GD_SN_CS23 : 64), 32, R16)         // A[8][16][R16]   (+ MaxPool of Down(8,16))
    GD_SN_LAYER(4, 8, 16, 16, false, GD_SN_QUAD, A, B, (C5 < 64 ? GD_SN_CS4 : 64), R16, R16) // B[16][16][R16]
    GD_SN_LAYER(5, 16, 16, 16, true, true, B, A, C5, R16, 8) // A[16][8][8]    (+ MaxPool of Down(16,16))
    GD_SN_LAYER(6, 16, 16, 8, false, false, A, B, C67, 8, 8)  // B[16][8][8]  (per pixel: 2 x 2 blocks would idle half the threads)
    // last conv of Down(16,16) straight to the feature vector [16][8][8]
    conv_layer<16, 16, 8, false, false, C67>(B, out, P + woff(7), P + woff(7) + 16 * 16 * 9, tid);
    SN_TRACE(10);
#endif
#undef GD_SN_LAYER
}

__global__ __launch_bounds__(kThreads) void k_subnet_features(const float2* __restrict__ otf128,
                                                             const float* __restrict__ params,
                                                             float* __restrict__ feat, int N) {
    __shared__ __attribute__((aligned(16))) float A[kRegionA];
    __shared__ __attribute__((aligned(16))) float B[kRegionB];
    const int g = blockIdx.x;
    if (g >= N) return;  // uniform per block; no barrier crossed
    conv_stack(otf128, params, feat + (size_t)g * 1024, A, B, g, threadIdx.x);
}

// ---- the same features straight from the PSF (h <= 64, even): |FFT2(pad128(psf))|^2 computed in the
// workgroup (the separate OTF128 row / column launches and their 65 x 128 complex spectrum per galaxy
// in HBM go away).  |FFT|^2 is invariant under circular shifts, so the PSF sits at the origin of the
// 128 x 128 grid instead of F.pad's centred placement (:79-81).  Rows: 32 lines of 8 lanes transform
// the packed row pairs (rows 2l + i 2l+1, zero beyond h); columns: 64 lines, line kx (< 64) one half-
// spectrum column (its rows split out of the packed pairs), line 0 columns 0 and 64 (both real) packed;
// |H|^2 of the 65 columns -> M [128][kMS], then MaxPool2 of the full map via Hermitian symmetry -> A.
// LDS (float2 units of the 80 KiB A | B union): exchange areas [0, 64 x 136), packed row spectra
// [4352, 8448), M (floats, rows of kMS) [4096, 4096 + 128 kMS), twiddles [10112, 10240); the conv stack
// overwrites them all.  Bank-conflict-free LDS traffic around M (64 banks): row stride kMS = 72 puts a
// wave's column-FFT results (lanes j + 8 line at rows j + 8 r, column line) in 64 distinct banks (the
// stride 65 shared 15), and the pool's lanes take consecutive output columns so its stores are
// contiguous (lanes on consecutive rows all hit one bank: 64-way).
constexpr int kPsfMaxH = 64;
constexpr int kMS = 72;
static_assert(4096 + 128 * kMS <= 2 * 10112, "M below the twiddles");
__device__ __forceinline__ void psf_pool(const float* __restrict__ psf, int h, float* AB, int tid) {
    constexpr int L = 128, F1 = 8, F2 = 16, XCH = F1 * (F2 + 1);
    float2* S2 = reinterpret_cast<float2*>(AB);
    float2* tw = S2 + 10112;
    float2* Z = S2 + 4352;
    float* M = AB + 4096;
    SN_TRACE(0);
    fill_twiddles<L>(tw, tid, kThreads);
    const int line = tid / F1, j = tid - line * F1;
    __syncthreads();
    if (line < kPsfMaxH / 2) {  // rows 2 line, 2 line + 1 (zero when >= h)
        float2 v[F2];
#pragma unroll
        for (int r = 0; r < F2; ++r) {
            const int c = j + F1 * r;
            const bool in = r < kPsfMaxH / F1 && 2 * line < h && c < h;  // r >= 8: compile-time zeros (h <= 64)
            v[r] = in ? make_float2(psf[(2 * line) * h + c], psf[(2 * line + 1) * h + c]) : make_float2(0.f, 0.f);
        }
        line_fft<L, false>(v, j, S2 + line * XCH, tw);
        __syncthreads();  // exchange areas -> packed spectra
#pragma unroll
        for (int r = 0; r < F2; ++r) Z[line * L + j + F1 * r] = v[r];
    } else {
        __syncthreads();
    }
    __syncthreads();
    // column kx = line (line 0: 0 and 64 packed); row i = j + 8 r
    float2 c[F2];
    const int kx = line, km = (L - kx) & (L - 1);
#pragma unroll
    for (int r = 0; r < F2; ++r) {
        const int i = j + F1 * r;
        float2 val = make_float2(0.f, 0.f);
        if (r < kPsfMaxH / F1 && i < h) {  // r >= 8: compile-time zeros (h <= 64)
            const float2* zp = Z + (i >> 1) * L;
            if (line == 0) {
                const float2 z0 = zp[0], z64 = zp[L / 2];
                val = (i & 1) ? make_float2(z0.y, z64.y) : make_float2(z0.x, z64.x);
            } else {
                const float2 zk = zp[kx], zm = zp[km];
                val = (i & 1) ? make_float2(0.5f * (zk.y + zm.y), 0.5f * (zm.x - zk.x))
                              : make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
            }
        }
        c[r] = val;
    }
    __syncthreads();  // packed spectra read -> exchange areas
    float2* my = S2 + line * XCH;
    line_fft<L, false>(c, j, my, tw);
    float m[F2], m64[F2];
    if (line == 0) {  // split C0 + i C64 (both real columns) through the line's own exchange area
#pragma unroll
        for (int r = 0; r < F2; ++r) my[j + F1 * r] = c[r];
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < F2; ++r) {
            const int ky = j + F1 * r;
            const float2 z = c[r], zm = my[(L - ky) & (L - 1)];
            const float2 c0 = make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
            const float2 c64 = make_float2(0.5f * (z.y + zm.y), 0.5f * (zm.x - z.x));
            m[r] = c0.x * c0.x + c0.y * c0.y;
            m64[r] = c64.x * c64.x + c64.y * c64.y;
        }
    } else {
#pragma unroll
        for (int r = 0; r < F2; ++r) m[r] = c[r].x * c[r].x + c[r].y * c[r].y;
    }
    __syncthreads();  // exchange areas -> M
    SN_TRACE(1);
#pragma unroll
    for (int r = 0; r < F2; ++r) {
        const int ky = j + F1 * r;
        M[ky * kMS + kx] = m[r];
        if (line == 0) M[ky * kMS + 64] = m64[r];
    }
    __syncthreads();
    // MaxPool2d(2) of the full 128 x 128 |H|^2 -> A[64][64] (as k_subnet_features' first stage)
    for (int p = tid; p < 64 * 64; p += kThreads) {
        const int ii = p >> 6, jj = p & 63;
        float mx = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            int ky = 2 * ii + (e & 1), kxx = 2 * jj + (e >> 1);
            if (kxx > 64) {
                kxx = 128 - kxx;
                ky = (128 - ky) & 127;
            }
            mx = e == 0 ? M[ky * kMS + kxx] : fmaxf(mx, M[ky * kMS + kxx]);
        }
        AB[ii * 64 + jj] = mx;
    }
    __syncthreads();
    SN_TRACE(2);
}

__global__ __launch_bounds__(kThreads) void k_subnet_features_psf(const float* __restrict__ psf, long long psf_gstride,
                                                                 int h, const float* __restrict__ params,
                                                                 float* __restrict__ feat, int N) {
    __shared__ __attribute__((aligned(16))) float AB[kRegionA + kRegionB];
    const int g = blockIdx.x;
    if (g >= N) return;  // uniform per block; no barrier crossed
    psf_pool(psf + (long long)g * psf_gstride, h, AB, threadIdx.x);
    conv_layers<kCSBatched, kCSBatched>(params, feat + (size_t)g * 1024, AB, AB + kRegionA, threadIdx.x);
}

// ---- the SubNet's MLP (models/Unrolled_ADMM.py:68-74, :85-86) over a batch of feature vectors:
//   h1 = ReLU(W1 [feat; alpha] + b1)  (1025 -> 64), h2 = ReLU(W2 h1 + b2)  (64 -> 64),
//   out = Softplus(W3 h2 + b3) + 1e-6  (64 -> n_out)
// kMlpG galaxies per 256-thread workgroup: thread (o, q) computes neuron o for galaxies q, q + 4, ...
// reading the transposed weights (one coalesced 256-byte row per input for the whole wave) once per
// workgroup - per galaxy a workgroup would re-read W1 (262 KB) through L2 for every galaxy.  fp32
// FMAs in input order (a summation order of its own: within rounding of the GEMMs it replaces).
// mlp: W1^T [1025][64] | b1 [64] | W2^T [64][64] | b2 [64] | W3^T [64][n_out] | b3 [n_out].
constexpr int kHidden = 64, kFeat = 1024, kMaxOut = 64, kMlpG = 8, kMlpThreads = 512;
constexpr int kMlpWaves = kMlpThreads / kHidden;  // layer 1: wave q sums inputs [q KQ, (q + 1) KQ)
constexpr int kMlpKQ = kFeat / kMlpWaves;
constexpr int mlp_param_count(int n_out) {
    return (kFeat + 1) * kHidden + kHidden + kHidden * kHidden + kHidden + kHidden * n_out + n_out;
}

__global__ __launch_bounds__(kMlpThreads) void k_subnet_mlp(const float* __restrict__ feat,
                                                           const float* __restrict__ mlp,
                                                           const float* __restrict__ alpha, long long alpha_stride,
                                                           float* __restrict__ rhos, int n_out, int N) {
    static_assert(kMlpG == kMlpWaves, "layers 2, 3: one galaxy per wave");
    __shared__ float X[kMlpG][kFeat + 1];
    __shared__ float H[2][kMlpG][kHidden];
    const int tid = threadIdx.x, g0 = blockIdx.x * kMlpG;
    const int ng = N - g0 < kMlpG ? N - g0 : kMlpG;
    for (int i = tid; i < kMlpG * kFeat; i += kMlpThreads) {
        const int gg = i / kFeat, f = i - gg * kFeat;
        X[gg][f] = gg < ng ? feat[(size_t)(g0 + gg) * kFeat + f] : 0.f;
    }
    if (tid < kMlpG) X[tid][kFeat] = tid < ng ? alpha[(long long)(g0 + tid) * alpha_stride] : 0.f;
    __syncthreads();
    const float* W1 = mlp;
    const float* b1 = W1 + (kFeat + 1) * kHidden;
    const float* W2 = b1 + kHidden;
    const float* b2 = W2 + kHidden * kHidden;
    const float* W3 = b2 + kHidden;
    const float* b3 = W3 + kHidden * n_out;
    const int o = tid % kHidden, q = tid / kHidden;  // q is wave-uniform
    {
        // layer 1: wave q sums inputs [KQ q, KQ q + KQ) (+ alpha, input 1024, for the last wave) for all
        // the workgroup's galaxies (W1 read once per workgroup, 8 loads in flight per lane); then the
        // waves' partial sums are added in a fixed order
        float part[kMlpG];
#pragma unroll
        for (int gg = 0; gg < kMlpG; ++gg) part[gg] = 0.f;
        const int i0 = q * kMlpKQ;
        float wv[kMlpKQ];  // this lane's W1 column slice, all loads issued before the first FMA
#pragma unroll
        for (int k = 0; k < kMlpKQ; ++k) wv[k] = W1[(i0 + k) * kHidden + o];
#pragma unroll
        for (int k = 0; k < kMlpKQ; ++k) {
#pragma unroll
            for (int gg = 0; gg < kMlpG; ++gg) part[gg] = fmaf(wv[k], X[gg][i0 + k], part[gg]);
        }
        if (q == kMlpWaves - 1) {
            const float w = W1[kFeat * kHidden + o];
#pragma unroll
            for (int gg = 0; gg < kMlpG; ++gg) part[gg] = fmaf(w, X[gg][kFeat], part[gg]);
        }
        float* P = &X[0][0];  // the inputs are consumed: partial sums [waves][G][64] reuse X
        __syncthreads();
#pragma unroll
        for (int gg = 0; gg < kMlpG; ++gg) P[(q * kMlpG + gg) * kHidden + o] = part[gg];
        __syncthreads();
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < kMlpWaves; ++w) v += P[(w * kMlpG + q) * kHidden + o];  // galaxy q
        H[0][q][o] = fmaxf(v + b1[o], 0.f);
    }
    __syncthreads();
    float acc = 0.f;
#pragma unroll 8
    for (int i = 0; i < kHidden; ++i) acc = fmaf(W2[i * kHidden + o], H[0][q][i], acc);
    H[1][q][o] = fmaxf(acc + b2[o], 0.f);
    __syncthreads();
    if (o < n_out) {
        acc = 0.f;
#pragma unroll 8
        for (int i = 0; i < kHidden; ++i) acc = fmaf(W3[i * n_out + o], H[1][q][i], acc);
        {
            const int gg = q;
            if (gg < ng) {
                const float v = acc + b3[o];
                // nn.Softplus(beta = 1, threshold = 20), then + 1e-6 (:86)
                rhos[(size_t)(g0 + gg) * n_out + o] = (v > 20.f ? v : log1pf(expf(v))) + 1e-6f;
            }
        }
    }
}

// ---- the batched MLP on the matrix cores (GD_MLP_MFMA): k_subnet_mlp's arithmetic as v_mfma_f32_16x16x4_f32
// chains, 16 galaxies (M) x 16 outputs (N) per tile.  Every sum keeps its order: layer 1's partial of wave w
// is the k-ordered chain over inputs [128 w, 128 w + 128) from 0 (wave 7 then adds the alpha input as one more
// k-step whose other three slots are 0 * 0), the 8 partials are added in wave order, layers 2 and 3 are chains
// over their 64 inputs from 0 - the f32 MFMA is a k-ordered fmaf chain, so the rhos are bit-identical to
// k_subnet_mlp's and to the one-launch k_subnet_rhos_psf's.  W1 is read once per 16 galaxies (k_subnet_mlp:
// per 8) and a wave's 4 N-tiles share each A read; 1/16 of k_subnet_mlp's instructions per product.
#ifndef GD_MLP_MFMA
#define GD_MLP_MFMA 1
#endif
constexpr int kMG = 16, kXLD = 1026;  // galaxies per workgroup; X row stride (2 mod 32: conflict-free A reads)
__global__ __launch_bounds__(kMlpThreads) void k_subnet_mlp_mfma(const float* __restrict__ feat,
                                                                const float* __restrict__ mlp,
                                                                const float* __restrict__ alpha, long long alpha_stride,
                                                                float* __restrict__ rhos, int n_out, int N) {
    static_assert(kMlpThreads == 512 && kHidden == 64 && kFeat == 1024, "8 waves x 128 inputs; 4 N-tiles of 16");
    __shared__ __attribute__((aligned(16))) float X[kMG * kXLD];  // [galaxy][input], then the layer-1 partials
    __shared__ float Hs[2][kMG][kHidden];
    const int tid = threadIdx.x, g0 = blockIdx.x * kMG;
    const int ng = N - g0 < kMG ? N - g0 : kMG;
    for (int i = tid; i < kMG * (kFeat / 2); i += kMlpThreads) {
        const int gg = i / (kFeat / 2), f2 = i - gg * (kFeat / 2);
        const float2 v = gg < ng ? reinterpret_cast<const float2*>(feat + (size_t)(g0 + gg) * kFeat)[f2] : make_float2(0.f, 0.f);
        *reinterpret_cast<float2*>(X + gg * kXLD + 2 * f2) = v;
    }
    if (tid < kMG) {
        X[tid * kXLD + kFeat] = tid < ng ? alpha[(long long)(g0 + tid) * alpha_stride] : 0.f;
        X[tid * kXLD + kFeat + 1] = 0.f;
    }
    __syncthreads();
    const float* W1 = mlp;
    const float* b1 = W1 + (kFeat + 1) * kHidden;
    const float* W2 = b1 + kHidden;
    const float* b2 = W2 + kHidden * kHidden;
    const float* W3 = b2 + kHidden;
    const float* b3 = W3 + kHidden * n_out;
    const int w = tid >> 6, lane = tid & 63, gi = lane & 15, qk = lane >> 4, col = lane & 15;
    // layer 1: wave w, inputs [128 w, 128 w + 128), all 64 outputs (4 N-tiles), chains from 0
    sn_f4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = sn_f4{0.f, 0.f, 0.f, 0.f};
    {
        constexpr int CH = 8, NCH = (kFeat / kMlpWaves) / 4 / CH;  // 32 k-steps per wave in chunks of 8
        const float* xa = X + gi * kXLD + 128 * w + qk;
        const float* wb = W1 + (size_t)(128 * w + qk) * kHidden + col;
        float bv[2][CH][4];
#pragma unroll
        for (int s = 0; s < CH; ++s)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) bv[0][s][nt] = wb[(4 * s) * kHidden + 16 * nt];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (c + 1 < NCH) {
#pragma unroll
                for (int s = 0; s < CH; ++s)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt) bv[(c + 1) & 1][s][nt] = wb[(4 * (CH * (c + 1) + s)) * kHidden + 16 * nt];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                const float a = xa[4 * (CH * c + s)];
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[c & 1][s][nt], acc[nt], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (w == kMlpWaves - 1) {  // the alpha input (k = 1024) as one k-step, the other slots 0 * 0
            const float a = qk == 0 ? X[gi * kXLD + kFeat] : 0.f;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float bb = qk == 0 ? W1[kFeat * kHidden + 16 * nt + col] : 0.f;
                acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb, acc[nt], 0, 0, 0);
            }
        }
    }
    __syncthreads();  // X read -> the partials P[w][g][o] reuse it
    float* P = X;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) P[(w * kMG + 4 * qk + r) * kHidden + 16 * nt + col] = acc[nt][r];
    __syncthreads();
    for (int e = tid; e < kMG * kHidden; e += kMlpThreads) {
        const int gg = e / kHidden, o = e - gg * kHidden;
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < kMlpWaves; ++ww) v += P[(ww * kMG + gg) * kHidden + o];
        Hs[0][gg][o] = fmaxf(v + b1[o], 0.f);
    }
    __syncthreads();
    // layer 2: wave w < 4 computes N-tile w, a chain over the 64 inputs from 0
    if (w < 4) {
        sn_f4 a2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kHidden / 4; ++s)
            a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(Hs[0][gi][4 * s + qk], W2[(4 * s + qk) * kHidden + 16 * w + col], a2, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) Hs[1][4 * qk + r][16 * w + col] = fmaxf(a2[r] + b2[16 * w + col], 0.f);
    }
    __syncthreads();
    // layer 3: n_out outputs in N-tiles of 16
    if (16 * w < n_out) {
        const int o = 16 * w + col;
        sn_f4 a3 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kHidden / 4; ++s)
            a3 = __builtin_amdgcn_mfma_f32_16x16x4f32(Hs[1][gi][4 * s + qk], o < n_out ? W3[(4 * s + qk) * n_out + o] : 0.f,
                                                      a3, 0, 0, 0);
        if (o < n_out) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gg = 4 * qk + r;
                if (gg < ng) {
                    const float v = a3[r] + b3[o];
                    // nn.Softplus(beta = 1, threshold = 20), then + 1e-6 (:86)
                    rhos[(size_t)(g0 + gg) * n_out + o] = (v > 20.f ? v : log1pf(expf(v))) + 1e-6f;
                }
            }
        }
    }
}

// ---- the whole SubNet of one galaxy in one workgroup (small batches): k_subnet_features_psf, then the MLP
// on the workgroup's own feature vector (in LDS), in k_subnet_mlp's summation order (wave q sums inputs
// [q KQ, (q + 1) KQ) in order, the 8 partial sums added in wave order, layers 2 and 3 in input order), so
// the rhos are bit-identical to the batched path.  Each workgroup reads W1 (262 KB) from L2 / the Infinity
// Cache: at a few hundred galaxies (one workgroup per CU) that costs ~2 us per galaxy, against a separate
// batched launch of 32 workgroups (18 us at 256 x 48^2).
static_assert(kThreads == kMlpThreads, "the fused kernel runs the MLP with the feature kernel's threads");
#ifndef GD_SN_MLP2
#define GD_SN_MLP2 1  // 0: the round-3 MLP of the one-launch SubNet (W1 slice loaded whole, W2 / W3 from L2 in the chains)
#endif
#ifndef GD_SN_WPE
#define GD_SN_WPE 4  // waves per SIMD the one-launch kernels are compiled for: two 512-thread workgroups per CU
#endif
#ifndef GD_SN_MLP2_CH
#define GD_SN_MLP2_CH 16  // W1 rows per chunk (two chunks in flight)
#endif
// a value the compiler cannot see through: loads addressed from it stay after this point (the W1 chunks
// were otherwise all hoisted to the MLP's start and spilled)
__device__ __forceinline__ int sn_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ float sn_opaquef(float v) {  // (and a chunk's FMAs complete before the next chunk)
    asm volatile("" : "+v"(v));
    return v;
}
// The kernels pass their own __restrict__ pointer arguments (read-only weights through a struct member
// lose the no-alias proof that lets them be scalar loads: the SubNet ran 43 -> 58 us at 256 that way).
__device__ __forceinline__ void rhos_body(const float* __restrict__ psf, long long psf_gstride, int h,
                                          const float* __restrict__ params, const float* __restrict__ mlp,
                                          const float* __restrict__ alpha, long long alpha_stride,
                                          float* __restrict__ rhos, int n_out, float* AB, int g, int tid) {
    psf_pool(psf + (long long)g * psf_gstride, h, AB, tid);
    float* X = AB;                 // features [1024] (region A is free once layer 6 has been read)
    float* P = AB + kRegionA;      // partial sums [8][64], then h1, h2 (region B, after layer 7 read it)
    conv_layers<kCSOneRound, kCSOneRound>(params, X, AB, AB + kRegionA, tid);
    __syncthreads();
    const float xa = alpha[(long long)g * alpha_stride];
    const float* W1 = mlp;
    const float* b1 = W1 + (kFeat + 1) * kHidden;
    const float* W2 = b1 + kHidden;
    const float* b2 = W2 + kHidden * kHidden;
    const float* W3 = b2 + kHidden;
    const float* b3 = W3 + kHidden * n_out;
    const int o = tid % kHidden, q = tid / kHidden;  // q is wave-uniform
#if GD_SN_MLP2
    // W2 and W3 are staged in region B above the partial sums by all 512 threads: their loads are issued with
    // layer 1's last W1 chunk, so they land while layer 1 computes, and layers 2 and 3 (wave 0, chains over
    // 64 inputs) read each lane's weight column from LDS in one batch instead of waiting on L2 every 8 inputs.  Layer 1 streams W1 in 4 chunks of 32
    // rows, chunk c + 1 in flight while chunk c's FMAs issue.  Every sum keeps its order.
    float* W2s = P + 1024;                 // [64][64]
    float* W3s = W2s + kHidden * kHidden;  // [64][n_out]
    constexpr int N2 = kHidden * kHidden / kThreads, N3 = kHidden * kMaxOut / kThreads;
    static_assert(N2 * kThreads == kHidden * kHidden && 1024 + kHidden * (kHidden + kMaxOut) <= kRegionB, "W2, W3 in region B");
    const int n3 = kHidden * n_out;
    float w2r[N2], w3r[N3], bo[3];
    {
        constexpr int CH = GD_SN_MLP2_CH, NCH = kMlpKQ / CH;
        const int i0 = q * kMlpKQ;
        const float* wp = W1 + (size_t)i0 * kHidden + o;
        float part = 0.f;
        float wb[2][CH];
        {
            const float* wc = wp + sn_opaque(0);
#pragma unroll
            for (int k = 0; k < CH; ++k) wb[0][k] = wc[k * kHidden];
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (c + 1 < NCH) {
                const float* wc = wp + sn_opaque(CH * (c + 1) * kHidden);
#pragma unroll
                for (int k = 0; k < CH; ++k) wb[(c + 1) & 1][k] = wc[k * kHidden];
            }
            if (c + 2 == NCH) {  // after the last W1 chunk: waiting for a chunk never waits for these
#pragma unroll
                for (int e = 0; e < N2; ++e) w2r[e] = W2[tid + e * kThreads];
#pragma unroll
                for (int e = 0; e < N3; ++e) w3r[e] = tid + e * kThreads < n3 ? W3[tid + e * kThreads] : 0.f;
                bo[0] = b1[o];
                bo[1] = b2[o];
                bo[2] = o < n_out ? b3[o] : 0.f;
            }
            __builtin_amdgcn_sched_barrier(0);
            const float* xc = X + i0 + sn_opaque(CH * c);  // (the LDS reads were hoisted whole as well)
#pragma unroll
            for (int k = 0; k < CH; ++k) part = fmaf(wb[c & 1][k], xc[k], part);
            part = sn_opaquef(part);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (q == kMlpWaves - 1) part = fmaf(W1[kFeat * kHidden + o], xa, part);
        P[q * kHidden + o] = part;
#pragma unroll
        for (int e = 0; e < N2; ++e) W2s[tid + e * kThreads] = w2r[e];
#pragma unroll
        for (int e = 0; e < N3; ++e)
            if (tid + e * kThreads < n3) W3s[tid + e * kThreads] = w3r[e];
    }
    __syncthreads();
    SN_TRACE(11);
    if (q == 0) {
        // layers 2 and 3 in wave 0: lane o holds h1[o] (h2[o]); input i of the chain is lane i's value, broadcast
        // with v_readlane; the 64 weights of the lane's output column come from LDS in one batch of reads
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < kMlpWaves; ++w) v += P[w * kHidden + o];
        const float h1 = fmaxf(v + bo[0], 0.f);
        float wc[kHidden];
#pragma unroll
        for (int i = 0; i < kHidden; ++i) wc[i] = W2s[i * kHidden + o];
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < kHidden; ++i)
            acc = fmaf(wc[i], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h1), i)), acc);
        const float h2 = fmaxf(acc + bo[1], 0.f);
        const int o3 = o < n_out ? o : 0;
#pragma unroll
        for (int i = 0; i < kHidden; ++i) wc[i] = W3s[i * n_out + o3];
        acc = 0.f;
#pragma unroll
        for (int i = 0; i < kHidden; ++i)
            acc = fmaf(wc[i], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h2), i)), acc);
        if (o < n_out) {
            const float v3 = acc + bo[2];
            // nn.Softplus(beta = 1, threshold = 20), then + 1e-6 (:86)
            rhos[(size_t)g * n_out + o] = (v3 > 20.f ? v3 : log1pf(expf(v3))) + 1e-6f;
        }
    }
    SN_TRACE(12);
#else
    {
        const int i0 = q * kMlpKQ;
        float wv[kMlpKQ];
#pragma unroll
        for (int k = 0; k < kMlpKQ; ++k) wv[k] = W1[(i0 + k) * kHidden + o];
        float part = 0.f;
#pragma unroll
        for (int k = 0; k < kMlpKQ; ++k) part = fmaf(wv[k], X[i0 + k], part);
        if (q == kMlpWaves - 1) part = fmaf(W1[kFeat * kHidden + o], xa, part);
        P[q * kHidden + o] = part;
    }
    __syncthreads();
    float* H1 = P + kMlpWaves * kHidden;
    float* H2 = H1 + kHidden;
    if (q == 0) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < kMlpWaves; ++w) v += P[w * kHidden + o];
        H1[o] = fmaxf(v + b1[o], 0.f);
        // layers 2 and 3 inside wave 0
        wave_lds_sync();  // H1 written and read by this wave only
        float acc = 0.f;
#pragma unroll 8
        for (int i = 0; i < kHidden; ++i) acc = fmaf(W2[i * kHidden + o], H1[i], acc);
        H2[o] = fmaxf(acc + b2[o], 0.f);
        wave_lds_sync();
        if (o < n_out) {
            acc = 0.f;
#pragma unroll 8
            for (int i = 0; i < kHidden; ++i) acc = fmaf(W3[i * n_out + o], H2[i], acc);
            const float v3 = acc + b3[o];
            // nn.Softplus(beta = 1, threshold = 20), then + 1e-6 (:86)
            rhos[(size_t)g * n_out + o] = (v3 > 20.f ? v3 : log1pf(expf(v3))) + 1e-6f;
        }
    }
    SN_TRACE(11);
#endif
}
__global__ __launch_bounds__(kThreads, GD_SN_WPE) void k_subnet_rhos_psf(const float* __restrict__ psf, long long psf_gstride,
                                                             int h, const float* __restrict__ params,
                                                             const float* __restrict__ mlp,
                                                             const float* __restrict__ alpha, long long alpha_stride,
                                                             float* __restrict__ rhos, int n_out, int N) {
    __shared__ __attribute__((aligned(16))) float AB[kRegionA + kRegionB];
    const int g = blockIdx.x;
    if (g >= N) return;  // uniform per block; no barrier crossed
    rhos_body(psf, psf_gstride, h, params, mlp, alpha, alpha_stride, rhos, n_out, AB, g, threadIdx.x);
}

}  // namespace subnet
}  // namespace gd
