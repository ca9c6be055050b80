// galaxy-deconv_amd: MI355X-native spectral engine for unrolled PnP-ADMM deconvolution.
//
// Three streaming kernels per 2D spectral round trip, all fp32:
//   k_row_fwd  (RF)  : per block RB rows of one galaxy (of one or two images).  Two adjacent rows
//                      of the same image are packed as one complex line (even row = Re, odd = Im),
//                      length-L FFT along the row inside one wave, split into the two rows' half
//                      spectra (kx = 0..L/2) and stored TRANSPOSED to the workspace
//                      T[N][2][K][L] (K = L/2+1) so the column pass reads contiguous columns.
//                      Mode-specific producers fuse the preceding elementwise work (z - u1, PSF
//                      placement + circular shift, max(y,0)/alpha, ...).
//   k_col      (C)  : per line one (galaxy, kx) column of each image: column FFTs, the fused
//                      spectral operator (X-update divide, Wiener divide, OTF capture, conv
//                      multiply), inverse column FFTs, stored back in place.
//   k_row_inv  (RI) : per block RB rows: Hermitian extension of row-pair half spectra, inverse row
//                      FFT, result image staged in LDS, then the fused elementwise sink with
//                      16-byte coalesced accesses (dual updates, V step, next denoiser input, output).
//   k_row_invfwd (RIF): RI + a pointwise nonlinearity + RF of the result in one kernel (clamp in
//                      init_l2, Richardson-Lucy ratio / multiplicative update).
//
// Reference mapping (paths relative to the reference root):
//   psf_to_otf          utils/utils_torch.py:79-92      -> RF_PSF*, C_OTF*
//   conv_fft_batch      utils/utils_torch.py:46-50      -> RF_ONE, C_CONV[C], RI_OUT1
//   init_l2             models/Unrolled_ADMM.py:170-175 -> RF_PSF_Y, C_OTF_INIT, RIF_CLAMP, C_CONV, RI_INIT
//   ADMM loop body      models/Unrolled_ADMM.py:199-214 -> RF_ITER, C_ITER, RI_ITER
//   Wiener.forward      models/Wiener.py:10-20          -> RF_PSF_RAW, C_WIENER, RI_OUT1
//   Richard_Lucy.forward models/Richard_Lucy.py:10-24   -> RF_PSF_YP, C_OTF_CONV, RIF_RL_RATIO,
//                                                          C_CONVC, RIF_RL_UPDATE / RI_RL_FINAL, C_CONV
//
// ADMM state carried between iterations (all [N,1,L,L] fp32): u1, w = v - u2, zin (denoiser input)
// plus y and the half-spectrum OTF.  u2 and v are never stored: u2_{n+1} = Hx_{n+1} - w_n and
// v_{n+1} - u2_{n+1} is all the next X-update needs (algebraically identical to :207-213).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gdeconv.h"
#include "gd_fft.hpp"
#include "gd_subnet.hpp"

namespace gd {

// ---------------------------------------------------------------- per-galaxy scalar views
struct GalScalar {
    const float* p;
    long long stride;  // elements between galaxies; 0 = broadcast
    __device__ __forceinline__ float operator()(int g) const { return p[(long long)g * stride]; }
};

struct Args {
    int N;                 // galaxies in this launch
    float2* T;             // workspace spectra [N][2][K][L]
    float2* otf;           // half-spectrum OTF [N][K][L] (read or written depending on mode)
    const float* y;        // raw observation [N][L][L]
    const float* psf;      // [*, h, h]
    long long psf_gstride; // elements between galaxies' PSFs (0 = one shared PSF)
    int h;                 // PSF side (even, <= L)
    const float* a0;       // mode inputs
    const float* a1;
    const float* a2;
    float* o0;             // mode outputs
    float* o1;
    float* o2;
    GalScalar alpha, rho1, rho2, rho2n;
    int llh;               // GD_LLH_GAUSSIAN / GD_LLH_POISSON
    int last;              // final ADMM iteration: write x (times alpha for Poisson)
    int first;             // first ADMM iteration: spectral u1 is zero (not read)
    float2* s_yal;         // Gaussian spectral state [N][K][L]: F(max(y,0)/alpha)
    float2* s_u1;          //                                     F(u1)
    float2* s_w;           //                                     F(v - u2)
};

enum RowFwdMode { RF_ITER, RF_PSF_Y, RF_PSF_YP, RF_PSF_RAW, RF_PSF, RF_ONE, RF_TWO };
enum ColMode { C_ITER, C_OTF_INIT, C_OTF_CONV, C_WIENER, C_OTF, C_CONV, C_CONVC, C_CONV2, C_FWD, C_INV,
               C_G_OTF_INIT, C_G_INIT_W, C_G_ITER };
enum RowInvMode { RI_ITER, RI_INIT, RI_OUT1, RI_OUT2, RI_RL_FINAL };
enum RowInvFwdMode { RIF_CLAMP, RIF_RL_RATIO, RIF_RL_UPDATE };

constexpr int rows_per_block(int lpb, int L) {
    int rw = lpb < L ? lpb : L;
    while (L % rw || rw % 2) --rw;
    return rw;
}
constexpr int cmax(int x, int y) { return x > y ? x : y; }

template <int L>
struct Geo {
    static constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2;
    static constexpr int K = L / 2 + 1;
    static constexpr int LPB = 256 / F1;               // lines per 256-thread block
    static constexpr int RB = rows_per_block(LPB, L);  // rows per row-kernel block (even, divides L)
    static constexpr int RLD = L + 2;                  // row buffer leading dim (bank spread)
    static constexpr int XCH = xch_elems<L>();
    // row kernels (at most LPB lines): row buffer | exchange areas | staged / result images
    static constexpr int ROW_LDS = cmax(cmax(LPB * RLD, LPB * XCH), LPB * L);
    static constexpr int COL_LDS = LPB * XCH;
    static_assert(L % RB == 0 && RB % 2 == 0, "rows per block must be even and divide L");
};

__device__ __forceinline__ size_t tidx(int g, int img, int k, int row, int K, int L) {
    return ((size_t)(g * 2 + img) * K + k) * L + row;
}

__device__ __forceinline__ float shifted_psf(const Args& a, int g, int r, int c, int L) {
    const int c0 = a.h >> 1;
    int i = r + c0, jj = c + c0;
    if (i >= L) i -= L;
    if (jj >= L) jj -= L;
    if (i >= a.h || jj >= a.h) return 0.0f;
    return a.psf[(long long)g * a.psf_gstride + (long long)i * a.h + jj];
}

// V step (runtime classes, models/Unrolled_ADMM.py:326-328 and :335-336); yp = max(y, 0)
__device__ __forceinline__ float v_step(int llh, float vt, float yp, float rho2, float alpha) {
    if (llh == GD_LLH_POISSON) {
        const float t1 = rho2 * vt - alpha;
        return 0.5f * (1.0f / rho2) * (-t1 + sqrtf(t1 * t1 + 4.0f * yp * rho2));
    }
    return (rho2 * vt + yp / alpha) / (1.0f + rho2);
}

// ---------------------------------------------------------------- row-side building blocks
// Row kernels pack two ADJACENT ROWS OF THE SAME IMAGE into one complex line (row 2m -> real part,
// row 2m+1 -> imaginary part).  Packing two different images instead would extract the smaller
// one's spectrum from the rounding noise of the larger (a PSF of sum 1/16 next to an observation of
// ~1e2 ADU loses every digit), while rows of one image share its scale exactly as a 2D FFT does.
template <int L, int NI>
struct RowGeo {
    using G = Geo<L>;
    // rows per block, per image (even, divides L): up to LPB lines (256 threads) per block, so a
    // single-image kernel takes twice the rows of a two-image one
    static constexpr int RB = rows_per_block(2 * G::LPB / NI, L);
    static constexpr int PAIRS = RB / 2;    // lines per image
    static constexpr int LINES = NI * PAIRS;
    static constexpr int THREADS = LINES * G::F1;
    static_assert(RB % 2 == 0, "row pairs");
};

// Split line spectra C = FFT(row_even + i row_odd) (row buffer [line][k]) into the two rows'
// half spectra, stored transposed T[g][im][k][row0 + rr]; consecutive threads take consecutive rows.
template <int L, int NI>
__device__ __forceinline__ void split_store(const Args& a, const float2* rowbuf, int g, int row0, int tid) {
    using G = Geo<L>;
    using R = RowGeo<L, NI>;
    for (int idx = tid; idx < NI * G::K * R::RB; idx += R::THREADS) {
        const int rr = idx % R::RB, t = idx / R::RB;
        const int k = t % G::K, im = t / G::K;
        const int line = im * R::PAIRS + (rr >> 1);
        const float2 C = rowbuf[line * G::RLD + k];
        const float2 D = rowbuf[line * G::RLD + (k == 0 ? 0 : L - k)];
        const float2 o = (rr & 1) ? make_float2(0.5f * (C.y + D.y), 0.5f * (D.x - C.x))   // (C - conj D)/(2i)
                                  : make_float2(0.5f * (C.x + D.x), 0.5f * (C.y - D.y));  // (C + conj D)/2
        a.T[tidx(g, im, k, row0 + rr, G::K, L)] = o;
    }
}

// Gather the half spectra of rows 2m, 2m+1 of each image into the Hermitian-extended packed line
// spectrum D = R_even + i R_odd over kx in [0, L) (row buffer [line][k]).  One 16-byte load per
// (image, k, pair): the two rows are adjacent in the transposed layout.
template <int L, int NI>
__device__ __forceinline__ void gather_rows(const Args& a, float2* rowbuf, int g, int row0, int tid) {
    using G = Geo<L>;
    using R = RowGeo<L, NI>;
    for (int idx = tid; idx < NI * G::K * R::PAIRS; idx += R::THREADS) {
        const int m = idx % R::PAIRS, t = idx / R::PAIRS;
        const int k = t % G::K, im = t / G::K;
        const float4 q = *reinterpret_cast<const float4*>(a.T + tidx(g, im, k, row0 + 2 * m, G::K, L));
        float2 Re = make_float2(q.x, q.y), Ro = make_float2(q.z, q.w);
        const bool self = (k == 0) || (2 * k == L);  // self-conjugate bins: real parts only (irfft)
        if (self) {
            Re.y = 0.f;
            Ro.y = 0.f;
        }
        const int line = im * R::PAIRS + m;
        rowbuf[line * G::RLD + k] = make_float2(Re.x - Ro.y, Re.y + Ro.x);
        if (!self) rowbuf[line * G::RLD + (L - k)] = make_float2(Re.x + Ro.y, Ro.x - Re.y);
    }
}

// ---------------------------------------------------------------- RF: row forward
template <int MODE>
struct RfTraits {
    static constexpr int NI = (MODE == RF_PSF || MODE == RF_ONE) ? 1 : 2;
};

// Four consecutive pixels of image `im` starting at flat pixel index `pix` (row-major, 16-byte
// aligned) for the RF producers; (r, c) locate the first of them inside the galaxy.
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float f4(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
__device__ __forceinline__ void f4set(float4& v, int i, float x) {
    if (i == 0) v.x = x; else if (i == 1) v.y = x; else if (i == 2) v.z = x; else v.w = x;
}

template <int L, int MODE>
__device__ __forceinline__ float4 rf_source4(const Args& a, int g, int im, int r, int c, size_t pix) {
    if constexpr (MODE == RF_ITER) {
        if (im == 0) {                                                 // z - u1
            const float4 z = ld4(a.a0 + pix), u = ld4(a.a1 + pix);
            return make_float4(z.x - u.x, z.y - u.y, z.z - u.z, z.w - u.w);
        }
        return ld4(a.a2 + pix);                                        // w = v - u2
    } else if constexpr (MODE == RF_PSF || MODE == RF_PSF_Y || MODE == RF_PSF_YP || MODE == RF_PSF_RAW) {
        if (im == 0)
            return make_float4(shifted_psf(a, g, r, c, L), shifted_psf(a, g, r, c + 1, L),
                               shifted_psf(a, g, r, c + 2, L), shifted_psf(a, g, r, c + 3, L));
        const float4 y = ld4(a.y + pix);
        if constexpr (MODE == RF_PSF_RAW) return y;
        float4 yp = make_float4(fmaxf(y.x, 0.f), fmaxf(y.y, 0.f), fmaxf(y.z, 0.f), fmaxf(y.w, 0.f));
        if constexpr (MODE == RF_PSF_YP) {
            st4(a.o0 + pix, yp);                                       // Richardson-Lucy x0 = max(y, 0)
            return yp;
        } else {
            const float al = a.alpha(g);                               // max(y,0) / alpha
            return make_float4(yp.x / al, yp.y / al, yp.z / al, yp.w / al);
        }
    } else if constexpr (MODE == RF_ONE) {
        return ld4(a.a0 + pix);
    } else {
        return ld4((im == 0 ? a.a0 : a.a1) + pix);
    }
}

template <int L, int MODE>
__global__ __launch_bounds__((RowGeo<L, RfTraits<MODE>::NI>::THREADS)) void k_row_fwd(Args a) {
    constexpr int NI = RfTraits<MODE>::NI;
    using G = Geo<L>;
    using R = RowGeo<L, NI>;
    constexpr int F1 = G::F1, F2 = G::F2;
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 lds[G::ROW_LDS];
    const int tid = threadIdx.x;
    const int blocks_per_g = L / R::RB;
    const int g = blockIdx.x / blocks_per_g;
    const int row0 = (blockIdx.x - g * blocks_per_g) * R::RB;
    const int line = tid / F1, j = tid - line * F1;
    const int im = line / R::PAIRS, m = line - im * R::PAIRS;
    fill_twiddles<L>(tw, tid, R::THREADS);
    // stage the block's RB rows of each image through LDS with 16-byte coalesced loads
    float* stage = reinterpret_cast<float*>(lds);  // [im][rr][c]
    for (int q = tid * 4; q < NI * R::RB * L; q += R::THREADS * 4) {
        const int imq = q / (R::RB * L), rem = q - imq * (R::RB * L);
        const int rr = rem / L, c = rem - rr * L;
        const size_t pix = ((size_t)g * L + row0 + rr) * L + c;
        st4(stage + q, rf_source4<L, MODE>(a, g, imq, row0 + rr, c, pix));
    }
    __syncthreads();
    float2 v[F2];
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        const int c = j + F1 * s;
        v[s] = make_float2(stage[(im * R::RB + 2 * m) * L + c], stage[(im * R::RB + 2 * m + 1) * L + c]);
    }
    __syncthreads();  // staging -> exchange areas
    line_fft<L, false>(v, j, lds + line * G::XCH, tw);
    __syncthreads();  // exchange areas -> row buffer
#pragma unroll
    for (int s = 0; s < F2; ++s) lds[line * G::RLD + j + F1 * s] = v[s];
    __syncthreads();
    split_store<L, NI>(a, lds, g, row0, tid);
}

// ---------------------------------------------------------------- C: column pass
template <int MODE>
struct ColTraits {
    static constexpr bool IN2 = (MODE == C_ITER || MODE == C_OTF_INIT || MODE == C_OTF_CONV ||
                                 MODE == C_WIENER || MODE == C_CONV2 || MODE == C_G_OTF_INIT);
    static constexpr bool OUT2 = (MODE == C_ITER || MODE == C_CONV2);
    static constexpr bool HAS_OUT = (MODE != C_OTF && MODE != C_FWD && MODE != C_G_INIT_W);
    static constexpr bool STORE_OTF = (MODE == C_OTF_INIT || MODE == C_OTF_CONV || MODE == C_OTF ||
                                       MODE == C_G_OTF_INIT);
    static constexpr bool LOAD_OTF = (MODE == C_ITER || MODE == C_CONV || MODE == C_CONVC || MODE == C_CONV2 ||
                                      MODE == C_G_INIT_W || MODE == C_G_ITER);
    static constexpr bool FWD = (MODE != C_INV);
};

// VAR: experiment switch for tools/kbench.hip (0 = production; 1 = no FFTs, memory only;
// 2 = G_ITER operands H and W loaded before the forward FFT)
template <int L, int MODE, int VAR = 0>
__global__ __launch_bounds__(256) void k_col(Args a) {
    using G = Geo<L>;
    using TR = ColTraits<MODE>;
    constexpr int F1 = G::F1, F2 = G::F2, K = G::K;
    __shared__ float2 tw[L];
    __shared__ float2 xch[G::COL_LDS];
    const int tid = threadIdx.x;
    const int line = tid / F1, j = tid - line * F1;
    const int f = blockIdx.x * G::LPB + line;
    const bool valid = f < a.N * K;
    const int fc = valid ? f : 0;
    const int g = fc / K, kx = fc - g * K;
    fill_twiddles<L>(tw, tid, 256);
    float2* my = xch + line * G::XCH;

    float2 P[F2], Q[F2];
    const size_t c0 = tidx(g, 0, kx, 0, K, L), c1 = tidx(g, 1, kx, 0, K, L);
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        P[s] = a.T[c0 + j + F1 * s];
        if constexpr (TR::IN2) Q[s] = a.T[c1 + j + F1 * s];
    }
    float2 Hpre[VAR == 2 ? F2 : 1], Wpre[VAR == 2 ? F2 : 1];
    if constexpr (VAR == 2 && MODE == C_G_ITER) {
        const size_t ob0 = ((size_t)g * K + kx) * L;
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            Hpre[s] = a.otf[ob0 + j + F1 * s];
            Wpre[s] = a.s_w[ob0 + j + F1 * s];
        }
    }
    __syncthreads();  // twiddles
    if constexpr (TR::FWD && VAR != 1) {
        line_fft<L, false>(P, j, my, tw);
        if constexpr (TR::IN2) line_fft<L, false>(Q, j, my, tw);
    }
    constexpr float inv_n = float(1.0 / double(L * L));  // exact for L = 2^k
    const size_t ob = ((size_t)g * K + kx) * L;
    const float al = (MODE == C_OTF_INIT || MODE == C_WIENER || MODE == C_G_OTF_INIT) ? a.alpha(g) : 1.f;
    const float r1 = (MODE == C_ITER || MODE == C_G_ITER) ? a.rho1(g) : 0.f;
    const float r2 = (MODE == C_ITER || MODE == C_G_ITER) ? a.rho2(g) : 0.f;
    const bool glast = (MODE == C_G_ITER) && a.last;
    const float r2n = (MODE == C_G_INIT_W || (MODE == C_G_ITER && !glast)) ? a.rho2n(g) : 0.f;
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        const int ky = j + F1 * s;
        float2 Hk = make_float2(0.f, 0.f);
        if constexpr (VAR == 2 && MODE == C_G_ITER) Hk = Hpre[s];
        else if constexpr (TR::LOAD_OTF) Hk = a.otf[ob + ky];
        if constexpr (TR::STORE_OTF || MODE == C_WIENER) Hk = P[s];
        if constexpr (TR::STORE_OTF) {
            if (valid) a.otf[ob + ky] = Hk;
        }
        if constexpr (MODE == C_ITER) {
            // runtime X_Update (models/Unrolled_ADMM.py:315-319):
            //   X = (rho1 F(z-u1) + rho2 conj(H) F(v-u2)) / (rho1 |H|^2 + rho2);  HX = H X
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float lhs = r1 * HtH + r2;
            const float2 HtW = cmulc(Q[s], Hk);
            const float2 rhs = make_float2(r1 * P[s].x + r2 * HtW.x, r1 * P[s].y + r2 * HtW.y);
            const float2 X = make_float2(rhs.x / lhs, rhs.y / lhs);
            P[s] = cscale(X, inv_n);
            Q[s] = cscale(cmul(Hk, X), inv_n);
        } else if constexpr (MODE == C_OTF_INIT) {
            // init_l2 (models/Unrolled_ADMM.py:170-175): conj(H) F(y/alpha) / (|H|^2 + 1/alpha)
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float lhs = HtH + 1.0f / al;
            const float2 rhs = cmulc(Q[s], Hk);
            P[s] = cscale(make_float2(rhs.x / lhs, rhs.y / lhs), inv_n);
        } else if constexpr (MODE == C_G_OTF_INIT) {
            // as C_OTF_INIT, and keep F(y/alpha) as Gaussian spectral state
            if (valid) a.s_yal[ob + ky] = Q[s];
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float lhs = HtH + 1.0f / al;
            const float2 rhs = cmulc(Q[s], Hk);
            P[s] = cscale(make_float2(rhs.x / lhs, rhs.y / lhs), inv_n);
        } else if constexpr (MODE == C_G_INIT_W) {
            // first V step in the spectral domain (u1 = u2 = 0): W1 = V1 = (rho2 (H X0 + 0) + F(y/alpha)) / (1 + rho2)
            const float2 HX = cmul(Hk, P[s]);
            const float2 Ya = a.s_yal[ob + ky];
            const float d = 1.0f + r2n;
            if (valid) a.s_w[ob + ky] = make_float2((r2n * HX.x + Ya.x) / d, (r2n * HX.y + Ya.y) / d);
        } else if constexpr (MODE == C_G_ITER) {
            // Gaussian ADMM iteration entirely in the spectral domain (all steps of
            // models/Unrolled_ADMM.py:207-213 are linear for llh='Gaussian'):
            //   X   = (rho1 (Z - U1) + rho2 conj(H) W) / (rho1 |H|^2 + rho2)      runtime X_Update :315-319
            //   U1' = (U1 + X) - Z ;  U2' = H X - W                               :212-213 (W = V - U2)
            //   V'  = (rho2' (H X + U2') + F(y/alpha)) / (1 + rho2') ;  W' = V' - U2'   V step :335-336
            //   out = X + U1' (next denoiser input)  |  X (last iteration)
            const float2 Zk = P[s];
            const float2 U1 = a.first ? make_float2(0.f, 0.f) : a.s_u1[ob + ky];
            float2 Wk;
            if constexpr (VAR == 2) Wk = Wpre[s];
            else Wk = a.s_w[ob + ky];
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float lhs = r1 * HtH + r2;
            const float2 A = csub(Zk, U1);
            const float2 HtW = cmulc(Wk, Hk);
            const float2 rhs = make_float2(r1 * A.x + r2 * HtW.x, r1 * A.y + r2 * HtW.y);
            const float2 X = make_float2(rhs.x / lhs, rhs.y / lhs);
            if (glast) {
                P[s] = cscale(X, inv_n);
            } else {
                const float2 U1n = csub(cadd(U1, X), Zk);
                const float2 HX = cmul(Hk, X);
                const float2 U2n = csub(HX, Wk);
                const float2 Ya = a.s_yal[ob + ky];
                const float d = 1.0f + r2n;
                const float2 Vn = make_float2((r2n * (HX.x + U2n.x) + Ya.x) / d, (r2n * (HX.y + U2n.y) + Ya.y) / d);
                if (valid) {
                    a.s_u1[ob + ky] = U1n;
                    a.s_w[ob + ky] = csub(Vn, U2n);
                }
                P[s] = cscale(cadd(X, U1n), inv_n);
            }
        } else if constexpr (MODE == C_WIENER) {
            // models/Wiener.py:16-18: conj(H) F(y) / (|H|^2 + 350/alpha)
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float div = HtH + 350.0f / al;
            const float2 num = cmulc(Q[s], Hk);
            P[s] = cscale(make_float2(num.x / div, num.y / div), inv_n);
        } else if constexpr (MODE == C_OTF_CONV) {
            P[s] = cscale(cmul(Q[s], Hk), inv_n);
        } else if constexpr (MODE == C_CONV) {
            P[s] = cscale(cmul(P[s], Hk), inv_n);
        } else if constexpr (MODE == C_CONVC) {
            P[s] = cscale(cmulc(P[s], Hk), inv_n);
        } else if constexpr (MODE == C_CONV2) {
            P[s] = cscale(cmul(P[s], Hk), inv_n);
            Q[s] = cscale(cmul(Q[s], Hk), inv_n);
        } else if constexpr (MODE == C_INV) {
            P[s] = cscale(P[s], inv_n);
        }
    }
    if constexpr (TR::HAS_OUT && MODE != C_FWD && VAR != 1) {
        line_fft<L, true>(P, j, my, tw);
        if constexpr (TR::OUT2) line_fft<L, true>(Q, j, my, tw);
    }
    if (valid) {
        if constexpr (MODE == C_FWD) {
#pragma unroll
            for (int s = 0; s < F2; ++s) a.T[c0 + j + F1 * s] = P[s];
        } else if constexpr (TR::HAS_OUT) {
#pragma unroll
            for (int s = 0; s < F2; ++s) {
                a.T[c0 + j + F1 * s] = P[s];
                if constexpr (TR::OUT2) a.T[c1 + j + F1 * s] = Q[s];
            }
        }
    }
}

// ---------------------------------------------------------------- RI: row inverse + sink
template <int MODE>
struct RiTraits {
    static constexpr int NI = (MODE == RI_ITER || MODE == RI_OUT2) ? 2 : 1;
};

template <int L, int MODE>
__global__ __launch_bounds__((RowGeo<L, RiTraits<MODE>::NI>::THREADS)) void k_row_inv(Args a) {
    constexpr int NI = RiTraits<MODE>::NI;
    using G = Geo<L>;
    using R = RowGeo<L, NI>;
    constexpr int F1 = G::F1, F2 = G::F2;
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 lds[G::ROW_LDS];
    const int tid = threadIdx.x;
    const int blocks_per_g = L / R::RB;
    const int g = blockIdx.x / blocks_per_g;
    const int row0 = (blockIdx.x - g * blocks_per_g) * R::RB;
    const int line = tid / F1, j = tid - line * F1;
    const int im = line / R::PAIRS, m = line - im * R::PAIRS;
    fill_twiddles<L>(tw, tid, R::THREADS);
    gather_rows<L, NI>(a, lds, g, row0, tid);
    __syncthreads();
    float2 v[F2];
#pragma unroll
    for (int s = 0; s < F2; ++s) v[s] = lds[line * G::RLD + j + F1 * s];
    __syncthreads();  // row buffer -> exchange area
    line_fft<L, true>(v, j, lds + line * G::XCH, tw);
    __syncthreads();  // every line done with its exchange area -> result image
    float* res = reinterpret_cast<float*>(lds);  // [im][rr][c], RB x L per image
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        const int c = j + F1 * s;
        res[(im * R::RB + 2 * m) * L + c] = v[s].x;
        res[(im * R::RB + 2 * m + 1) * L + c] = v[s].y;
    }
    __syncthreads();

    float al = 1.f, r2n = 1.f, div = 1.f;
    if constexpr (MODE == RI_ITER || MODE == RI_INIT) {
        al = a.alpha(g);
        if (!(MODE == RI_ITER && a.last)) r2n = a.rho2n(g);
    }
    if constexpr (MODE == RI_RL_FINAL) div = a.otf[(size_t)g * G::K * L].x;  // conv(Ht, ones) = H(0,0)
    const bool poisson = a.llh == GD_LLH_POISSON;
    // elementwise sink over this block's RB x L pixels, 4 consecutive pixels per thread step
    for (int q = tid * 4; q < R::RB * L; q += R::THREADS * 4) {
        const int rr = q / L, c = q - rr * L;
        const size_t pix = ((size_t)g * L + row0 + rr) * L + c;
        const float4 X = ld4(res + rr * L + c);
        if constexpr (MODE == RI_ITER) {
            // models/Unrolled_ADMM.py:207-215 (x = image 0, conv(H, x) = image 1)
            const float4 HX = ld4(res + (R::RB + rr) * L + c);
            if (a.last) {
                float4 o = X;
                if (poisson) o = make_float4(X.x * al, X.y * al, X.z * al, X.w * al);
                st4(a.o2 + pix, o);
            } else {
                const float4 Z = ld4(a.a0 + pix), U1 = ld4(a.o0 + pix), Wv = ld4(a.o1 + pix), Y = ld4(a.y + pix);
                float4 u1o, wo, zo;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = f4(X, e), hx = f4(HX, e);
                    const float u1 = (f4(U1, e) + x) - f4(Z, e);      // u1 + x - z
                    const float u2 = hx - f4(Wv, e);                  // u2 + conv(H,x) - v  (w = v - u2)
                    const float vn = v_step(a.llh, hx + u2, fmaxf(f4(Y, e), 0.f), r2n, al);
                    f4set(u1o, e, u1);
                    f4set(wo, e, vn - u2);
                    f4set(zo, e, x + u1);                             // next denoiser input
                }
                st4(a.o0 + pix, u1o);
                st4(a.o1 + pix, wo);
                st4(a.o2 + pix, zo);
            }
        } else if constexpr (MODE == RI_INIT) {
            // first V step with x = x0, u1 = u2 = 0: v = V(conv(H, x0) + 0, ...)
            const float4 Y = ld4(a.y + pix);
            float4 wo;
#pragma unroll
            for (int e = 0; e < 4; ++e) f4set(wo, e, v_step(a.llh, f4(X, e) + 0.0f, fmaxf(f4(Y, e), 0.f), r2n, al));
            st4(a.o1 + pix, wo);
            st4(a.o0 + pix, make_float4(0.f, 0.f, 0.f, 0.f));
        } else if constexpr (MODE == RI_OUT1) {
            st4(a.o0 + pix, X);
        } else if constexpr (MODE == RI_OUT2) {
            st4(a.o0 + pix, X);
            st4(a.o1 + pix, ld4(res + (R::RB + rr) * L + c));
        } else if constexpr (MODE == RI_RL_FINAL) {
            const float4 X0 = ld4(a.o0 + pix);
            float4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) f4set(o, e, f4(X0, e) * f4(X, e) / div);   // x * numerator / divisor
            st4(a.o0 + pix, o);
        }
    }
}

// ---------------------------------------------------------------- RIF: row inverse -> pointwise -> row forward
template <int L, int MODE>
__device__ __forceinline__ float rif_point(const Args& a, int g, int r, int c, float re, float div) {
    const size_t pix = ((size_t)g * L + r) * L + c;
    if constexpr (MODE == RIF_CLAMP) {
        const float p = fminf(fmaxf(re, 0.f), 1.f);   // torch.clamp(x0, 0, 1)
        a.o0[pix] = p;
        return p;
    } else if constexpr (MODE == RIF_RL_RATIO) {
        return fmaxf(a.y[pix], 0.f) / re;             // y / Hx
    } else {
        const float p = a.o0[pix] * re / div;         // x * numerator / divisor
        a.o0[pix] = p;
        return p;
    }
}

template <int L, int MODE>
__global__ __launch_bounds__((RowGeo<L, 1>::THREADS)) void k_row_invfwd(Args a) {
    using G = Geo<L>;
    using R = RowGeo<L, 1>;
    constexpr int F1 = G::F1, F2 = G::F2;
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 lds[G::ROW_LDS];
    const int tid = threadIdx.x;
    const int blocks_per_g = L / R::RB;
    const int g = blockIdx.x / blocks_per_g;
    const int row0 = (blockIdx.x - g * blocks_per_g) * R::RB;
    const int line = tid / F1, j = tid - line * F1;
    const int rA = row0 + 2 * line;
    fill_twiddles<L>(tw, tid, R::THREADS);
    gather_rows<L, 1>(a, lds, g, row0, tid);
    __syncthreads();
    float2 v[F2];
#pragma unroll
    for (int s = 0; s < F2; ++s) v[s] = lds[line * G::RLD + j + F1 * s];
    __syncthreads();
    line_fft<L, true>(v, j, lds + line * G::XCH, tw);
    float div = 1.f;
    if constexpr (MODE == RIF_RL_UPDATE) div = a.otf[(size_t)g * G::K * L].x;
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        const int c = j + F1 * s;
        v[s] = make_float2(rif_point<L, MODE>(a, g, rA, c, v[s].x, div),
                           rif_point<L, MODE>(a, g, rA + 1, c, v[s].y, div));
    }
    line_fft<L, false>(v, j, lds + line * G::XCH, tw);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < F2; ++s) lds[line * G::RLD + j + F1 * s] = v[s];
    __syncthreads();
    split_store<L, 1>(a, lds, g, row0, tid);
}

// ---------------------------------------------------------------- host-side launch helpers
thread_local std::string g_last_error;

constexpr const char* kRowFwdName = "k_row_fwd";
constexpr const char* kColName = "k_col";
constexpr const char* kRowInvName = "k_row_inv";
constexpr const char* kRowInvFwdName = "k_row_invfwd";

inline int fail(int code, const char* msg) {
    g_last_error = msg;
    return code;
}

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_error = std::string(what) + ": " + hipGetErrorString(e);
        return GD_ERR_HIP;
    }
    return GD_OK;
}

// Opt-in per-kernel timing (gd_profile_*): every launch is bracketed by two hipEvents recorded on
// the launch stream; durations are harvested by gd_profile_collect().  Off by default (no events,
// graph-capturable).
struct ProfEntry {
    std::string name;
    hipEvent_t start, stop;
};
struct ProfStat {
    double ms = 0.0;
    long long launches = 0;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfEntry> g_prof_pending;
std::vector<hipEvent_t> g_prof_pool;
std::map<std::string, ProfStat> g_prof_stats;

inline hipEvent_t prof_event() {
    if (!g_prof_pool.empty()) {
        hipEvent_t e = g_prof_pool.back();
        g_prof_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
}

struct ProfScope {
    bool on;
    ProfEntry ent;
    hipStream_t st;
    ProfScope(const std::string& name, hipStream_t s) : on(false), st(s) {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        if (!g_prof_on) return;
        on = true;
        ent.name = name;
        ent.start = prof_event();
        ent.stop = prof_event();
        (void)hipEventRecord(ent.start, st);
    }
    ~ProfScope() {
        if (!on) return;
        (void)hipEventRecord(ent.stop, st);
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof_pending.push_back(ent);
    }
};

template <int L>
struct Launcher {
    using G = Geo<L>;
    template <int NI>
    static int row_grid(int N) { return N * (L / RowGeo<L, NI>::RB); }
    static int col_grid(int N) { return (N * G::K + G::LPB - 1) / G::LPB; }
    static std::string nm(const char* k, int mode) {
        return std::string(k) + "<" + std::to_string(L) + "," + std::to_string(mode) + ">";
    }

    template <int MODE>
    static int rf(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kRowFwdName, MODE), st);
        hipLaunchKernelGGL((k_row_fwd<L, MODE>), dim3(row_grid<RfTraits<MODE>::NI>(a.N)), dim3(RowGeo<L, RfTraits<MODE>::NI>::THREADS), 0, st, a);
        return check_launch("k_row_fwd");
    }
    template <int MODE>
    static int col(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kColName, MODE), st);
        hipLaunchKernelGGL((k_col<L, MODE>), dim3(col_grid(a.N)), dim3(256), 0, st, a);
        return check_launch("k_col");
    }
    template <int MODE>
    static int ri(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kRowInvName, MODE), st);
        hipLaunchKernelGGL((k_row_inv<L, MODE>), dim3(row_grid<RiTraits<MODE>::NI>(a.N)), dim3(RowGeo<L, RiTraits<MODE>::NI>::THREADS), 0, st, a);
        return check_launch("k_row_inv");
    }
    template <int MODE>
    static int rif(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kRowInvFwdName, MODE), st);
        hipLaunchKernelGGL((k_row_invfwd<L, MODE>), dim3(row_grid<1>(a.N)), dim3(RowGeo<L, 1>::THREADS), 0, st, a);
        return check_launch("k_row_invfwd");
    }
};

#define GD_TRY(x)                    \
    do {                             \
        int _rc = (x);               \
        if (_rc != GD_OK) return _rc; \
    } while (0)

// ---------------------------------------------------------------- Infinity-Cache chunking
// A multi-kernel operation runs chunk by chunk over the batch: each chunk's spectral workspace
// (and the images the row passes read twice) stays resident in the 256 MiB Infinity Cache between
// its kernels instead of round-tripping through HBM.  g_chunk_bytes is the target resident working
// set per chunk (0 = whole batch in one pass).
size_t g_chunk_bytes = 0;  // measured: chunking slower at 256^2 (small-grid fill/drain > MALL gain)

inline Args offset_args(const Args& a, int g0, int n, int L) {
    Args b = a;
    b.N = n;
    const size_t img = (size_t)g0 * L * L;
    const size_t spec = (size_t)g0 * (L / 2 + 1) * L;
    if (b.otf) b.otf += spec;
    if (b.s_yal) b.s_yal += spec;
    if (b.s_u1) b.s_u1 += spec;
    if (b.s_w) b.s_w += spec;
    if (b.y) b.y += img;
    if (b.a0) b.a0 += img;
    if (b.a1) b.a1 += img;
    if (b.a2) b.a2 += img;
    if (b.o0) b.o0 += img;
    if (b.o1) b.o1 += img;
    if (b.o2) b.o2 += img;
    if (b.psf) b.psf += (long long)g0 * a.psf_gstride;
    GalScalar* gs[] = {&b.alpha, &b.rho1, &b.rho2, &b.rho2n};
    for (GalScalar* x : gs)
        if (x->p) x->p += (long long)g0 * x->stride;
    return b;  // T (workspace) is not offset: every chunk reuses its head
}

template <typename F>
int for_chunks(const Args& a, int L, size_t per_galaxy_bytes, F&& f) {
    int G = a.N;
    if (g_chunk_bytes && per_galaxy_bytes) {
        const size_t g = g_chunk_bytes / per_galaxy_bytes;
        G = (int)(g < 1 ? 1 : (g > (size_t)a.N ? (size_t)a.N : g));
    }
    for (int g0 = 0; g0 < a.N; g0 += G) {
        const int n = (a.N - g0 < G) ? a.N - g0 : G;
        GD_TRY(f(offset_args(a, g0, n, L)));
    }
    return GD_OK;
}

// Operation bodies, templated on L.
template <int L>
struct Ops {
    static constexpr size_t IMG = (size_t)L * L * 4, HALF = (size_t)(L / 2 + 1) * L * 8;
    using Lc = Launcher<L>;
    static int psf_to_otf(Args a, hipStream_t st) {
        GD_TRY(Lc::template rf<RF_PSF>(a, st));
        return Lc::template col<C_OTF>(a, st);
    }
    static int conv(Args a, int conj, hipStream_t st) {
        GD_TRY(Lc::template rf<RF_ONE>(a, st));
        GD_TRY(conj ? Lc::template col<C_CONVC>(a, st) : Lc::template col<C_CONV>(a, st));
        return Lc::template ri<RI_OUT1>(a, st);
    }
    static int rfft2(Args a, hipStream_t st) {
        GD_TRY(Lc::template rf<RF_ONE>(a, st));
        return Lc::template col<C_FWD>(a, st);
    }
    static int irfft2(Args a, hipStream_t st) {
        GD_TRY(Lc::template col<C_INV>(a, st));
        return Lc::template ri<RI_OUT1>(a, st);
    }
    static int admm_init(Args a0, hipStream_t st) {
        // a.o0 = u1, a.o1 = w, a.o2 = zin (x0)
        return for_chunks(a0, L, 2 * HALF + 4 * IMG, [&](const Args& a) {
            Args b = a;
            GD_TRY(Lc::template rf<RF_PSF_Y>(b, st));
            GD_TRY(Lc::template col<C_OTF_INIT>(b, st));
            b.o0 = a.o2;  // RIF_CLAMP writes x0 -> zin
            GD_TRY(Lc::template rif<RIF_CLAMP>(b, st));
            GD_TRY(Lc::template col<C_CONV>(b, st));
            return Lc::template ri<RI_INIT>(a, st);
        });
    }
    static int admm_init_gauss(Args a0, hipStream_t st) {
        // spectral state: otf, s_yal, s_w (s_u1 implicitly 0); a.o2 = zin (x0)
        return for_chunks(a0, L, 2 * HALF + 4 * IMG, [&](const Args& a) {
            Args b = a;
            GD_TRY(Lc::template rf<RF_PSF_Y>(b, st));
            GD_TRY(Lc::template col<C_G_OTF_INIT>(b, st));
            b.o0 = a.o2;  // RIF_CLAMP writes x0 -> zin
            GD_TRY(Lc::template rif<RIF_CLAMP>(b, st));
            return Lc::template col<C_G_INIT_W>(b, st);
        });
    }
    static int admm_iter_gauss(Args a0, hipStream_t st) {
        // a.a0 = z; spectral state updated in place; a.o0 = zin (or the output on the last iteration)
        return for_chunks(a0, L, HALF + 2 * IMG, [&](const Args& a) {
            GD_TRY(Lc::template rf<RF_ONE>(a, st));
            GD_TRY(Lc::template col<C_G_ITER>(a, st));
            return Lc::template ri<RI_OUT1>(a, st);
        });
    }
    static int admm_iter(Args a0, hipStream_t st) {
        // a.a0 = z, a.a1 = u1 (RF reads), a.a2 = w; RI: a.o0 = u1, a.o1 = w, a.o2 = zin / out
        return for_chunks(a0, L, 2 * HALF + 3 * IMG, [&](const Args& a) {
            GD_TRY(Lc::template rf<RF_ITER>(a, st));
            GD_TRY(Lc::template col<C_ITER>(a, st));
            return Lc::template ri<RI_ITER>(a, st);
        });
    }
    static int wiener(Args a0, hipStream_t st) {
        return for_chunks(a0, L, 2 * HALF + IMG, [&](const Args& a) {
            GD_TRY(Lc::template rf<RF_PSF_RAW>(a, st));
            GD_TRY(Lc::template col<C_WIENER>(a, st));
            return Lc::template ri<RI_OUT1>(a, st);
        });
    }
    static int richardson_lucy(Args a0, int n_iters, hipStream_t st) {
        // a.o0 = x (output, also the iterate); otf kept in a.otf.  The whole iteration loop runs per
        // chunk, so x, y, the OTF and the workspace stay cache-resident across all n_iters.
        return for_chunks(a0, L, 2 * HALF + 2 * IMG, [&](const Args& a) {
            GD_TRY(Lc::template rf<RF_PSF_YP>(a, st));
            if (n_iters <= 0) return GD_OK;
            GD_TRY(Lc::template col<C_OTF_CONV>(a, st));
            for (int it = 0; it < n_iters; ++it) {
                if (it > 0) GD_TRY(Lc::template col<C_CONV>(a, st));
                GD_TRY(Lc::template rif<RIF_RL_RATIO>(a, st));
                GD_TRY(Lc::template col<C_CONVC>(a, st));
                if (it + 1 < n_iters)
                    GD_TRY(Lc::template rif<RIF_RL_UPDATE>(a, st));
                else
                    GD_TRY(Lc::template ri<RI_RL_FINAL>(a, st));
            }
            return GD_OK;
        });
    }
};

template <template <int> class OP, typename F>
int dispatch(int L, F&& f) {
    switch (L) {
        case 32: return f(OP<32>{});
        case 48: return f(OP<48>{});
        case 64: return f(OP<64>{});
        case 96: return f(OP<96>{});
        case 128: return f(OP<128>{});
        case 256: return f(OP<256>{});
        default: return fail(GD_ERR_UNSUPPORTED, "unsupported image size (supported: 32, 48, 64, 96, 128, 256, square)");
    }
}

inline int check_shape(int N, int H, int W) {
    if (N < 0) return fail(GD_ERR_ARG, "negative batch");
    if (H != W) return fail(GD_ERR_UNSUPPORTED, "only square images are supported");
    if (!gd_supported_size(H, W)) return fail(GD_ERR_UNSUPPORTED, "unsupported image size");
    return GD_OK;
}

inline int check_psf(int h, int w, int H) {
    if (h != w) return fail(GD_ERR_ARG, "psf must be square (psf_to_otf uses ker.shape[2] for both axes)");
    if (h <= 0 || (h & 1)) return fail(GD_ERR_ARG, "psf side must be even (odd sizes fail in the reference's quadrant copy)");
    if (h > H) return fail(GD_ERR_ARG, "psf larger than the image");
    return GD_OK;
}

inline Args base_args(int N, void* ws, int L) {
    Args a;
    std::memset(&a, 0, sizeof(a));
    a.N = N;
    a.T = reinterpret_cast<float2*>(ws);
    (void)L;
    a.alpha = GalScalar{nullptr, 0};
    a.rho1 = a.rho2 = a.rho2n = a.alpha;
    return a;
}

}  // namespace gd

using namespace gd;

// ====================================================================== C ABI
extern "C" {

int gd_abi_version(void) { return GD_ABI_VERSION; }

const char* gd_last_error(void) { return g_last_error.c_str(); }

int gd_supported_size(int H, int W) {
    if (H != W) return 0;
    switch (H) {
        case 32: case 48: case 64: case 96: case 128: case 256: return 1;
        default: return 0;
    }
}

size_t gd_workspace_bytes(int N, int H, int W) {
    if (!gd_supported_size(H, W) || N <= 0) return 0;
    const size_t K = (size_t)W / 2 + 1;
    return (size_t)N * 2 * K * H * sizeof(float2);
}

size_t gd_otf_bytes(int N, int H, int W) {
    if (!gd_supported_size(H, W) || N <= 0) return 0;
    return (size_t)N * (W / 2 + 1) * H * sizeof(float2);
}

int gd_psf_to_otf(const float* psf, long long psf_gstride, int h, int w, int N, int H, int W,
                  void* otf_half, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H));
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H);
    a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.otf = reinterpret_cast<float2*>(otf_half);
    return dispatch<Ops>(H, [&](auto op) { return decltype(op)::psf_to_otf(a, (hipStream_t)stream); });
}

int gd_conv_fft_batch(const void* otf_half, int conj, const float* x, float* out, int N, int H, int W,
                      void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H);
    a.otf = reinterpret_cast<float2*>(const_cast<void*>(otf_half));
    a.a0 = x; a.o0 = out;
    return dispatch<Ops>(H, [&](auto op) { return decltype(op)::conv(a, conj, (hipStream_t)stream); });
}

int gd_rfft2(const float* x, void* spec, int N, int H, int W, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (N == 0) return GD_OK;
    Args a = base_args(N, spec, H);  // spectrum lives in image slot 0 of a T-shaped buffer
    a.a0 = x;
    return dispatch<Ops>(H, [&](auto op) { return decltype(op)::rfft2(a, (hipStream_t)stream); });
}

int gd_irfft2(void* spec, float* x, int N, int H, int W, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (N == 0) return GD_OK;
    Args a = base_args(N, spec, H);
    a.o0 = x;
    return dispatch<Ops>(H, [&](auto op) { return decltype(op)::irfft2(a, (hipStream_t)stream); });
}

size_t gd_admm_state_bytes(int N, int H, int W, int llh) {
    if (!gd_supported_size(H, W) || N <= 0) return 0;
    const size_t spec = (size_t)N * (W / 2 + 1) * H * sizeof(float2), img = (size_t)N * H * W * sizeof(float);
    return llh == GD_LLH_GAUSSIAN ? 4 * spec : spec + 2 * img;
}

namespace {
// state layout - Gaussian: [otf | F(y/alpha) | F(u1) | F(v-u2)] (spectral); Poisson: [otf | u1 | w]
void bind_state(Args& a, void* state, int N, int H, int W, int llh) {
    const size_t spec = (size_t)N * (W / 2 + 1) * H;
    float2* base = reinterpret_cast<float2*>(state);
    a.otf = base;
    if (llh == GD_LLH_GAUSSIAN) {
        a.s_yal = base + spec;
        a.s_u1 = base + 2 * spec;
        a.s_w = base + 3 * spec;
    } else {
        float* u1 = reinterpret_cast<float*>(base + spec);
        a.o0 = u1;                       // u1 (spatial)
        a.o1 = u1 + (size_t)N * H * W;   // w = v - u2 (spatial)
    }
}
}  // namespace

int gd_admm_init(const float* y, const float* psf, long long psf_gstride, int h, int w,
                 const float* alpha, long long alpha_stride, const float* rho2, long long rho2_stride,
                 int llh, int N, int H, int W, void* state, float* zin, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H));
    if (llh != GD_LLH_GAUSSIAN && llh != GD_LLH_POISSON) return fail(GD_ERR_ARG, "llh must be Gaussian or Poisson");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.alpha = GalScalar{alpha, alpha_stride};
    a.rho2n = GalScalar{rho2, rho2_stride};
    a.llh = llh;
    bind_state(a, state, N, H, W, llh);
    a.o2 = zin;
    if (llh == GD_LLH_GAUSSIAN)
        return dispatch<Ops>(H, [&](auto op) { return decltype(op)::admm_init_gauss(a, (hipStream_t)stream); });
    return dispatch<Ops>(H, [&](auto op) { return decltype(op)::admm_init(a, (hipStream_t)stream); });
}

int gd_admm_iter(const float* y, const float* z, float* zin_or_out, const float* alpha, long long alpha_stride,
                 const float* rho1, long long rho1_stride, const float* rho2, long long rho2_stride,
                 const float* rho2_next, long long rho2_next_stride, int llh, int iter, int last, int N, int H,
                 int W, void* state, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (llh != GD_LLH_GAUSSIAN && llh != GD_LLH_POISSON) return fail(GD_ERR_ARG, "llh must be Gaussian or Poisson");
    if (N == 0) return GD_OK;
    if (!last && rho2_next == nullptr) return fail(GD_ERR_ARG, "rho2_next required unless last");
    Args a = base_args(N, ws, H);
    a.y = y;
    bind_state(a, state, N, H, W, llh);
    a.alpha = GalScalar{alpha, alpha_stride};
    a.rho1 = GalScalar{rho1, rho1_stride};
    a.rho2 = GalScalar{rho2, rho2_stride};
    a.rho2n = GalScalar{rho2_next ? rho2_next : rho2, rho2_next ? rho2_next_stride : rho2_stride};
    a.llh = llh;
    a.last = last;
    a.first = iter == 0;
    if (llh == GD_LLH_GAUSSIAN) {
        a.a0 = z;
        a.o0 = zin_or_out;
        return dispatch<Ops>(H, [&](auto op) { return decltype(op)::admm_iter_gauss(a, (hipStream_t)stream); });
    }
    // Poisson: spatial u1 / w (RF reads z, u1, w; RI writes u1, w and zin_or_out)
    a.a0 = z; a.a1 = a.o0; a.a2 = a.o1;
    a.o2 = zin_or_out;
    return dispatch<Ops>(H, [&](auto op) { return decltype(op)::admm_iter(a, (hipStream_t)stream); });
}

int gd_wiener(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
              long long alpha_stride, float* x, int N, int H, int W, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H));
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.alpha = GalScalar{alpha, alpha_stride};
    a.o0 = x;
    return dispatch<Ops>(H, [&](auto op) { return decltype(op)::wiener(a, (hipStream_t)stream); });
}

int gd_richardson_lucy(const float* y, const float* psf, long long psf_gstride, int h, int w, int n_iters,
                       float* x, int N, int H, int W, void* otf_half, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H));
    if (n_iters < 0) return fail(GD_ERR_ARG, "n_iters must be >= 0");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.otf = reinterpret_cast<float2*>(otf_half);
    a.o0 = x;
    return dispatch<Ops>(H, [&](auto op) { return decltype(op)::richardson_lucy(a, n_iters, (hipStream_t)stream); });
}

int gd_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_on = on != 0;
    return GD_OK;
}

int gd_profile_collect(void) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (auto& e : g_prof_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(e.stop) != hipSuccess || hipEventElapsedTime(&ms, e.start, e.stop) != hipSuccess)
            return fail(GD_ERR_HIP, "profile event query failed");
        ProfStat& st = g_prof_stats[e.name];
        st.ms += ms;
        st.launches += 1;
        g_prof_pool.push_back(e.start);
        g_prof_pool.push_back(e.stop);
    }
    g_prof_pending.clear();
    return (int)g_prof_stats.size();
}

int gd_profile_get(int i, char* name, int name_len, double* total_ms, long long* launches) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (i < 0 || i >= (int)g_prof_stats.size()) return fail(GD_ERR_ARG, "profile index out of range");
    auto it = g_prof_stats.begin();
    std::advance(it, i);
    if (name && name_len > 0) {
        std::strncpy(name, it->first.c_str(), (size_t)name_len - 1);
        name[name_len - 1] = 0;
    }
    if (total_ms) *total_ms = it->second.ms;
    if (launches) *launches = it->second.launches;
    return GD_OK;
}

int gd_profile_reset(void) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_stats.clear();
    return GD_OK;
}

size_t gd_set_chunk_bytes(size_t bytes) {
    const size_t old = g_chunk_bytes;
    g_chunk_bytes = bytes;
    return old;
}

int gd_subnet_param_count(void) { return gd::subnet::kParams; }

int gd_subnet_features(const void* otf128_half, const float* params, float* feat, int N, void* stream) {
    if (N < 0) return fail(GD_ERR_ARG, "negative batch");
    if (N == 0) return GD_OK;
    ProfScope ps("k_subnet_features<128,0>", (hipStream_t)stream);
    hipLaunchKernelGGL(gd::subnet::k_subnet_features, dim3(N), dim3(gd::subnet::kThreads), 0, (hipStream_t)stream,
                       reinterpret_cast<const float2*>(otf128_half), params, feat, N);
    return check_launch("k_subnet_features");
}

}  // extern "C"
