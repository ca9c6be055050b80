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
// Whole-galaxy kernels (one workgroup per galaxy, spectra on chip) for the Gaussian ADMM path:
//   k_gal_reg / k_gal_reg_init (256^2, registers + LDS, slices of 64 columns; gd_galreg.hpp), k_gal_small
//   (iteration, 32^2 / 64^2) and k_gal_small_p (48^2), k_gal_small_init (init, L <= 64), k_gal_mid /
//   k_gal_mid_init (80^2 ... 160^2, multiples of 16).  The Gaussian state is spectral (|H|^2, G, U1, W~;
//   DESIGN.md section 2); the Poisson state below stays spatial except in the 256^2 two-pass form.
//
// Poisson ADMM state carried between iterations (all [N,1,L,L] fp32): u1, w = v - u2, zin (denoiser
// input) plus y and the half-spectrum OTF.  u2 and v are never stored: u2_{n+1} = Hx_{n+1} - w_n and
// v_{n+1} - u2_{n+1} is all the next X-update needs (algebraically identical to :207-213).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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
    float* s_hh;           // Gaussian spectral state [N][K][L]: |H|^2
    float2* s_g;           //   conj(H) F(max(y,0)/alpha)
    float2* s_u1;          //   F(u1)
    float2* s_w;           //   conj(H) F(v - u2)
    int t_slot;            // image slot of T that row-forward kernels write (RIF_CLAMP -> 1)
    float2* Tw;            // if set: row-forward kernels write here (full-batch layout) instead of T
    const float* ltl;      // Tikhonov |L|^2 half spectrum [*][K][L] (nullptr: filter 'Identity')
    long long ltl_gstride; // elements between galaxies' |L|^2 (0 = one shared filter)
    int otf_bcast;         // LOAD_OTF modes: one OTF for every galaxy (conv_fft_batch's broadcast H)
    float2* s_x;           // Poisson two-pass at 256^2: X (pass A -> pass B), state layout as s_u1
    int gH, gW;            // image rows / columns (the runtime-size path, gd_generic.hpp)
    int pw;                // PSF columns when the PSF is h x pw, not square (0 = h; the runtime-size path)
    int rev;               // k_gal_reg: workgroup b runs galaxy N - 1 - b (the previous launch's last galaxies first)
};

enum RowFwdMode { RF_ITER, RF_PSF_Y, RF_PSF_YP, RF_PSF_RAW, RF_PSF, RF_ONE, RF_TWO, RF_YA, RF_PSF_YAR,
                  RF_PADV, RF_PSF_YPAD, RF_PAD2 };  // RF_PAD*: L/2 x L/2 sources zero-padded to L x L
enum ColMode { C_ITER, C_OTF_INIT, C_OTF_CONV, C_WIENER, C_OTF, C_CONV, C_CONVC, C_CONV2, C_FWD, C_INV,
               C_G_INIT, C_G_ITER, C_G_W1, C_G_ITER_F, C_G_ITER_L, C_G_ITER_FL,  // _F first, _L last iteration
               C_TIKHONOV, C_POWER, C_GX_INIT, C_GX, C_GX_BWD };
enum RowInvMode { RI_ITER, RI_INIT, RI_OUT1, RI_OUT2, RI_RL_FINAL, RI_CROP, RI_CROP_BWD };  // RI_CROP*: L/2 x L/2 sinks
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
template <int L, int NI, int RBX = 0>
struct RowGeo {
    using G = Geo<L>;
    // rows per block, per image (even, divides L): by default up to LPB lines (256 threads) per
    // block, so a single-image kernel takes twice the rows of a two-image one; RBX overrides
    static constexpr int RB = RBX ? RBX : rows_per_block(2 * G::LPB / NI, L);
    static constexpr int PAIRS = RB / 2;    // lines per image
    static constexpr int LINES = NI * PAIRS;
    static constexpr int THREADS = LINES * G::F1;
    // LDS (float2): row buffer | per-line exchange areas | staged input / result rows, aliased
    static constexpr int LDS = cmax(cmax(LINES * G::RLD, LINES * G::XCH), (NI * RB * L + 1) / 2);
    static_assert(RB % 2 == 0 && L % RB == 0, "row pairs must tile the image");
    static_assert(THREADS <= 1024, "block too large");
};

// Split line spectra C = FFT(row_even + i row_odd) (row buffer [line][k]) into the two rows'
// half spectra, stored transposed T[g][im][k][row0 + rr]; consecutive threads take consecutive rows.
template <int L, typename R>
__device__ __forceinline__ void split_store(const Args& a, const float2* rowbuf, int g, int row0, int tid) {
    using G = Geo<L>;
    for (int idx = tid; idx < R::LINES * G::K; idx += R::THREADS) {
        const int m = idx % R::PAIRS, t = idx / R::PAIRS;
        const int k = t % G::K, im = t / G::K;
        const int line = im * R::PAIRS + m;
        const float2 C = rowbuf[line * G::RLD + k];
        const float2 D = rowbuf[line * G::RLD + (k == 0 ? 0 : L - k)];
        // row 2m: (C + conj D)/2 ; row 2m+1: (C - conj D)/(2i) -> adjacent in T: one 16-byte store
        *reinterpret_cast<float4*>((a.Tw ? a.Tw : a.T) + tidx(g, im + a.t_slot, k, row0 + 2 * m, G::K, L)) =
            make_float4(0.5f * (C.x + D.x), 0.5f * (C.y - D.y), 0.5f * (C.y + D.y), 0.5f * (D.x - C.x));
    }
}

// Gather the half spectra of rows 2m, 2m+1 of each image into the Hermitian-extended packed line
// spectrum D = R_even + i R_odd over kx in [0, L) (row buffer [line][k]).  One 16-byte load per
// (image, k, pair): the two rows are adjacent in the transposed layout.
template <int L, typename R>
__device__ __forceinline__ void gather_rows(const Args& a, float2* rowbuf, int g, int row0, int tid) {
    using G = Geo<L>;
    for (int idx = tid; idx < R::LINES * G::K; idx += R::THREADS) {
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
    static constexpr int NI = (MODE == RF_PSF || MODE == RF_ONE || MODE == RF_YA || MODE == RF_PADV) ? 1 : 2;
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
    } else if constexpr (MODE == RF_PSF || MODE == RF_PSF_Y || MODE == RF_PSF_YP || MODE == RF_PSF_RAW ||
                         MODE == RF_PSF_YAR) {
        if (im == 0)
            return make_float4(shifted_psf(a, g, r, c, L), shifted_psf(a, g, r, c + 1, L),
                               shifted_psf(a, g, r, c + 2, L), shifted_psf(a, g, r, c + 3, L));
        const float4 y = ld4(a.y + pix);
        if constexpr (MODE == RF_PSF_RAW) return y;
        if constexpr (MODE == RF_PSF_YAR) {                            // y / alpha (Tikhonov: no max)
            const float al = a.alpha(g);
            return make_float4(y.x / al, y.y / al, y.z / al, y.w / al);
        }
        float4 yp = make_float4(fmaxf(y.x, 0.f), fmaxf(y.y, 0.f), fmaxf(y.z, 0.f), fmaxf(y.w, 0.f));
        if constexpr (MODE == RF_PSF_YP) {
            st4(a.o0 + pix, yp);                                       // Richardson-Lucy x0 = max(y, 0)
            return yp;
        } else {
            const float al = a.alpha(g);                               // max(y,0) / alpha
            return make_float4(yp.x / al, yp.y / al, yp.z / al, yp.w / al);
        }
    } else if constexpr (MODE == RF_PADV || MODE == RF_PSF_YPAD || MODE == RF_PAD2) {
        // UnrolledADMMGaussian (models/unrolled_admm_gaussian.py): sources are Lh x Lh images placed at
        // the origin of the 2Lh x 2Lh grid.  pad_double + ifftshift put pixel i at (i - Lh/2) mod 2Lh
        // instead; that shift is a common phase of every spectrum, which cancels in conj(H) Y and |H|^2
        // and is undone by fftshift + crop_half.
        constexpr int Lh = L / 2;
        if constexpr (MODE == RF_PSF_YPAD) {
            if (im == 0)                                               // PSF (Lh x Lh) centred on (0,0)
                return make_float4(shifted_psf(a, g, r, c, L), shifted_psf(a, g, r, c + 1, L),
                                   shifted_psf(a, g, r, c + 2, L), shifted_psf(a, g, r, c + 3, L));
        }
        if (r >= Lh || c >= Lh) return make_float4(0.f, 0.f, 0.f, 0.f);
        const size_t p = ((size_t)g * Lh + r) * Lh + c;
        if constexpr (MODE == RF_PSF_YPAD) {                           // max(y, 0)
            const float4 y = ld4(a.y + p);
            return make_float4(fmaxf(y.x, 0.f), fmaxf(y.y, 0.f), fmaxf(y.z, 0.f), fmaxf(y.w, 0.f));
        } else if constexpr (MODE == RF_PAD2) {
            return ld4((im == 0 ? a.a0 : a.a1) + p);
        } else {
            // rho z - u (XUpdateGaussian :91), optionally after the dual update of the previous
            // iteration u = u + rho_prev (x_prev - z) (:145), written back in place (o1 = a1)
            const float4 z = ld4(a.a0 + p);
            const float rho = a.rho1(g);
            float4 u = a.a1 ? ld4(a.a1 + p) : make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.a2) {
                const float4 xp = ld4(a.a2 + p);
                const float rp = a.rho2(g);
                u = make_float4(u.x + rp * (xp.x - z.x), u.y + rp * (xp.y - z.y), u.z + rp * (xp.z - z.z),
                                u.w + rp * (xp.w - z.w));
                st4(a.o1 + p, u);
            }
            return make_float4(rho * z.x - u.x, rho * z.y - u.y, rho * z.z - u.z, rho * z.w - u.w);
        }
    } else if constexpr (MODE == RF_ONE) {
        return ld4(a.a0 + pix);
    } else if constexpr (MODE == RF_YA) {
        const float4 y = ld4(a.y + pix);
        const float al = a.alpha(g);                                   // max(y,0) / alpha
        return make_float4(fmaxf(y.x, 0.f) / al, fmaxf(y.y, 0.f) / al, fmaxf(y.z, 0.f) / al, fmaxf(y.w, 0.f) / al);
    } else {
        return ld4((im == 0 ? a.a0 : a.a1) + pix);
    }
}

template <int L, int MODE, int RBX = 0>
__global__ __launch_bounds__((RowGeo<L, RfTraits<MODE>::NI, RBX>::THREADS)) void k_row_fwd(Args a) {
    constexpr int NI = RfTraits<MODE>::NI;
    using G = Geo<L>;
    using R = RowGeo<L, NI, RBX>;
    constexpr int F1 = G::F1, F2 = G::F2;
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 lds[R::LDS];
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
    split_store<L, R>(a, lds, g, row0, tid);
}

// ---------------------------------------------------------------- PSF row spectra (init)
// psf_to_otf's row transform (utils/utils_torch.py:84-91), restricted to the h non-zero rows of the
// circularly shifted, zero-padded PSF: psf row i sits in padded row (i - h/2) mod L and its pixel jj in
// padded column (jj - h/2) mod L.  Rows 2p, 2p+1 ride one complex line (same image: the packing
// rule), split after the FFT and stored compactly as P[kx][i] (i < h, contiguous) in T slot 1, where
// k_col<C_G_INIT> picks its OTF column up with a few coalesced loads.
// TO_STATE: write the compact rows into this galaxy's U1 state slot instead (the fused init reads them
// there; U1 is first written by iteration 0, which does not read it), [kx][i] at s_u1 + g K L.
template <int L, bool TO_STATE = false>
__global__ __launch_bounds__(256) void k_psf_rows(Args a) {
    using G = Geo<L>;
    constexpr int F1 = G::F1, F2 = G::F2, LPB = G::LPB, K = G::K;
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 lds[cmax(LPB * G::RLD, LPB * G::XCH)];
    const int tid = threadIdx.x, line = tid / F1, j = tid - line * F1;
    const int h = a.h, c0 = h >> 1, pairs = h >> 1;
    const int blocks_per_g = (pairs + LPB - 1) / LPB;
    const int g = blockIdx.x / blocks_per_g;
    const int p0 = (blockIdx.x - g * blocks_per_g) * LPB;
    fill_twiddles<L>(tw, tid, 256);
    const int p = p0 + line;
    const float* ps = a.psf + (long long)g * a.psf_gstride + (long long)(2 * p) * h;
    float2 v[F2];
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        int jj = j + F1 * s + c0;
        if (jj >= L) jj -= L;
        v[s] = (p < pairs && jj < h) ? make_float2(ps[jj], ps[h + jj]) : make_float2(0.f, 0.f);
    }
    __syncthreads();  // twiddles
    line_fft<L, false>(v, j, lds + line * G::XCH, tw);
    __syncthreads();  // exchange areas -> row buffer
#pragma unroll
    for (int s = 0; s < F2; ++s) lds[line * G::RLD + j + F1 * s] = v[s];
    __syncthreads();
    float2* P = TO_STATE ? a.s_u1 + (size_t)g * K * L : a.T + tidx(g, 1, 0, 0, K, L);
    for (int idx = tid; idx < LPB * K; idx += 256) {
        const int m = idx % LPB, k = idx / LPB;
        if (p0 + m >= pairs) continue;
        const float2 C = lds[m * G::RLD + k];
        const float2 D = lds[m * G::RLD + (k == 0 ? 0 : L - k)];
        // row 2p: (C + conj D)/2 ; row 2p+1: (C - conj D)/(2i) -> adjacent: one 16-byte store
        float4 o = make_float4(0.5f * (C.x + D.x), 0.5f * (C.y - D.y), 0.5f * (C.y + D.y), 0.5f * (D.x - C.x));
        if (TO_STATE && k == 0) {
            // rows' bins 0 and L/2 are real (D = C there): kx = 0 holds P_0 + i P_{L/2}, the packed
            // column the fused init's line 0 transforms (kx = L/2 is not read)
            const float2 Cn = lds[m * G::RLD + L / 2];
            o = make_float4(C.x, Cn.x, C.y, Cn.y);
        }
        *reinterpret_cast<float4*>(P + (size_t)k * h + 2 * (p0 + m)) = o;
    }
}

// ---------------------------------------------------------------- C: column pass
template <int MODE>
struct ColTraits {
    static constexpr bool IN2 = (MODE == C_ITER || MODE == C_OTF_INIT || MODE == C_OTF_CONV ||
                                 MODE == C_WIENER || MODE == C_CONV2 || MODE == C_TIKHONOV || MODE == C_GX_INIT ||
                                 MODE == C_GX_BWD);
    static constexpr bool OUT2 = (MODE == C_ITER || MODE == C_CONV2);
    static constexpr bool HAS_OUT = (MODE != C_OTF && MODE != C_FWD && MODE != C_G_W1 && MODE != C_POWER);
    static constexpr bool STORE_OTF = (MODE == C_OTF_INIT || MODE == C_OTF_CONV || MODE == C_OTF);
    static constexpr bool LOAD_OTF = (MODE == C_ITER || MODE == C_CONV || MODE == C_CONVC || MODE == C_CONV2);
    static constexpr bool FWD = (MODE != C_INV);
};

// Gaussian ADMM iteration for one spectral element, entirely in the spectral domain (every step of
// models/Unrolled_ADMM.py:207-213 is linear for llh='Gaussian'), with the v - u2 state kept
// premultiplied by conj(H) (W~ = conj(H) W) so only |H|^2 and G are needed:
//   X    = (rho1 (Z - U1) + rho2 W~) / (rho1 |H|^2 + rho2)        X_Update :315-319
//   U1'  = (U1 + X) - Z                                            :212
//   U2~  = |H|^2 X - W~                     (= conj(H) (H X - W))   :213
//   V~   = (rho2' (|H|^2 X + U2~) + G) / (1 + rho2')               V step :335-336
//   W~'  = V~ - U2~ ;  returns (X + U1') / L^2 (next denoiser input) | X / L^2 (last iteration)
// First iteration: U1 = 0 (not read); W~ = conj(H) V1 was written by the init (C_G_W1).
#ifndef GD_RCP_DIV
#define GD_RCP_DIV 1  // Gaussian spectral update: reciprocal-multiply instead of division (-5 % iteration time)
#endif
// Streaming (single-use per iteration) state traffic: stores non-temporal, loads ordinary.  Measured on
// op_admm_iter (round 1): non-temporal stores (U1, W~, zin) 1.673/1.692 -> 1.658/1.666 ms; non-temporal loads
// (z, |H|^2, G, U1, W~) 1.75-1.87 ms, i.e. slower.  The parked registers stay ordinary (re-read by the same CU).
__device__ __forceinline__ float ld_s(const float* p) { return *p; }
__device__ __forceinline__ float2 ld_s(const float2* p) { return *p; }
__device__ __forceinline__ void st_s(float* p, float v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_s(float2* p, float2 v) {
    unsigned long long u;
    __builtin_memcpy(&u, &v, 8);
    __builtin_nontemporal_store(u, reinterpret_cast<unsigned long long*>(p));
}
// Gaussian ADMM state layout (|H|^2, G, U1, W~; [N][K][L], one column of L bins per (galaxy, kx)).  At
// L = 256 the bins inside a column are stored in the order the fused iteration's column lines hold
// them (lane j of a 16-lane line holds ky = j + 16 s), so a lane's bins are contiguous and move with
// 16-byte accesses (k_gal_reg): complex arrays at 32 (s >> 1) + 2 j + (s & 1), |H|^2 at 64 (s >> 2) +
// 4 j + (s & 3).  Other sizes keep ky order.  Every kernel touching this state indexes it through
// sidx_* / sflat_* (the state buffer is opaque to callers).
typedef float f4v __attribute__((ext_vector_type(4)));
template <int L>
__device__ __forceinline__ int sidx_c(int ky) {
    if constexpr (L == 256) {
        const int j = ky & 15, s = ky >> 4;
        return 32 * (s >> 1) + 2 * j + (s & 1);
    } else {
        return ky;
    }
}
template <int L>
__device__ __forceinline__ int sidx_h(int ky) {
    if constexpr (L == 256) {
        const int j = ky & 15, s = ky >> 4;
        return 64 * (s >> 2) + 4 * j + (s & 3);
    } else {
        return ky;
    }
}
// flat offsets o = (g K + kx) L + ky -> storage offsets (columns start at multiples of L)
template <int L>
__device__ __forceinline__ size_t sflat_c(size_t o) {
    if constexpr (L == 256) return (o & ~size_t(255)) | (size_t)sidx_c<L>((int)(o & 255));
    else return o;
}
template <int L>
__device__ __forceinline__ size_t sflat_h(size_t o) {
    if constexpr (L == 256) return (o & ~size_t(255)) | (size_t)sidx_h<L>((int)(o & 255));
    else return o;
}
// Iteration 0's W~1 = (rho2 (|H|^2 F(x0) + 0) + G) / (1 + rho2) (the first V step, models/
// Unrolled_ADMM.py:335-336, premultiplied by conj(H); the arithmetic of the reference's first loop body)
// is DEFERRED at every size: the init leaves F(x0) itself in the W~ slot and the first iteration - which
// reads |H|^2, G and that slot anyway, with rho2 = rho2[0] - forms W~1 bin by bin.  The init then never
// re-reads |H|^2 and G (1.5 half spectra per galaxy less) and reads no penalty parameter at all, so it
// can run while the SubNet computes the rhos (gd_admm_init_reads_rho).
__device__ __forceinline__ float2 w1_value(float hh, float2 Gk, float2 Xk, float r2n) {
    const float d0 = 1.0f + r2n;
#if GD_RCP_DIV
    const float rd = __builtin_amdgcn_rcpf(d0);  // as gauss_math's 1/(1 + rho2'): per galaxy, not two divisions per bin
    return make_float2((r2n * (hh * Xk.x + 0.0f) + Gk.x) * rd, (r2n * (hh * Xk.y + 0.0f) + Gk.y) * rd);
#else
    return make_float2((r2n * (hh * Xk.x + 0.0f) + Gk.x) / d0, (r2n * (hh * Xk.y + 0.0f) + Gk.y) / d0);
#endif
}

struct GState {  // one bin's Gaussian state as loaded (U1 / G zero where the variant skips them)
    float hh;
    float2 G, U1, W;
};
template <int L, bool FIRST, bool LAST>
__device__ __forceinline__ GState gauss_load(const Args& a, size_t o) {
    GState st;
    const size_t oc = sflat_c<L>(o);
    st.hh = ld_s(a.s_hh + sflat_h<L>(o));
    st.G = make_float2(0.f, 0.f);
    st.U1 = make_float2(0.f, 0.f);
    if constexpr (!LAST || FIRST) st.G = ld_s(a.s_g + oc);
    if constexpr (!FIRST) st.U1 = ld_s(a.s_u1 + oc);
    st.W = ld_s(a.s_w + oc);
    return st;
}
// One bin of the Gaussian iteration (the arithmetic every fused and chunked kernel shares): returns the
// next denoiser input's bin (X on the last iteration) and the updated U1, W~ (not on the last).
template <bool LAST>
__device__ __forceinline__ float2 gauss_math(float hh, float2 Gk, float2 U1, float2 Wt, float2 Zk, float r1, float r2,
                                             float r2n, float inv_n, float2& U1o, float2& Wo) {
    const float lhs = r1 * hh + r2;
    const float2 A = csub(Zk, U1);
#if GD_RCP_DIV
    const float rl = __builtin_amdgcn_rcpf(lhs);
    const float2 X = make_float2((r1 * A.x + r2 * Wt.x) * rl, (r1 * A.y + r2 * Wt.y) * rl);
#else
    const float2 X = make_float2((r1 * A.x + r2 * Wt.x) / lhs, (r1 * A.y + r2 * Wt.y) / lhs);
#endif
    if constexpr (LAST) return cscale(X, inv_n);
    const float2 U1n = csub(cadd(U1, X), Zk);
    const float2 HHX = cscale(X, hh);
    const float2 U2t = csub(HHX, Wt);
    const float d = 1.0f + r2n;
#if GD_RCP_DIV
    const float rd = __builtin_amdgcn_rcpf(d);
    const float2 Vt = make_float2((r2n * (HHX.x + U2t.x) + Gk.x) * rd, (r2n * (HHX.y + U2t.y) + Gk.y) * rd);
#else
    const float2 Vt = make_float2((r2n * (HHX.x + U2t.x) + Gk.x) / d, (r2n * (HHX.y + U2t.y) + Gk.y) / d);
#endif
    U1o = U1n;
    Wo = csub(Vt, U2t);
    return cscale(cadd(X, U1n), inv_n);
}
// gauss_math with the last-iteration choice at run time (uniform per launch): the same operations, in
// the same order, as gauss_math<false> / <true>
__device__ __forceinline__ float2 gauss_math_rt(float hh, float2 Gk, float2 U1, float2 Wt, float2 Zk, float r1,
                                                float r2, float r2n, float inv_n, float2& U1o, float2& Wo, bool last) {
    if (last) return gauss_math<true>(hh, Gk, U1, Wt, Zk, r1, r2, r2n, inv_n, U1o, Wo);
    return gauss_math<false>(hh, Gk, U1, Wt, Zk, r1, r2, r2n, inv_n, U1o, Wo);
}
template <int L, bool FIRST, bool LAST>
__device__ __forceinline__ float2 gauss_iter_st(const Args& a, size_t o, float2 Zk, const GState& st, float r1,
                                                float r2, float r2n, bool valid, float inv_n) {
    const float hh = st.hh;
    const float2 U1 = st.U1, Gk = st.G;
    float2 Wt = st.W;
    if constexpr (FIRST) Wt = w1_value(hh, Gk, st.W, r2);  // the slot holds F(x0)
    const float lhs = r1 * hh + r2;
    const float2 A = csub(Zk, U1);
#if GD_RCP_DIV
    // one hardware reciprocal per bin (1 ulp) instead of two IEEE divisions; 1/(1 + rho2') per galaxy
    const float rl = __builtin_amdgcn_rcpf(lhs);
    const float2 X = make_float2((r1 * A.x + r2 * Wt.x) * rl, (r1 * A.y + r2 * Wt.y) * rl);
#else
    const float2 X = make_float2((r1 * A.x + r2 * Wt.x) / lhs, (r1 * A.y + r2 * Wt.y) / lhs);
#endif
    if constexpr (LAST) return cscale(X, inv_n);
    const float2 U1n = csub(cadd(U1, X), Zk);
    const float2 HHX = cscale(X, hh);
    const float2 U2t = csub(HHX, Wt);
    const float d = 1.0f + r2n;
#if GD_RCP_DIV
    const float rd = __builtin_amdgcn_rcpf(d);
    const float2 Vt = make_float2((r2n * (HHX.x + U2t.x) + Gk.x) * rd, (r2n * (HHX.y + U2t.y) + Gk.y) * rd);
#else
    const float2 Vt = make_float2((r2n * (HHX.x + U2t.x) + Gk.x) / d, (r2n * (HHX.y + U2t.y) + Gk.y) / d);
#endif
    if (valid) {
        st_s(a.s_u1 + sflat_c<L>(o), U1n);
        st_s(a.s_w + sflat_c<L>(o), csub(Vt, U2t));
    }
    return cscale(cadd(X, U1n), inv_n);
}
template <int L, bool FIRST, bool LAST>
__device__ __forceinline__ float2 gauss_iter_elem(const Args& a, size_t o, float2 Zk, float r1, float r2,
                                                  float r2n, bool valid, float inv_n) {
    return gauss_iter_st<L, FIRST, LAST>(a, o, Zk, gauss_load<L, FIRST, LAST>(a, o), r1, r2, r2n, valid, inv_n);
}

#ifndef GD_COL_LEAN
#define GD_COL_LEAN 0  // measured: no effect on the chunked paths (bound by L2-fabric traffic, not occupancy)
#endif
#ifndef GD_COL_DPP
#define GD_COL_DPP 0  // same (occupancy 4 -> 6-7, no change in time)
#endif
// VAR: experiment switch for tools/kbench.hip (0 = production; 1 = no FFTs, memory only)
template <int L, int MODE, int VAR = 0>
__global__ __launch_bounds__(256) void k_col(Args a) {
    using G = Geo<L>;
    using TR = ColTraits<MODE>;
    constexpr int F1 = G::F1, F2 = G::F2, K = G::K;
    // lean twiddles (12 registers instead of 30 per line) where two spectra are live at once
    constexpr bool CLEAN = GD_COL_LEAN && F2 == 16;
    // register (DPP) transposes for 16 x 16 lines: no LDS exchange areas, occupancy set by VGPRs
    constexpr bool CDPP = GD_COL_DPP && F1 == 16 && F2 == 16;
    __shared__ float2 tw[L];
    __shared__ float2 xch[CDPP ? 1 : G::COL_LDS];
    const int tid = threadIdx.x;
    const int line = tid / F1, j = tid - line * F1;
    const int f = blockIdx.x * G::LPB + line;
    const bool valid = f < a.N * K;
    const int fc = valid ? f : 0;
    const int g = fc / K, kx = fc - g * K;
    fill_twiddles<L>(tw, tid, 256);
    float2* my = CDPP ? nullptr : xch + line * G::XCH;

    float2 P[F2], Q[F2];
    const size_t c0 = tidx(g, 0, kx, 0, K, L), c1 = tidx(g, 1, kx, 0, K, L);
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        P[s] = a.T[(MODE == C_G_W1 ? c1 : c0) + j + F1 * s];  // C_G_W1: x0's row spectra in slot 1
        if constexpr (TR::IN2) Q[s] = a.T[c1 + j + F1 * s];
    }
    __syncthreads();  // twiddles
    if constexpr (TR::FWD && VAR != 1) {
        line_fft<L, false, CLEAN, CDPP>(P, j, my, tw);
        if constexpr (TR::IN2) line_fft<L, false, CLEAN, CDPP>(Q, j, my, tw);
    }
    // C_G_INIT: the OTF column H(., kx) from the PSF's row spectra P[kx][i] (k_psf_rows, T slot 1):
    // padded row ky holds psf row i = (ky + h/2) mod L when i < h, zero otherwise; then the column FFT.
    float2 Hc[MODE == C_G_INIT ? F2 : 1];
    if constexpr (MODE == C_G_INIT) {
        const int h = a.h, c0p = h >> 1;
        const float2* Pr = a.T + tidx(g, 1, 0, 0, K, L) + (size_t)kx * h;
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            int i = j + F1 * s + c0p;
            if (i >= L) i -= L;
            Hc[s] = (i < h) ? Pr[i] : make_float2(0.f, 0.f);
        }
        line_fft<L, false, CLEAN, CDPP>(Hc, j, my, tw);
    }
    constexpr float inv_n = float(1.0 / double(L * L));  // exact for L = 2^k
    const size_t ob = ((size_t)g * K + kx) * L;
    const float al = (MODE == C_OTF_INIT || MODE == C_WIENER || MODE == C_G_INIT || MODE == C_GX_INIT) ? a.alpha(g) : 1.f;
    const float rgx = (MODE == C_GX || MODE == C_GX_BWD) ? a.rho1(g) : 0.f;
    float drho = 0.f;  // C_GX_BWD: this lane's part of d loss / d rho
    const float lam = (MODE == C_TIKHONOV) ? a.rho1(g) : 0.f;  // Tikhonov lambda rides in rho1
    constexpr bool giter = (MODE == C_G_ITER || MODE == C_G_ITER_F || MODE == C_G_ITER_L || MODE == C_G_ITER_FL);
    constexpr bool gfirst = (MODE == C_G_ITER_F || MODE == C_G_ITER_FL);
    constexpr bool glast = (MODE == C_G_ITER_L || MODE == C_G_ITER_FL);
    const float r1 = (MODE == C_ITER || giter) ? a.rho1(g) : 0.f;
    const float r2 = (MODE == C_ITER || giter) ? a.rho2(g) : 0.f;
    const float r2n = (giter && !glast) ? a.rho2n(g) : 0.f;
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        const int ky = j + F1 * s;
        float2 Hk = make_float2(0.f, 0.f);
        if constexpr (TR::LOAD_OTF) Hk = a.otf[(a.otf_bcast ? (size_t)kx * L : ob) + ky];
        if constexpr (TR::STORE_OTF || MODE == C_WIENER || MODE == C_TIKHONOV) Hk = P[s];
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
        } else if constexpr (MODE == C_G_INIT) {
            // init_l2 (models/Unrolled_ADMM.py:170-175) and the Gaussian constants:
            //   |H|^2, G = conj(H) F(y/alpha) kept as state;  X0 = G / (|H|^2 + 1/alpha)
            const float2 Hk2 = Hc[s];
            const float hh = Hk2.x * Hk2.x + Hk2.y * Hk2.y;
            const float2 Gk = cmulc(P[s], Hk2);
            if (valid) {
                a.s_hh[sflat_h<L>(ob + ky)] = hh;
                a.s_g[sflat_c<L>(ob + ky)] = a.llh == GD_LLH_POISSON ? Hk2 : Gk;  // Poisson two-pass: the OTF
            }
            const float lhs = hh + 1.0f / al;
            P[s] = cscale(make_float2(Gk.x / lhs, Gk.y / lhs), inv_n);
        } else if constexpr (giter) {
            P[s] = gauss_iter_elem<L, gfirst, glast>(a, ob + ky, P[s], r1, r2, r2n, valid, inv_n);
        } else if constexpr (MODE == C_G_W1) {
            // iteration 0's W~ = conj(H) V1 = (rho2 (|H|^2 X0 + 0) + G) / (1 + rho2): the V step
            // (models/Unrolled_ADMM.py:335-336) with Hx = H X0 and u2 = 0, premultiplied by conj(H)
            // F(x0): the first iteration forms W~1 (Poisson two-pass: H F(x0), pass B<INIT>'s input)
            if (valid)
                a.s_w[sflat_c<L>(ob + ky)] = a.llh == GD_LLH_POISSON ? cmul(a.s_g[sflat_c<L>(ob + ky)], P[s]) : P[s];
        } else if constexpr (MODE == C_WIENER) {
            // models/Wiener.py:16-18: conj(H) F(y) / (|H|^2 + 350/alpha)
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float div = HtH + 350.0f / al;
            const float2 num = cmulc(Q[s], Hk);
            P[s] = cscale(make_float2(num.x / div, num.y / div), inv_n);
        } else if constexpr (MODE == C_TIKHONOV) {
            // models/Tikhonet.py:19-29: conj(H) F(y/alpha) / (|H|^2 + lam)        (filter 'Identity')
            //                           conj(H) F(y/alpha) / (|H|^2 + lam |L|^2)  (filter 'Laplacian')
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float div = a.ltl ? HtH + lam * a.ltl[(size_t)g * a.ltl_gstride + (size_t)kx * L + ky] : HtH + lam;
            const float2 num = cmulc(Q[s], Hk);
            P[s] = cscale(make_float2(num.x / div, num.y / div), inv_n);
        } else if constexpr (MODE == C_GX_INIT) {
            // UnrolledADMMGaussian (models/unrolled_admm_gaussian.py:111-127): H from the PSF, Y = F(max(y,0));
            // state |H|^2 and G = Y conj(H); x0 spectrum (Y Ht) / (HtH + 1/alpha)
            const float2 Hk2 = P[s];
            const float hh = Hk2.x * Hk2.x + Hk2.y * Hk2.y;
            const float2 Gk = cmulc(Q[s], Hk2);
            if (valid) {
                a.s_hh[ob + ky] = hh;
                a.s_g[ob + ky] = Gk;
            }
            const float lhs = hh + 1.0f / al;
            P[s] = cscale(make_float2(Gk.x / lhs, Gk.y / lhs), inv_n);
        } else if constexpr (MODE == C_GX) {
            // XUpdateGaussian (:89-93): X = (Ht Y + F(rho z - u)) / (rho + HtH); X kept for the backward
            const float hh = a.s_hh[ob + ky];
            const float2 Gk = a.s_g[ob + ky];
            const float lhs = rgx + hh;
            const float2 rhs = cadd(Gk, P[s]);
            const float2 X = make_float2(rhs.x / lhs, rhs.y / lhs);
            if (a.s_w && valid) a.s_w[ob + ky] = X;
            P[s] = cscale(X, inv_n);
        } else if constexpr (MODE == C_GX_BWD) {
            // adjoint of the X update (self-adjoint: real, symmetric 1/D): dv = crop IFFT(F(pad g) / D);
            // d/drho = <pad g, IFFT((F(pad z) - X) / D)> = (1/L^2) sum_k Re(conj(Gg) (Z - X)) / D over the
            // full spectrum: half-spectrum bins other than kx = 0, L/2 count twice
            const float hh = a.s_hh[ob + ky];
            const float D = rgx + hh;
            const float2 X = a.s_w[ob + ky];
            const float2 d = csub(Q[s], X);
            const float wk = (kx == 0 || 2 * kx == L) ? 1.f : 2.f;
            drho += wk * (P[s].x * d.x + P[s].y * d.y) / D;
            P[s] = cscale(make_float2(P[s].x / D, P[s].y / D), inv_n);
        } else if constexpr (MODE == C_POWER) {
            // |F(x)|^2 of a real filter image (the Laplacian's LtL, models/Tikhonet.py:26-27)
            if (valid) a.s_hh[ob + ky] = P[s].x * P[s].x + P[s].y * P[s].y;
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
    if constexpr (MODE == C_GX_BWD) {
#pragma unroll
        for (int off = F1 / 2; off > 0; off >>= 1) drho += __shfl_xor(drho, off, F1);
        if (valid && j == 0) a.o2[(size_t)g * K + kx] = drho * inv_n;
    }
    if constexpr (TR::HAS_OUT && MODE != C_FWD && VAR != 1) {
        line_fft<L, true, CLEAN, CDPP>(P, j, my, tw);
        if constexpr (TR::OUT2) line_fft<L, true, CLEAN, CDPP>(Q, j, my, tw);
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

// A copy of v the compiler cannot see through: addresses recomputed from it are not CSE'd with
// (and kept live from) an earlier phase's identical computation (register budget: 128 VGPRs at
// 1024 threads).
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// Optional per-workgroup phase timestamps (tools/kbench_fused.hip builds with GD_FUSED_TRACE=1).
#if GD_FUSED_TRACE
__device__ unsigned long long* g_fused_trace;
#define GD_TRACE(k)                                                                                   \
    if (tid == 0) g_fused_trace[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define GD_TRACE(k)
#endif

template <int L>
struct FusedGeo {
    static constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2, K = L / 2 + 1;
    static constexpr int THREADS = 1024, LINES = THREADS / F1;
    static constexpr int NP = L / 2, PPL = NP / LINES;  // row pairs; pairs per line
    static constexpr int KS = L / 4;                    // columns per slice (one per line)
    static constexpr int SLD = 2 * KS + 4;              // slice layout [pair][SLD]: X_p[kx], X_p[L-kx]
    static constexpr int ALD = KS + 2;                  // row layout [row][ALD]: one slice's columns
    static constexpr int XCH = xch_elems<L>();
    static constexpr int U = cmax(cmax(NP * SLD, L * ALD), LINES * XCH);
    static_assert(LINES == KS, "one column per line and slice");
    static_assert(NP == 2 * LINES && PPL == 2, "two row pairs per line; half the rows per inverse pass");
    static_assert(KS % F1 == 0 && (L / 2) % F1 == 0, "slice edges on lane-register boundaries");
    static_assert(L <= THREADS && (NP * KS) % THREADS == 0, "Nyquist column: one element per thread");
};

// Column c of a slice from S = [pair][SLD] holding X_p[kx] at [c] and X_p[(L - kx) mod L] at [KS + c]:
// row y's half spectrum R_y[kx] = (X + conj X')/2 (y even) or (X - conj X')/(2i) (y odd).
template <int L, int SLD = FusedGeo<L>::SLD>
__device__ __forceinline__ void fused_gather(const float2* S, int c, int j, float2 (&C)[FusedGeo<L>::F2]) {
    using FG = FusedGeo<L>;
    c = opaque(c);
    j = opaque(j);
#pragma unroll
    for (int s = 0; s < FG::F2; ++s) {
        const int y = j + FG::F1 * s;
        const float2 u = S[(y >> 1) * SLD + c], v = S[(y >> 1) * SLD + FG::KS + c];
        C[s] = (y & 1) ? make_float2(0.5f * (u.y + v.y), 0.5f * (v.x - u.x))
                       : make_float2(0.5f * (u.x + v.x), 0.5f * (u.y - v.y));
    }
}

// Workgroup barrier that orders LDS only: outstanding global loads and stores stay in flight
// (__syncthreads would drain them at every phase boundary).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---- helpers of the fused Gaussian init at 256^2 (k_gal_reg_init, gd_galreg.hpp):
//   y -> max(y,0)/alpha -> R, A, B with the OTF column built in-kernel: |H|^2, G (state), X0 =
//   G / (|H|^2 + 1/alpha) -> inverse -> I: x0 = clamp(., 0, 1) -> zin   (RF_YA, C_G_INIT, RIF_CLAMP)
// The OTF column kx comes from the PSF's compact row spectra (k_psf_rows<L, true>, parked in the U1
// slot): placed row ky holds psf row i = (ky + h/2) mod L when i < h.  Line 0 carries columns 0 and
// L/2 (real over the rows) packed as P0 + i P_{L/2}, like the data, and splits them after the FFT.
template <int L>
__device__ __forceinline__ void init_hload(const Args& a, float2 (&Hc)[FusedGeo<L>::F2], int g, int kx, int j) {
    using FG = FusedGeo<L>;
    static_assert((L & (L - 1)) == 0, "power-of-two side");
    const int h = a.h, c0p = h >> 1;
    const float2* P0 = a.s_u1 + (size_t)g * FG::K * L + (size_t)opaque(kx) * h;  // kx = 0: P_0 + i P_{L/2}
    j = opaque(j);
    // h <= 64 (the host checks): rows ky in [2 F1, L - 2 F1) are zero for every lane, so only lane
    // registers 0, 1, F2-2, F2-1 are loaded and the others are compile-time zeros (the first DFT
    // stage folds them away)
    static_assert(FG::F1 == 16 && FG::F2 == 16, "sparse OTF column for 16 x 16 lines");
#pragma unroll
    for (int s = 0; s < FG::F2; ++s) {
        Hc[s] = make_float2(0.f, 0.f);
        if (s < 2 || s >= FG::F2 - 2) {
            const int i = (j + FG::F1 * s + c0p) & (L - 1);
            if (i < h) Hc[s] = P0[i];
        }
    }
}
// init_hload in two halves: the 4 loaded registers (s = 0, 1, F2-2, F2-1) issued early (h4), then the
// column assembled from them with the compile-time zeros (same values as init_hload)
template <int L>
__device__ __forceinline__ void init_hload4(const Args& a, float2 (&h4)[4], int g, int kx, int j) {
    using FG = FusedGeo<L>;
    const int h = a.h, c0p = h >> 1;
    const float2* P0 = a.s_u1 + (size_t)g * FG::K * L + (size_t)opaque(kx) * h;
    j = opaque(j);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int s = t < 2 ? t : FG::F2 - 4 + t;
        const int i = (j + FG::F1 * s + c0p) & (L - 1);
        h4[t] = i < h ? P0[i] : make_float2(0.f, 0.f);
    }
}
template <int L>
__device__ __forceinline__ void init_hcol(float2 (&Hc)[FusedGeo<L>::F2], const float2 (&h4)[4]) {
    using FG = FusedGeo<L>;
#pragma unroll
    for (int s = 0; s < FG::F2; ++s) Hc[s] = make_float2(0.f, 0.f);
    Hc[0] = h4[0];
    Hc[1] = h4[1];
    Hc[FG::F2 - 2] = h4[2];
    Hc[FG::F2 - 1] = h4[3];
}
// init_l2 (models/Unrolled_ADMM.py:170-175) per bin: |H|^2, G = conj(H) F(max(y,0)/alpha) kept as
// state; returns X0 / L^2 = G / (|H|^2 + 1/alpha) / L^2 (the arithmetic of k_col<C_G_INIT>)
template <int L>
__device__ __forceinline__ float2 init_bin(const Args& a, size_t o, float2 Yk, float2 Hk, float al, float inv_n,
                                           bool store_h = false) {
    const float hh = Hk.x * Hk.x + Hk.y * Hk.y;
    const float2 Gk = cmulc(Yk, Hk);
    a.s_hh[sflat_h<L>(o)] = hh;
    a.s_g[sflat_c<L>(o)] = store_h ? Hk : Gk;  // Poisson (two-pass): the OTF itself in the G slot
    const float lhs = hh + 1.0f / al;
    return cscale(make_float2(Gk.x / lhs, Gk.y / lhs), inv_n);
}
// iteration 0's W~ (k_col<C_G_W1>'s arithmetic): the V step (:335-336) with Hx = H X0, u2 = 0, times conj(H)
template <int L>
__device__ __forceinline__ void w1_bin(const Args& a, size_t o, float2 Xk) {
    // F(x0): the first iteration forms W~1 (Poisson two-pass: H F(x0), pass B<INIT>'s input)
    a.s_w[sflat_c<L>(o)] = a.llh == GD_LLH_POISSON ? cmul(a.s_g[sflat_c<L>(o)], Xk) : Xk;
}
#include "gd_galreg.hpp"  // k_gal_reg: the 512-thread, register-resident fused iteration
#include "gd_rlreg.hpp"   // k_rl_reg: the whole Richardson-Lucy loop per galaxy on the same skeleton
#include "gd_poisreg.hpp" // k_pois_b: Poisson pass B (pass A is k_gal_reg<L, true>)

// Small-image helpers (L <= 128, spectra in LDS as D[kx][ky]):
// a line's forward-FFT result (packed rows r, r+1) -> the two rows' half spectra, via the line's own
// exchange area (F1 (F2 + 1) >= L + 2 for every plan)
template <int L>
__device__ __forceinline__ void small_split(const float2 (&v)[Plan<L>::F2], int j, float2* my, float2* D, int r) {
    constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2, K = L / 2 + 1;
#pragma unroll
    for (int s = 0; s < F2; ++s) my[j + F1 * s] = v[s];
    wave_lds_sync();
    for (int k = j; k < K; k += F1) {
        const float2 C = my[k], Dm = my[k == 0 ? 0 : L - k];
        D[k * L + r] = make_float2(0.5f * (C.x + Dm.x), 0.5f * (C.y - Dm.y));
        D[k * L + r + 1] = make_float2(0.5f * (C.y + Dm.y), 0.5f * (Dm.x - C.x));
    }
    wave_lds_sync();  // the next line_fft rewrites the area
}
// rows r, r+1's half spectra in D -> their packed line spectrum over kx in [0, L) (Hermitian
// extension; the self-conjugate bins kx = 0, L/2 keep real parts only, as irfft does)
template <int L>
__device__ __forceinline__ void small_gather(const float2* D, int j, int r, float2 (&v)[Plan<L>::F2]) {
    constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2;
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        const int k = j + F1 * s;
        const bool self = (k == 0) || (2 * k == L);
        float2 be, bo;
        if (2 * k <= L) {
            be = D[k * L + r];
            bo = D[k * L + r + 1];
        } else {
            be = cconj(D[(L - k) * L + r]);
            bo = cconj(D[(L - k) * L + r + 1]);
        }
        if (self) {
            be.y = 0.f;
            bo.y = 0.f;
        }
        v[s] = make_float2(be.x - bo.y, be.y + bo.x);
    }
}

#ifndef GD_SMALL_ZPRE
#define GD_SMALL_ZPRE 1  // k_gal_small: z's row pair loaded before the twiddles (one pair per line)
#endif
// ---------------------------------------------------------------- fused small-image Gaussian iteration
// L <= 128 (LSST stamps are 48^2): a galaxy's whole half spectrum fits in LDS (9.6 KiB at 48^2, 66.5 KiB
// at 128^2), so one 256-thread workgroup per galaxy runs the whole iteration on chip - row FFTs of z,
// column FFTs + the spectral update (gauss_iter_elem, same state layout as k_col<G_ITER*>), inverse
// column FFTs, inverse row FFTs, zin stored - in ONE launch instead of RF -> C -> RI through the
// workspace.  Moves z, the state and zin only (the 2 img + 5.5 half of k_gal_reg).  A line's row
// buffer for the post-FFT split is its own exchange area (F1 (F2 + 1) >= L + 2 for every plan).
template <int L, bool FIRST, bool LAST>
__global__ __launch_bounds__(256) void k_gal_small(Args a) {
    constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2, K = L / 2 + 1, LINES = 256 / F1, XCH = xch_elems<L>();
    static_assert(XCH >= L + 2, "row buffer inside the exchange area");
    constexpr float inv_n = float(1.0 / double(L * L));
    __shared__ float2 tw[L];
    __shared__ float2 S[K * L];  // [kx][ky]
    __shared__ float2 xch[LINES * XCH];
    const int tid = threadIdx.x, line = tid / F1, j = tid - line * F1;
    const int g = blockIdx.x;
    float2* my = xch + line * XCH;
    GD_TRACE(0);
    // z's row pair of this line (one pair per line when L / 2 <= LINES), loaded first so that its latency
    // hides behind the twiddles and the state prefetch
    constexpr bool ZPRE = GD_SMALL_ZPRE && L / 2 <= LINES;
    const float* z = a.a0 + (size_t)g * L * L;
    float2 zv[ZPRE ? F2 : 1];
    if (ZPRE && line < L / 2) {
#pragma unroll
        for (int s = 0; s < (ZPRE ? F2 : 0); ++s)
            zv[s] = make_float2(z[(2 * line) * L + j + F1 * s], z[(2 * line + 1) * L + j + F1 * s]);
    }
    fill_twiddles<L>(tw, tid, 256);
    const float r1 = a.rho1(g), r2 = a.rho2(g), r2n = LAST ? 0.f : a.rho2n(g);
    // the state of this line's first column, loaded now so that its latency hides behind phase R (at
    // 48^2 one workgroup per CU: the launch is a latency chain, not a bandwidth one)
    constexpr bool PRE = L <= 64;  // 96^2 / 128^2 (24 / 16 points per lane): registers are short
    GState pre[PRE ? F2 : 1];
    if (PRE && line < K) {
        const size_t ob = ((size_t)g * K + line) * L + j;
#pragma unroll
        for (int s = 0; s < (PRE ? F2 : 0); ++s) pre[s] = gauss_load<L, FIRST, LAST>(a, ob + F1 * s);
    }
    __syncthreads();
    GD_TRACE(1);

    // R: row pair p -> FFT -> the two rows' half spectra into S (transposed)
    for (int p = line; p < L / 2; p += LINES) {
        float2 v[F2];
        if constexpr (ZPRE) {
#pragma unroll
            for (int s = 0; s < F2; ++s) v[s] = zv[s];
        } else {
#pragma unroll
            for (int s = 0; s < F2; ++s) v[s] = make_float2(z[(2 * p) * L + j + F1 * s], z[(2 * p + 1) * L + j + F1 * s]);
        }
        line_fft<L, false>(v, j, my, tw);
        small_split<L>(v, j, my, S, 2 * p);
    }
    __syncthreads();  // all of z read (zin may alias z), S complete
    GD_TRACE(2);

    // C: column kx -> FFT -> spectral update -> IFFT (back in place)
    for (int kx = line; kx < K; kx += LINES) {
        float2 v[F2];
#pragma unroll
        for (int s = 0; s < F2; ++s) v[s] = S[kx * L + j + F1 * s];
        line_fft<L, false>(v, j, my, tw);
        const size_t ob = ((size_t)g * K + kx) * L + j;
        if (PRE && kx == line) {
#pragma unroll
            for (int s = 0; s < (PRE ? F2 : 0); ++s)
                v[s] = gauss_iter_st<L, FIRST, LAST>(a, ob + F1 * s, v[s], pre[s], r1, r2, r2n, true, inv_n);
        } else {
#pragma unroll
            for (int s = 0; s < F2; ++s)
                v[s] = gauss_iter_elem<L, FIRST, LAST>(a, ob + F1 * s, v[s], r1, r2, r2n, true, inv_n);
        }
        line_fft<L, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < F2; ++s) S[kx * L + j + F1 * s] = v[s];
    }
    __syncthreads();
    GD_TRACE(3);

    // I: Hermitian-extended packed pair spectrum -> inverse row FFT -> zin (x on the last iteration)
    float* out = a.o0 + (size_t)g * L * L;
    for (int p = line; p < L / 2; p += LINES) {
        float2 v[F2];
        small_gather<L>(S, j, 2 * p, v);
        line_fft<L, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            out[(2 * p) * L + j + F1 * s] = v[s].x;
            out[(2 * p + 1) * L + j + F1 * s] = v[s].y;
        }
    }
    GD_TRACE(4);
}

// The 48^2 iteration (k_gal_small_p<48, 8, 6>): one 256-thread workgroup per galaxy on a transposing line plan
// (tline_fft: 8 lanes x 6 points per 48-point line, DFT-6 + DFT-8 per lane instead of the 4 x 12 plan's DFT-12 and
// three DFT-4s), with the row pairs' PACKED spectra in LDS.  The row phase stores each pair's
// transform as it leaves tline_fft (PR[kx][p], kx in [0, L), no split through the exchange area), the column
// line kx reads the packed columns kx and L - kx and separates its rows' bins on the fly (the split's
// arithmetic), and after the inverse column transform it writes the next row phase's packed input for both
// columns kx and L - kx (the gather's Hermitian extension, bins kx = 0, L/2 real) in place - the columns
// {kx, L - kx} belong to that line alone, so no barrier separates its reads and writes.  A lane holds rows
// r = j + TP r' (one parity per lane): the packing pairs lanes j, j ^ 1 through a DPP quad swap.  Per line:
// R 8 LDS stores instead of 8 + 2 syncs + ~16 split accesses, I 8 reads instead of 16 (round 4: bit-identical
// to the retired unpacked form).
template <int L, int TP, int TQ, bool FIRST, bool LAST>
__global__ __launch_bounds__(256) void k_gal_small_p(Args a) {
    constexpr int G = TP > TQ ? TP : TQ, K = L / 2 + 1, LINES = 256 / G, XCH = TP * (TQ + 1) > TQ * (TP + 1)
                                                                               ? TP * (TQ + 1) : TQ * (TP + 1);
    constexpr int SP = L / 2 + 1;  // PR row stride (float2): [kx][p]
    static_assert(TP * TQ == L && G == TP && TP % 2 == 0 && L / 2 <= LINES && K <= LINES, "one line per thread");
    constexpr float inv_n = float(1.0 / double(L * L));
    __shared__ float2 tw[L];
    __shared__ float2 PR[L * SP];
    __shared__ float2 xch[LINES * XCH];
    const int tid = threadIdx.x, line = tid / G, j = tid - line * G;
    const int g = blockIdx.x;
    float2* my = xch + line * XCH;
    GD_TRACE(0);
    const float* z = a.a0 + (size_t)g * L * L;
    float2 v[G];
    if (line < L / 2) {
#pragma unroll
        for (int s = 0; s < TQ; ++s) v[s] = make_float2(z[(2 * line) * L + j + TP * s], z[(2 * line + 1) * L + j + TP * s]);
    }
    fill_twiddles<L>(tw, tid, 256);
    const float r1 = a.rho1(g), r2 = a.rho2(g), r2n = LAST ? 0.f : a.rho2n(g);
    GState pre[TP];
    const bool cl = line < K && j < TQ;
    if (cl) {
        const size_t ob = ((size_t)g * K + line) * L + j;
#pragma unroll
        for (int k1 = 0; k1 < TP; ++k1) pre[k1] = gauss_load<L, FIRST, LAST>(a, ob + TQ * k1);
    }
    __syncthreads();
    GD_TRACE(1);

    // R: row pair p = line -> FFT -> its packed spectrum P_p[kx] (6 x 8 layout: lane j < TQ holds kx = j + TQ k1)
    if (line < L / 2) {
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) PR[(j + TQ * k1) * SP + line] = v[k1];
        }
    }
    __syncthreads();  // all of z read (zin may alias z), PR complete
    GD_TRACE(2);

    // C: column kx = line: lane j holds rows r = j + TP r' (p = r / 2, parity j & 1) of the column, separated
    // from the packed columns kx and L - kx as small_split does
    if (line < K) {
        const int kx = line, km = kx == 0 ? 0 : L - kx;
        const bool odd = j & 1;
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const int p = (j >> 1) + (TP / 2) * s;
            const float2 C = PR[kx * SP + p], Dm = PR[km * SP + p];
            v[s] = odd ? make_float2(0.5f * (C.y + Dm.y), 0.5f * (Dm.x - C.x)) : make_float2(0.5f * (C.x + Dm.x), 0.5f * (C.y - Dm.y));
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        const size_t ob = ((size_t)g * K + kx) * L + (j < TQ ? j : 0);
#pragma unroll
        for (int k1 = 0; k1 < TP; ++k1)
            v[k1] = gauss_iter_st<L, FIRST, LAST>(a, ob + TQ * k1, v[k1], pre[k1], r1, r2, r2n, cl, inv_n);
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
        // lane j: X_r[kx], r = j + TP s.  Pair rows 2p (even lane) and 2p + 1 (odd lane): the even lane writes
        // Q_p[kx] = X_2p + i X_2p+1, the odd lane Q_p[L - kx] = conj(X_2p) + i conj(X_2p+1) (small_gather's
        // arithmetic); the self-conjugate columns kx = 0, L/2 keep real parts only and only the even lane writes
        const bool self = (kx == 0) || (2 * kx == L);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const float ox = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[s].x), 0xB1, 0xF, 0xF, false));
            const float oy = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[s].y), 0xB1, 0xF, 0xF, false));
            const int p = (j >> 1) + (TP / 2) * s;
            float2 be = odd ? make_float2(ox, oy) : v[s], bo = odd ? v[s] : make_float2(ox, oy);
            if (odd) {
                be = cconj(be);
                bo = cconj(bo);
            }
            if (self) {
                be.y = 0.f;
                bo.y = 0.f;
            }
            if (!(odd && self)) PR[(odd ? km : kx) * SP + p] = make_float2(be.x - bo.y, be.y + bo.x);
        }
    }
    __syncthreads();
    GD_TRACE(3);

    // I: row pair p's packed spectrum (6 x 8 layout) -> inverse row FFT -> zin (x on the last iteration)
    float* out = a.o0 + (size_t)g * L * L;
    if (line < L / 2) {
        const int r = 2 * line;
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) v[k1] = PR[(j + TQ * k1) * SP + line];
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            out[r * L + j + TP * s] = v[s].x;
            out[(r + 1) * L + j + TP * s] = v[s].y;
        }
    }
    GD_TRACE(4);
}

// ---------------------------------------------------------------- fused Gaussian iteration at 160^2
// k_gal_small_p's one-pass design for a runtime-planned size whose half spectrum still fits in LDS (80, 112, 144 and
// 160: mid_size, with lines of 16 lanes x L / 16 points; the numbers below are 160^2's): at 160^2 the
// packed row spectra PR[kx][p] take 160 x 81 complex = 101 KiB, the 32 lines' exchange areas 44 KiB, so one
// 512-thread workgroup per galaxy runs rows -> columns + update -> inverse rows on chip (the runtime-planned
// three-kernel chain moves ~19 words per pixel through the workspace; this moves 2 img + 5.5 half = 7.5).  Lines
// are 16 lanes x 10 points (tline_fft<160, 16, 10>: DFT-10 = 2 x 5, then DFT-16 across the lanes; the inverse
// back), looped over the 80 row pairs / 81 columns.  The state layout is the generic path's [N][K][L] (what
// its init writes), the per-bin arithmetic gauss_iter_elem's, so this is a drop-in for the C_G_ITER* chain.
#ifndef GD_MID_PF
#define GD_MID_PF 1  // k_gal_mid: the next row pair's z and each column's state loaded ahead of the transforms
#endif
#ifndef GD_MID_FUSED
#define GD_MID_FUSED 1  // 1: Gaussian iterations (and init) at the mid_size sizes in one launch (k_gal_mid); 0: the runtime-planned chains
#endif
template <int L, int TP, int TQ, int NT, bool FIRST, bool LAST>
__global__ __launch_bounds__(NT) void k_gal_mid(Args a) {
    constexpr int G = TP, K = L / 2 + 1, LINES = NT / G, SP = L / 2 + 1;
    constexpr int XCH = TP * (TQ + 1) > TQ * (TP + 1) ? TP * (TQ + 1) : TQ * (TP + 1);
    static_assert(TP * TQ == L && TP >= TQ && TP % 2 == 0 && NT % G == 0, "lines of TP lanes, rows paired per lane");
    constexpr float inv_n = float(1.0 / double(L * L));
    __shared__ float2 tw[L];
    __shared__ float2 PR[L * SP];
    __shared__ float2 xch[LINES * XCH];
    const int tid = threadIdx.x, line = tid / G, j = tid - line * G;
    const int g = blockIdx.x;
    float2* my = xch + line * XCH;
    fill_twiddles<L>(tw, tid, NT);
    const float r1 = a.rho1(g), r2 = a.rho2(g), r2n = LAST ? 0.f : a.rho2n(g);
    __syncthreads();
    const float* z = a.a0 + (size_t)g * L * L;
    float2 v[G];

    // R: row pair p -> FFT -> packed spectrum PR[kx][p] (lane j < TQ holds kx = j + TQ k1).  GD_MID_PF: the next
    // pair's z is loaded while this pair transforms (at 144 / 160^2 one galaxy per CU: nothing else hides a round's
    // load latency; at 80 / 112^2 it costs a workgroup per CU and still wins, r04midnt_ab.txt)
    constexpr bool PF = GD_MID_PF != 0;
    float2 nz[TQ];
    if (PF && line < L / 2) {
#pragma unroll
        for (int s = 0; s < TQ; ++s) nz[s] = make_float2(z[(2 * line) * L + j + TP * s], z[(2 * line + 1) * L + j + TP * s]);
    }
    for (int p = line; p < L / 2; p += LINES) {
        if constexpr (PF) {
#pragma unroll
            for (int s = 0; s < TQ; ++s) v[s] = nz[s];
            const int pn = p + LINES;
            if (pn < L / 2) {
#pragma unroll
                for (int s = 0; s < TQ; ++s) nz[s] = make_float2(z[(2 * pn) * L + j + TP * s], z[(2 * pn + 1) * L + j + TP * s]);
            }
        } else {
#pragma unroll
            for (int s = 0; s < TQ; ++s) v[s] = make_float2(z[(2 * p) * L + j + TP * s], z[(2 * p + 1) * L + j + TP * s]);
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) PR[(j + TQ * k1) * SP + p] = v[k1];
        }
    }
    __syncthreads();  // all of z read (zin may alias z), PR complete

    // C: column kx (lane j: rows r = j + TP r', separated from the packed columns kx and L - kx), FFT, update,
    // IFFT, then the next row phase's packed input for both columns written in place (k_gal_small_p's scheme)
    const bool odd = j & 1;
    for (int kx = line; kx < K; kx += LINES) {
        const int km = kx == 0 ? 0 : L - kx;
        const bool cl = j < TQ;
        const size_t ob = ((size_t)g * K + kx) * L + (cl ? j : 0);
        GState pre[TP];  // (PF) this column's state, in flight during its forward transform
        if constexpr (PF) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) pre[k1] = gauss_load<L, FIRST, LAST>(a, ob + TQ * k1);
        }
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const int p = (j >> 1) + (TP / 2) * s;
            const float2 C = PR[kx * SP + p], Dm = PR[km * SP + p];
            v[s] = odd ? make_float2(0.5f * (C.y + Dm.y), 0.5f * (Dm.x - C.x)) : make_float2(0.5f * (C.x + Dm.x), 0.5f * (C.y - Dm.y));
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
#pragma unroll
        for (int k1 = 0; k1 < TP; ++k1) {
            if constexpr (PF) v[k1] = gauss_iter_st<L, FIRST, LAST>(a, ob + TQ * k1, v[k1], pre[k1], r1, r2, r2n, cl, inv_n);
            else v[k1] = gauss_iter_elem<L, FIRST, LAST>(a, ob + TQ * k1, v[k1], r1, r2, r2n, cl, inv_n);
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
        const bool self = (kx == 0) || (2 * kx == L);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const float ox = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[s].x), 0xB1, 0xF, 0xF, false));
            const float oy = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[s].y), 0xB1, 0xF, 0xF, false));
            const int p = (j >> 1) + (TP / 2) * s;
            float2 be = odd ? make_float2(ox, oy) : v[s], bo = odd ? v[s] : make_float2(ox, oy);
            if (odd) {
                be = cconj(be);
                bo = cconj(bo);
            }
            if (self) {
                be.y = 0.f;
                bo.y = 0.f;
            }
            if (!(odd && self)) PR[(odd ? km : kx) * SP + p] = make_float2(be.x - bo.y, be.y + bo.x);
        }
    }
    __syncthreads();

    // I: row pair p's packed spectrum -> inverse row FFT -> zin (x on the last iteration)
    float* out = a.o0 + (size_t)g * L * L;
    for (int p = line; p < L / 2; p += LINES) {
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) v[k1] = PR[(j + TQ * k1) * SP + p];
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            out[(2 * p) * L + j + TP * s] = v[s].x;
            out[(2 * p + 1) * L + j + TP * s] = v[s].y;
        }
    }
}
// ---------------------------------------------------------------- fused Poisson iteration, L <= 112
// The reference's default llh (models/Unrolled_ADMM.py:154): the V step's sqrt keeps u1 and w = v - u2 in the
// image domain, so an iteration transforms TWO images (z - u1 and w) and inverts two spectra (X and H X).  At
// L <= 112 both images' packed row spectra fit in LDS (2 L (L/2 + 1) complex: 100 KiB at 112^2), so the
// three-kernel chain RF_ITER -> C_ITER -> RI_ITER (two workspace round trips per iteration) becomes one
// workgroup per galaxy, on k_gal_mid's layout and lines (TP lanes x TQ points):
//   R  row pairs of z - u1 (image 0) and of w (image 1) -> FFT -> packed spectra PR[im][kx][p]
//   C  per column kx: both images' columns (separated from the packed columns kx, L - kx), FFT; C_ITER's
//      X = (rho1 F(z - u1) + rho2 conj(H) F(w)) / (rho1 |H|^2 + rho2) and H X (IEEE divisions, as the chain);
//      IFFT both; the packed inputs of the inverse rows written in place
//   I  row pairs: IFFT -> x, H x -> RI_ITER's pointwise update (u1, w, zin; x alpha on the last iteration)
// State: the OTF [N][K][L] (C_OTF_INIT's, not re-read by the row phases), u1, w (images); reads z, u1, w, y, the
// OTF; writes u1, w, zin: 6 img + 1 half per galaxy against 10 img + 7 half for the chain.
// FIRST (state layout 4, after a SPLIT init): the w slot holds H x0; the row phase forms w1 = V(H x0 + 0, y, rho2,
// alpha) there (RI_INIT's arithmetic with this iteration's rho2, the init's rho2_iters[0]) and stores it back
#ifndef GD_POIS_PF
#define GD_POIS_PF 1  // k_pois_small: the next row job's inputs loaded ahead of its transform (64^2: 0.188 -> 0.173 ms)
#endif
template <int L, int TP, int TQ, int NT, bool LAST, bool FIRST = false>
__global__ __launch_bounds__(NT) void k_pois_small(Args a) {
    constexpr int G = TP, K = L / 2 + 1, LINES = NT / G, SP = L / 2 + 1, IMS = L * SP;
    constexpr int XCH = TP * (TQ + 1) > TQ * (TP + 1) ? TP * (TQ + 1) : TQ * (TP + 1);
    static_assert(TP * TQ == L && TP >= TQ && TP % 2 == 0 && NT % G == 0 && 64 % TP == 0, "lines of TP lanes in one wave");
    constexpr float inv_n = float(1.0 / double(L * L));
    __shared__ float2 tw[L];
    __shared__ float2 PR[2 * IMS];
    __shared__ float2 xch[LINES * XCH];
    const int tid = threadIdx.x, line = tid / G, j = tid - line * G;
    const int g = blockIdx.x;
    float2* my = xch + line * XCH;
    fill_twiddles<L>(tw, tid, NT);
    const float r1 = a.rho1(g), r2 = a.rho2(g), al = a.alpha(g), r2n = LAST ? 1.f : a.rho2n(g);
    const size_t gi = (size_t)g * L * L;
    const float* z = a.a0 + gi;
    const float* u1 = a.a1 + gi;
    const float* wv = a.a2 + gi;
    __syncthreads();
    float2 v[G], q[G];

    // R: job t < L/2: pair t of z - u1; job t >= L/2: pair t - L/2 of w.  PF: the next job's inputs are in flight
    // during this job's transform
    constexpr bool PF = GD_POIS_PF != 0;
    auto rload = [&](float4 (&b)[TQ], int t) {
        const int im = t >= L / 2, p = t - im * (L / 2), o0 = (2 * p) * L + j, o1 = o0 + L;
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            if (im) b[s] = make_float4(wv[o0 + TP * s], wv[o1 + TP * s], FIRST ? a.y[gi + o0 + TP * s] : 0.f,
                                       FIRST ? a.y[gi + o1 + TP * s] : 0.f);
            else b[s] = make_float4(z[o0 + TP * s], z[o1 + TP * s], u1[o0 + TP * s], u1[o1 + TP * s]);
        }
    };
    float4 pf[TQ];
    if (PF && line < L) rload(pf, line);
    for (int t = line; t < L; t += LINES) {
        const int im = t >= L / 2, p = t - im * (L / 2), o0 = (2 * p) * L + j, o1 = o0 + L;
        float4 cur[TQ];
        if constexpr (PF) {
#pragma unroll
            for (int s = 0; s < TQ; ++s) cur[s] = pf[s];
            if (t + LINES < L) rload(pf, t + LINES);
        } else {
            rload(cur, t);
        }
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            if (FIRST && im) {  // w1 from H x0 (the SPLIT init), stored for the update phase
                const size_t p0 = gi + o0 + TP * s, p1 = gi + o1 + TP * s;
                const float w0 = v_step(GD_LLH_POISSON, cur[s].x + 0.0f, fmaxf(cur[s].z, 0.f), r2, al);
                const float w1 = v_step(GD_LLH_POISSON, cur[s].y + 0.0f, fmaxf(cur[s].w, 0.f), r2, al);
                a.o1[p0] = w0;
                a.o1[p1] = w1;
                v[s] = make_float2(w0, w1);
            } else {
                v[s] = im ? make_float2(cur[s].x, cur[s].y) : make_float2(cur[s].x - cur[s].z, cur[s].y - cur[s].w);
            }
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) PR[im * IMS + (j + TQ * k1) * SP + p] = v[k1];
        }
    }
    __syncthreads();

    // C
    const bool odd = j & 1, cl = j < TQ;
    for (int kx = line; kx < K; kx += LINES) {
        const int km = kx == 0 ? 0 : L - kx;
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const int p = (j >> 1) + (TP / 2) * s;
            const float2 C = PR[kx * SP + p], Dm = PR[km * SP + p];
            const float2 E = PR[IMS + kx * SP + p], Fm = PR[IMS + km * SP + p];
            v[s] = odd ? make_float2(0.5f * (C.y + Dm.y), 0.5f * (Dm.x - C.x)) : make_float2(0.5f * (C.x + Dm.x), 0.5f * (C.y - Dm.y));
            q[s] = odd ? make_float2(0.5f * (E.y + Fm.y), 0.5f * (Fm.x - E.x)) : make_float2(0.5f * (E.x + Fm.x), 0.5f * (E.y - Fm.y));
        }
        const size_t ob = ((size_t)g * K + kx) * L + (cl ? j : 0);
        float2 hk[TP];  // this column's OTF, in flight during the forward transforms
#pragma unroll
        for (int k1 = 0; k1 < TP; ++k1) hk[k1] = a.otf[ob + TQ * k1];
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        tline_fft<L, TP, TQ, false>(q, j, my, tw);
#pragma unroll
        for (int k1 = 0; k1 < TP; ++k1) {
            const float2 Hk = hk[k1];
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;  // C_ITER's arithmetic
            const float lhs = r1 * HtH + r2;
            const float2 HtW = cmulc(q[k1], Hk);
            const float2 rhs = make_float2(r1 * v[k1].x + r2 * HtW.x, r1 * v[k1].y + r2 * HtW.y);
            const float2 X = make_float2(rhs.x / lhs, rhs.y / lhs);
            v[k1] = cscale(X, inv_n);
            q[k1] = cscale(cmul(Hk, X), inv_n);
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
        tline_fft<L, TQ, TP, true>(q, j, my, tw);
        const bool self = (kx == 0) || (2 * kx == L);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {  // both images' packed inverse-row inputs (k_gal_mid's write-back)
            const int p = (j >> 1) + (TP / 2) * s;
#pragma unroll
            for (int im = 0; im < 2; ++im) {
                const float2 c = im ? q[s] : v[s];
                const float ox = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(c.x), 0xB1, 0xF, 0xF, false));
                const float oy = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(c.y), 0xB1, 0xF, 0xF, false));
                float2 be = odd ? make_float2(ox, oy) : c, bo = odd ? c : make_float2(ox, oy);
                if (odd) {
                    be = cconj(be);
                    bo = cconj(bo);
                }
                if (self) {
                    be.y = 0.f;
                    bo.y = 0.f;
                }
                if (!(odd && self)) PR[im * IMS + (odd ? km : kx) * SP + p] = make_float2(be.x - bo.y, be.y + bo.x);
            }
        }
    }
    __syncthreads();

    // I: x (image 0), H x (image 1) -> RI_ITER (models/Unrolled_ADMM.py:207-215)
    for (int p = line; p < L / 2; p += LINES) {
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) {
                v[k1] = PR[(j + TQ * k1) * SP + p];
                q[k1] = PR[IMS + (j + TQ * k1) * SP + p];
            }
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
        tline_fft<L, TQ, TP, true>(q, j, my, tw);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const size_t pix = gi + (size_t)(2 * p + h) * L + j + TP * s;
                const float x = h ? v[s].y : v[s].x, hx = h ? q[s].y : q[s].x;
                if (LAST) {
                    a.o2[pix] = x * al;  // Poisson: x_list[-1] * alpha (:215)
                } else {
                    const float un = (a.a1[pix] + x) - a.a0[pix];        // u1 + x - z
                    const float u2 = hx - a.a2[pix];                     // u2 + conv(H, x) - v  (w = v - u2)
                    const float vn = v_step(GD_LLH_POISSON, hx + u2, fmaxf(a.y[pix], 0.f), r2n, al);
                    a.o0[pix] = un;
                    a.o1[pix] = vn - u2;
                    a.o2[pix] = x + un;                                  // next denoiser input
                }
            }
        }
    }
}

// The Poisson init at L <= 112 in one launch (k_pois_small_init): init_l2 (models/Unrolled_ADMM.py:170-175) and
// the first V step (:207) on k_pois_small's layout - the chain RF_PSF_Y -> C_OTF_INIT -> RIF_CLAMP -> C_CONV ->
// RI_INIT, bin for bin and pixel for pixel:
//   R  row pairs of the placed PSF (psf_to_otf's circular placement) and of max(y, 0) / alpha -> PR[0], PR[1]
//   C  per column: both FFT'd; the OTF -> state; X0 = conj(H) Y / (|H|^2 + 1/alpha) / L^2; IFFT -> PR[1]
//   I  x0 = clamp(IFFT, 0, 1) -> zin; FFT -> PR[1]
//   C  per column: F(x0) H / L^2 (the OTF column read back); IFFT -> PR[1]
//   I  H x0 -> w1 = V(H x0 + 0, y, rho2, alpha) (u2 = 0: w = v), u1 = 0
// SPLIT (the state layout gd_admm_state_layout 4): the last step stores H x0 itself in the w slot and reads no
// rho; iteration 0 (k_pois_small<FIRST>) forms w1 from it with its own rho2 (= the init's rho2_iters[0]), so the
// init runs beside the SubNet (k_subnet_rhos_init) like the Gaussian one.  Same w1 bits either way.
template <int L, int TP, int TQ, int NT>
struct PoisInitLds {
    static constexpr int SP = L / 2 + 1, IMS = L * SP, LINES = NT / TP;
    static constexpr int XCH = TP * (TQ + 1) > TQ * (TP + 1) ? TP * (TQ + 1) : TQ * (TP + 1);
    static constexpr int TW = 0, PR = L, XC = PR + 2 * IMS, SIZE = XC + LINES * XCH;  // float2 units
};
template <int L, int TP, int TQ, int NT, bool SPLIT>
__device__ __forceinline__ void pois_small_init_body(const Args& a, int g, int tid, float2* lds) {
    constexpr int G = TP, K = L / 2 + 1, LINES = NT / G, SP = L / 2 + 1, IMS = L * SP;
    using LY = PoisInitLds<L, TP, TQ, NT>;
    constexpr int XCH = LY::XCH;
    static_assert(TP * TQ == L && TP >= TQ && TP % 2 == 0 && NT % G == 0 && 64 % TP == 0, "lines of TP lanes in one wave");
    constexpr float inv_n = float(1.0 / double(L * L));
    float2* tw = lds + LY::TW;
    float2* PR = lds + LY::PR;
    float2* xch = lds + LY::XC;
    const int line = tid / G, j = tid - line * G;
    float2* my = xch + line * XCH;
    fill_twiddles<L>(tw, tid, NT);
    const float al = a.alpha(g), r2 = SPLIT ? 1.f : a.rho2n(g);
    const int h = a.h, h2 = h >> 1;
    const float* psf = a.psf + (long long)g * a.psf_gstride;
    const size_t gi = (size_t)g * L * L;
    const float* y = a.y + gi;
    __syncthreads();
    float2 v[G], q[G];
    const bool odd = j & 1, cl = j < TQ;
    // the packed row-pair spectra of image im -> column kx's bins (lane j: rows j + TP s)
    auto separate = [&](float2 (&c)[G], int im, int kx, int km) {
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const int p = (j >> 1) + (TP / 2) * s;
            const float2 C = PR[im * IMS + kx * SP + p], Dm = PR[im * IMS + km * SP + p];
            c[s] = odd ? make_float2(0.5f * (C.y + Dm.y), 0.5f * (Dm.x - C.x)) : make_float2(0.5f * (C.x + Dm.x), 0.5f * (C.y - Dm.y));
        }
    };
    // column results (transposed back) -> the packed inputs of the inverse rows of image im, in place
    auto pack_back = [&](const float2 (&c)[G], int im, int kx, int km) {
        const bool self = (kx == 0) || (2 * kx == L);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const int p = (j >> 1) + (TP / 2) * s;
            const float ox = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(c[s].x), 0xB1, 0xF, 0xF, false));
            const float oy = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(c[s].y), 0xB1, 0xF, 0xF, false));
            float2 be = odd ? make_float2(ox, oy) : c[s], bo = odd ? c[s] : make_float2(ox, oy);
            if (odd) {
                be = cconj(be);
                bo = cconj(bo);
            }
            if (self) {
                be.y = 0.f;
                bo.y = 0.f;
            }
            if (!(odd && self)) PR[im * IMS + (odd ? km : kx) * SP + p] = make_float2(be.x - bo.y, be.y + bo.x);
        }
    };
    // R: job t < L/2: padded PSF row pair t; t >= L/2: row pair t - L/2 of max(y, 0) / alpha (RF_PSF_Y)
    for (int t = line; t < L; t += LINES) {
        const int im = t >= L / 2, p = t - im * (L / 2);
        if (im) {
#pragma unroll
            for (int s = 0; s < TQ; ++s) {
                const int o = (2 * p) * L + j + TP * s;
                v[s] = make_float2(fmaxf(y[o], 0.f) / al, fmaxf(y[o + L], 0.f) / al);
            }
        } else {
            int i0 = 2 * p + h2, i1 = i0 + 1;  // padded rows 2p, 2p + 1 -> PSF rows (r + h/2) mod L (gpsf)
            if (i0 >= L) i0 -= L;
            if (i1 >= L) i1 -= L;
#pragma unroll
            for (int s = 0; s < TQ; ++s) {
                int jj = j + TP * s + h2;
                if (jj >= L) jj -= L;
                const bool in = jj < h;
                v[s] = make_float2((in && i0 < h) ? psf[i0 * h + jj] : 0.f, (in && i1 < h) ? psf[i1 * h + jj] : 0.f);
            }
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) PR[im * IMS + (j + TQ * k1) * SP + p] = v[k1];
        }
    }
    __syncthreads();
    // C: the OTF and X0 (C_OTF_INIT)
    for (int kx = line; kx < K; kx += LINES) {
        const int km = kx == 0 ? 0 : L - kx;
        separate(v, 0, kx, km);
        separate(q, 1, kx, km);
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        tline_fft<L, TP, TQ, false>(q, j, my, tw);
        const size_t ob = ((size_t)g * K + kx) * L + (cl ? j : 0);
#pragma unroll
        for (int k1 = 0; k1 < TP; ++k1) {
            const float2 Hk = v[k1];
            if (cl) a.otf[ob + TQ * k1] = Hk;
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float lhs = HtH + 1.0f / al;
            const float2 rhs = cmulc(q[k1], Hk);
            q[k1] = cscale(make_float2(rhs.x / lhs, rhs.y / lhs), inv_n);
        }
        tline_fft<L, TQ, TP, true>(q, j, my, tw);
        pack_back(q, 1, kx, km);
    }
    __syncthreads();
    // I: x0 = clamp -> zin (RIF_CLAMP); FFT of x0's rows
    float* zin = a.o2 + gi;
    for (int p = line; p < L / 2; p += LINES) {
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) v[k1] = PR[IMS + (j + TQ * k1) * SP + p];
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            v[s] = make_float2(fminf(fmaxf(v[s].x, 0.f), 1.f), fminf(fmaxf(v[s].y, 0.f), 1.f));
            zin[(2 * p) * L + j + TP * s] = v[s].x;
            zin[(2 * p + 1) * L + j + TP * s] = v[s].y;
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) PR[IMS + (j + TQ * k1) * SP + p] = v[k1];
        }
    }
    __syncthreads();
    // C: conv(H, x0) (C_CONV)
    for (int kx = line; kx < K; kx += LINES) {
        const int km = kx == 0 ? 0 : L - kx;
        separate(v, 1, kx, km);
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        const size_t ob = ((size_t)g * K + kx) * L + (cl ? j : 0);
#pragma unroll
        for (int k1 = 0; k1 < TP; ++k1) v[k1] = cscale(cmul(v[k1], a.otf[ob + TQ * k1]), inv_n);
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
        pack_back(v, 1, kx, km);
    }
    __syncthreads();
    // I: w1 = V(H x0 + 0, y, rho2, alpha), u1 = 0 (RI_INIT)
    for (int p = line; p < L / 2; p += LINES) {
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) v[k1] = PR[IMS + (j + TQ * k1) * SP + p];
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const size_t pix = gi + (size_t)(2 * p + hh) * L + j + TP * s;
                const float hx = hh ? v[s].y : v[s].x;
                a.o1[pix] = SPLIT ? hx : v_step(GD_LLH_POISSON, hx + 0.0f, fmaxf(a.y[pix], 0.f), r2, al);
                a.o0[pix] = 0.f;
            }
        }
    }
}
template <int L, int TP, int TQ, int NT, bool SPLIT>
__global__ __launch_bounds__(NT) void k_pois_small_init(Args a) {
    __shared__ __attribute__((aligned(16))) float2 lds[PoisInitLds<L, TP, TQ, NT>::SIZE];
    pois_small_init_body<L, TP, TQ, NT, SPLIT>(a, blockIdx.x, threadIdx.x, lds);
}
// k_pois_small's line plans (TP lanes x TQ points, threads).  Not at 128^2: there both images fill 152 KiB of LDS,
// one 256-thread workgroup per CU, and the chain's kernels were faster (4096 galaxies: 1.33 vs 0.95 ms per
// iteration; profiles/r04pois_*); at 64^2 / 96^2 / 112^2 the fused form takes 0.82 / 0.95 / 0.46 of the chain's time
template <int L>
struct PoisSmallPlan;
template <> struct PoisSmallPlan<32> { static constexpr int TP = 8, TQ = 4, NT = 256; };
#ifndef GD_POIS48_NT
#define GD_POIS48_NT 512  // measured: 512 threads 2.21 M vs 2.155 M gal/s graphed (256 x 48^2, profiles/r04p48ab.txt)
#endif
template <> struct PoisSmallPlan<48> { static constexpr int TP = 8, TQ = 6, NT = GD_POIS48_NT; };
template <> struct PoisSmallPlan<64> { static constexpr int TP = 8, TQ = 8, NT = 256; };
template <> struct PoisSmallPlan<80> { static constexpr int TP = 16, TQ = 5, NT = 256; };
template <> struct PoisSmallPlan<96> { static constexpr int TP = 16, TQ = 6, NT = 512; };
template <> struct PoisSmallPlan<112> { static constexpr int TP = 16, TQ = 7, NT = 512; };

// ---------------------------------------------------------------- fused Gaussian init at 160^2
// init_l2 (models/Unrolled_ADMM.py:170-175), the Gaussian constants and F(x0) in one launch, one 512-thread
// workgroup per galaxy on k_gal_mid's layout: the runtime-planned chain RF_PSF_Y -> C_G_INIT -> RIF_CLAMP ->
// C_G_W1 (four launches through the chunked workspace), bin for bin:
//   P  the placed PSF's row pairs (psf_to_otf's circular placement, gpsf) -> FFT -> packed spectra, parked
//      in the galaxy's U1 slot as [kx][pair] (the slot is not read before iteration 0 writes it)
//   R  max(y, 0) / alpha row pairs -> FFT -> PR
//   C  per column kx: the OTF column (rows separated from the parked spectra, FFT) and Y's (from PR);
//      |H|^2, G = conj(H) Y -> state; X0 = G / (|H|^2 + 1/alpha) / L^2; IFFT -> PR (packed, in place)
//   I  row pairs: IFFT -> x0 = clamp(., 0, 1) -> zin; FFT -> PR
//   W  per column: FFT -> F(x0) -> the W~ slot (iteration 0 forms W~1 from it, w1_value)
template <int L, int TP, int TQ, int NT>
__global__ __launch_bounds__(NT) void k_gal_mid_init(Args a) {
    constexpr int G = TP, K = L / 2 + 1, LINES = NT / G, SP = L / 2 + 1;
    constexpr int XCH = TP * (TQ + 1) > TQ * (TP + 1) ? TP * (TQ + 1) : TQ * (TP + 1);
    static_assert(TP * TQ == L && TP >= TQ && TP % 2 == 0 && NT % G == 0, "lines of TP lanes, rows paired per lane");
    constexpr float inv_n = float(1.0 / double(L * L));
    __shared__ float2 tw[L];
    __shared__ float2 PR[L * SP];
    __shared__ float2 xch[LINES * XCH];
    const int tid = threadIdx.x, line = tid / G, j = tid - line * G;
    const int g = blockIdx.x;
    float2* my = xch + line * XCH;
    fill_twiddles<L>(tw, tid, NT);
    const int h = a.h, h2 = h >> 1, npp = (h + 1) >> 1;
    const float al = a.alpha(g);
    const float ial = 1.0f / al;  // the chain's lhs = |H|^2 + 1.0f / alpha
    const float* psf = a.psf + (long long)g * a.psf_gstride;
    float2* pc = a.s_u1 + (size_t)g * K * L;  // parked PSF spectra [kx][pair], L npp <= K L
    __syncthreads();
    float2 v[G];

    // P: PSF rows 2p, 2p + 1 placed on the L-point circle (column c holds PSF column (c + h/2) mod L when < h)
    for (int p = line; p < npp; p += LINES) {
        const int i0 = 2 * p, i1 = i0 + 1;
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            int jj = j + TP * s + h2;
            if (jj >= L) jj -= L;
            const bool in = jj < h;
            v[s] = make_float2(in ? psf[i0 * h + jj] : 0.f, (in && i1 < h) ? psf[i1 * h + jj] : 0.f);
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) pc[(j + TQ * k1) * npp + p] = v[k1];
        }
    }
    // R: max(y, 0) / alpha (RF_PSF_Y's slot 1)
    const float* y = a.y + (size_t)g * L * L;
    for (int p = line; p < L / 2; p += LINES) {
#pragma unroll
        for (int s = 0; s < TQ; ++s)
            v[s] = make_float2(fmaxf(y[(2 * p) * L + j + TP * s], 0.f) / al, fmaxf(y[(2 * p + 1) * L + j + TP * s], 0.f) / al);
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) PR[(j + TQ * k1) * SP + p] = v[k1];
        }
    }
    __syncthreads();  // PR complete, the parked PSF spectra visible to the workgroup

    const bool odd = j & 1, cl = j < TQ;
    // C: column kx; lane j holds rows r = j + TP s (pair (j >> 1) + (TP / 2) s, parity j & 1)
    for (int kx = line; kx < K; kx += LINES) {
        const int km = kx == 0 ? 0 : L - kx;
        float2 hv[G];
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const int p = (j >> 1) + (TP / 2) * s;
            const float2 C = PR[kx * SP + p], Dm = PR[km * SP + p];
            v[s] = odd ? make_float2(0.5f * (C.y + Dm.y), 0.5f * (Dm.x - C.x)) : make_float2(0.5f * (C.x + Dm.x), 0.5f * (C.y - Dm.y));
            int i = j + TP * s + h2;  // padded row r -> PSF row (r + h/2) mod L (gpsf)
            if (i >= L) i -= L;
            float2 hval = make_float2(0.f, 0.f);
            if (i < h) {
                const float2 Cp = pc[kx * npp + (i >> 1)], Dp = pc[km * npp + (i >> 1)];
                hval = (i & 1) ? make_float2(0.5f * (Cp.y + Dp.y), 0.5f * (Dp.x - Cp.x))
                               : make_float2(0.5f * (Cp.x + Dp.x), 0.5f * (Cp.y - Dp.y));
            }
            hv[s] = hval;
        }
#pragma unroll
        for (int s = TQ; s < G; ++s) hv[s] = make_float2(0.f, 0.f);
        tline_fft<L, TP, TQ, false>(hv, j, my, tw);
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        const size_t ob = ((size_t)g * K + kx) * L + (cl ? j : 0);
#pragma unroll
        for (int k1 = 0; k1 < TP; ++k1) {
            const float2 Hk = hv[k1], Yk = v[k1];
            const float hh = Hk.x * Hk.x + Hk.y * Hk.y;  // C_G_INIT's arithmetic
            const float2 Gk = cmulc(Yk, Hk);
            if (cl) {
                a.s_hh[ob + TQ * k1] = hh;
                a.s_g[ob + TQ * k1] = Gk;
            }
            const float lhs = hh + ial;
            v[k1] = cscale(make_float2(Gk.x / lhs, Gk.y / lhs), inv_n);
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
        const bool self = (kx == 0) || (2 * kx == L);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {  // the next row phase's packed input (k_gal_mid)
            const float ox = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[s].x), 0xB1, 0xF, 0xF, false));
            const float oy = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[s].y), 0xB1, 0xF, 0xF, false));
            const int p = (j >> 1) + (TP / 2) * s;
            float2 be = odd ? make_float2(ox, oy) : v[s], bo = odd ? v[s] : make_float2(ox, oy);
            if (odd) {
                be = cconj(be);
                bo = cconj(bo);
            }
            if (self) {
                be.y = 0.f;
                bo.y = 0.f;
            }
            if (!(odd && self)) PR[(odd ? km : kx) * SP + p] = make_float2(be.x - bo.y, be.y + bo.x);
        }
    }
    __syncthreads();

    // I: IFFT -> x0 = clamp(x0, 0, 1) -> zin (RIF_CLAMP); FFT of the clamped rows -> PR
    float* out = a.o2 + (size_t)g * L * L;
    for (int p = line; p < L / 2; p += LINES) {
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) v[k1] = PR[(j + TQ * k1) * SP + p];
        }
        tline_fft<L, TQ, TP, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            v[s] = make_float2(fminf(fmaxf(v[s].x, 0.f), 1.f), fminf(fmaxf(v[s].y, 0.f), 1.f));
            out[(2 * p) * L + j + TP * s] = v[s].x;
            out[(2 * p + 1) * L + j + TP * s] = v[s].y;
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (j < TQ) {
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) PR[(j + TQ * k1) * SP + p] = v[k1];
        }
    }
    __syncthreads();

    // W: F(x0)'s columns -> the W~ slot (C_G_W1)
    for (int kx = line; kx < K; kx += LINES) {
        const int km = kx == 0 ? 0 : L - kx;
#pragma unroll
        for (int s = 0; s < TQ; ++s) {
            const int p = (j >> 1) + (TP / 2) * s;
            const float2 C = PR[kx * SP + p], Dm = PR[km * SP + p];
            v[s] = odd ? make_float2(0.5f * (C.y + Dm.y), 0.5f * (Dm.x - C.x)) : make_float2(0.5f * (C.x + Dm.x), 0.5f * (C.y - Dm.y));
        }
        tline_fft<L, TP, TQ, false>(v, j, my, tw);
        if (cl) {
            const size_t ob = ((size_t)g * K + kx) * L + j;
#pragma unroll
            for (int k1 = 0; k1 < TP; ++k1) a.s_w[ob + TQ * k1] = v[k1];
        }
    }
}
// ---------------------------------------------------------------- fused small-image Gaussian init
// L <= 96: init_l2 (models/Unrolled_ADMM.py:170-175), the Gaussian constants |H|^2 and
// G = conj(H) F(max(y,0)/alpha), and F(x0) into the W~ slot (iteration 0 forms W~1 from it, see w1_value)
// in one workgroup per galaxy.  The observation's and the placed PSF's half spectra both fit in LDS
// (2 x 37.6 KiB at 96^2), so y -> |H|^2, G, X0 -> x0 = clamp(., 0, 1) = zin -> F(x0) is one launch instead of
// RF_YA -> psf_rows -> G_INIT -> RIF_CLAMP -> G_W1 through the workspace; same arithmetic as that chain.
// LDS of the body on NT threads (float2 units): twiddles | S [kx][ky] (row spectra of max(y,0)/alpha ->
// X0 -> row spectra of x0) | SH [kx][ky] (row spectra of the placed PSF) | the lines' exchange areas
template <int L, int NT>
struct SmallInitLds {
    static constexpr int K = L / 2 + 1, LINES = NT / Plan<L>::F1;
    static constexpr int TW = 0, S = L, SH = S + K * L, XCH = SH + K * L, SIZE = XCH + LINES * xch_elems<L>();
};
template <int L, int NT>
__device__ __forceinline__ void gal_small_init_body(const Args& a, int g, int tid, float2* lds) {
    using LY = SmallInitLds<L, NT>;
    constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2, K = L / 2 + 1, LINES = LY::LINES, XCH = xch_elems<L>();
    constexpr float inv_n = float(1.0 / double(L * L));
    float2* tw = lds + LY::TW;
    float2* S = lds + LY::S;
    float2* SH = lds + LY::SH;
    float2* xch = lds + LY::XCH;
    const int line = tid / F1, j = tid - line * F1;
    float2* my = xch + line * XCH;
    fill_twiddles<L>(tw, tid, NT);
    const float al = a.alpha(g);
    __syncthreads();

    // R: pairs q < L/2 of max(y,0)/alpha, pairs q >= L/2 of the placed PSF -> row half spectra
    const float* y = a.y + (size_t)g * L * L;
    for (int q = line; q < L; q += LINES) {
        const bool isp = q >= L / 2;
        const int p = isp ? q - L / 2 : q;
        float2 v[F2];
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            const int c = j + F1 * s;
            v[s] = isp ? make_float2(shifted_psf(a, g, 2 * p, c, L), shifted_psf(a, g, 2 * p + 1, c, L))
                       : make_float2(fmaxf(y[(2 * p) * L + c], 0.f) / al, fmaxf(y[(2 * p + 1) * L + c], 0.f) / al);
        }
        line_fft<L, false>(v, j, my, tw);
        small_split<L>(v, j, my, isp ? SH : S, 2 * p);
    }
    __syncthreads();

    // C1: columns of Y and H -> |H|^2, G (state); X0 = G / (|H|^2 + 1/alpha) -> inverse column FFT
    for (int kx = line; kx < K; kx += LINES) {
        float2 v[F2], hc[F2];
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            v[s] = S[kx * L + j + F1 * s];
            hc[s] = SH[kx * L + j + F1 * s];
        }
        line_fft<L, false>(v, j, my, tw);
        line_fft<L, false>(hc, j, my, tw);
        const size_t ob = ((size_t)g * K + kx) * L + j;
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            const float hh = hc[s].x * hc[s].x + hc[s].y * hc[s].y;
            const float2 Gk = cmulc(v[s], hc[s]);
            a.s_hh[ob + F1 * s] = hh;
            a.s_g[ob + F1 * s] = Gk;
            const float lhs = hh + 1.0f / al;
            v[s] = cscale(make_float2(Gk.x / lhs, Gk.y / lhs), inv_n);
        }
        line_fft<L, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < F2; ++s) S[kx * L + j + F1 * s] = v[s];
    }
    __syncthreads();

    // I: X0's rows -> inverse row FFT -> x0 = clamp(., 0, 1) -> zin; forward row FFT of x0 -> S
    float* zin = a.o2 + (size_t)g * L * L;
    for (int p = line; p < L / 2; p += LINES) {
        float2 v[F2];
        small_gather<L>(S, j, 2 * p, v);
        line_fft<L, true>(v, j, my, tw);
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            const int c = j + F1 * s;
            const float p0 = fminf(fmaxf(v[s].x, 0.f), 1.f), p1 = fminf(fmaxf(v[s].y, 0.f), 1.f);
            zin[(2 * p) * L + c] = p0;
            zin[(2 * p + 1) * L + c] = p1;
            v[s] = make_float2(p0, p1);
        }
        line_fft<L, false>(v, j, my, tw);
        small_split<L>(v, j, my, S, 2 * p);
    }
    __syncthreads();

    // C2: F(x0) columns -> the W~ slot (the first iteration forms W~1 from it: no |H|^2 / G re-read, no rho)
    for (int kx = line; kx < K; kx += LINES) {
        float2 v[F2];
#pragma unroll
        for (int s = 0; s < F2; ++s) v[s] = S[kx * L + j + F1 * s];
        line_fft<L, false>(v, j, my, tw);
        const size_t ob = ((size_t)g * K + kx) * L + j;
#pragma unroll
        for (int s = 0; s < F2; ++s) a.s_w[ob + F1 * s] = v[s];
    }
}
template <int L>
__global__ __launch_bounds__(256) void k_gal_small_init(Args a) {
    __shared__ float2 lds[SmallInitLds<L, 256>::SIZE];
    gal_small_init_body<L, 256>(a, blockIdx.x, threadIdx.x, lds);
}

// The SubNet (k_subnet_rhos_psf) and the fused small init in ONE launch (configs[1]: 256 x 48^2, both a
// single latency-bound round of workgroups): blocks [0, N) run galaxy b's SubNet, blocks [N, 2N) galaxy
// b - N's init on the same 512 threads and the same 80 KiB of LDS, so each CU holds one of each and the
// init's ~12 us hide under the SubNet's ~43 us (as two launches on one stream they ran back to back; on
// two streams a hipGraph replay still started the SubNet only once the init had drained).  The init reads
// no rho (iteration 0 forms W~1), so nothing orders the two halves.
// Block -> (role, galaxy) maps (map): 0 = SubNets in [0, N), inits in [N, 2N); 1 = the two roles alternate
// in each XCD's arrival order (block b runs on XCD b % 8; its q = b / 8-th arrival there), over a grid of
// 2 roundup(N, 8); 2 = the roles alternate block by block.  Blocks of galaxies >= N return at once.
template <int L>
__global__ __launch_bounds__(subnet::kThreads, GD_SN_WPE) void k_subnet_rhos_init(Args a, const float* __restrict__ psf, long long psf_gstride,
                                                                        int h, const float* __restrict__ params,
                                                                        const float* __restrict__ mlp,
                                                                        const float* __restrict__ alpha,
                                                                        long long alpha_stride, float* __restrict__ rhos,
                                                                        int n_out, int map) {
    static_assert(SmallInitLds<L, subnet::kThreads>::SIZE * 8 <= (subnet::kRegionA + subnet::kRegionB) * 4,
                  "the init's LDS inside the SubNet's");
    static_assert(PoisInitLds<L, PoisSmallPlan<L>::TP, PoisSmallPlan<L>::TQ, subnet::kThreads>::SIZE * 8 <=
                      (subnet::kRegionA + subnet::kRegionB) * 4, "the Poisson init's LDS inside the SubNet's");
    __shared__ __attribute__((aligned(16))) float AB[subnet::kRegionA + subnet::kRegionB];
    const int b = blockIdx.x;
    int g, init;
    if (map == 1) {
        const int q = b >> 3;
        g = ((q >> 1) << 3) | (b & 7);
        init = q & 1;
    } else if (map == 2) {
        g = b >> 1;
        init = b & 1;
    } else {
        init = b >= a.N;
        g = init ? b - a.N : b;
    }
    if (g >= a.N) return;  // uniform per block; no barrier crossed
    if (!init) subnet::rhos_body(psf, psf_gstride, h, params, mlp, alpha, alpha_stride, rhos, n_out, AB, g, threadIdx.x);
    else if (a.llh == GD_LLH_POISSON)  // the SPLIT Poisson init (state layout 4: reads no rho; LDS inside the SubNet's)
        pois_small_init_body<L, PoisSmallPlan<L>::TP, PoisSmallPlan<L>::TQ, subnet::kThreads, true>(
            a, g, threadIdx.x, reinterpret_cast<float2*>(AB));
    else gal_small_init_body<L, subnet::kThreads>(a, g, threadIdx.x, reinterpret_cast<float2*>(AB));
}

// ---------------------------------------------------------------- RI: row inverse + sink
template <int MODE>
struct RiTraits {
    static constexpr int NI = (MODE == RI_ITER || MODE == RI_OUT2) ? 2 : 1;
};

template <int L, int MODE, int RBX = 0>
__global__ __launch_bounds__((RowGeo<L, RiTraits<MODE>::NI, RBX>::THREADS)) void k_row_inv(Args a) {
    constexpr int NI = RiTraits<MODE>::NI;
    using G = Geo<L>;
    using R = RowGeo<L, NI, RBX>;
    constexpr int F1 = G::F1, F2 = G::F2;
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 lds[R::LDS];
    const int tid = threadIdx.x;
    const int blocks_per_g = L / R::RB;
    const int g = blockIdx.x / blocks_per_g;
    const int row0 = (blockIdx.x - g * blocks_per_g) * R::RB;
    const int line = tid / F1, j = tid - line * F1;
    const int im = line / R::PAIRS, m = line - im * R::PAIRS;
    fill_twiddles<L>(tw, tid, R::THREADS);
    gather_rows<L, R>(a, lds, g, row0, tid);
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
    if constexpr (MODE == RI_CROP || MODE == RI_CROP_BWD) {
        // UnrolledADMMGaussian: crop_half(fftshift(.)) = the Lh x Lh corner at the origin (see RF_PADV)
        constexpr int Lh = L / 2;
        const float rho = (MODE == RI_CROP_BWD || a.o2) ? a.rho1(g) : 0.f;
        for (int q = tid * 4; q < R::RB * L; q += R::THREADS * 4) {
            const int rr = q / L, c = q - rr * L, r = row0 + rr;
            if (r >= Lh || c >= Lh) continue;
            const size_t p = ((size_t)g * Lh + r) * Lh + c;
            const float4 X = ld4(res + rr * L + c);
            if constexpr (MODE == RI_CROP) {
                st4(a.o0 + p, X);                                  // x (or z0 = init_l2)
                if (a.o2) {                                        // next denoiser input rho x + u (:142)
                    const float4 u = a.a1 ? ld4(a.a1 + p) : make_float4(0.f, 0.f, 0.f, 0.f);
                    st4(a.o2 + p, make_float4(rho * X.x + u.x, rho * X.y + u.y, rho * X.z + u.z, rho * X.w + u.w));
                }
            } else {                                               // dz = rho dv, du = -dv
                st4(a.o0 + p, make_float4(rho * X.x, rho * X.y, rho * X.z, rho * X.w));
                st4(a.o1 + p, make_float4(-X.x, -X.y, -X.z, -X.w));
            }
        }
        return;
    }
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

template <int L, int MODE, int RBX = 0>
__global__ __launch_bounds__((RowGeo<L, 1, RBX>::THREADS)) void k_row_invfwd(Args a) {
    using G = Geo<L>;
    using R = RowGeo<L, 1, RBX>;
    constexpr int F1 = G::F1, F2 = G::F2;
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 lds[R::LDS];
    const int tid = threadIdx.x;
    const int blocks_per_g = L / R::RB;
    const int g = blockIdx.x / blocks_per_g;
    const int row0 = (blockIdx.x - g * blocks_per_g) * R::RB;
    const int line = tid / F1, j = tid - line * F1;
    const int rA = row0 + 2 * line;
    fill_twiddles<L>(tw, tid, R::THREADS);
    gather_rows<L, R>(a, lds, g, row0, tid);
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
    split_store<L, R>(a, lds, g, row0, tid);
}

// ---------------------------------------------------------------- sparse filter power
// |L(kx, ky)|^2 of a filter image with few non-zero taps (the Tikhonov Laplacian), by direct DFT in
// double: sum_t v_t exp(-2 pi i (ky r_t + kx c_t) / L), rounded once.  The regulariser divides the
// spectrum where |H|^2 is ~0, so its absolute error matters there; an fp32 FFT of the placed 3x3
// stencil carries ~1e-6 absolute error, this carries none beyond the final rounding.
__global__ __launch_bounds__(256) void k_sparse_power(const int* rc, const float* vals, int ntaps, float* out,
                                                      int H, int W, int K) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= K * H) return;
    const int kx = idx / H, ky = idx - kx * H;
    const long long HW = (long long)H * W;
    double re = 0.0, im = 0.0;
    for (int t = 0; t < ntaps; ++t) {
        // phase ky r / H + kx c / W as an exact index modulo H W
        const long long ph = ((long long)ky * rc[2 * t] * W + (long long)kx * rc[2 * t + 1] * H) % HW;
        double sn, cs;
        sincospi(-2.0 * double(ph) / double(HW), &sn, &cs);
        re += double(vals[t]) * cs;
        im += double(vals[t]) * sn;
    }
    out[idx] = float(re * re + im * im);
}

// ---------------------------------------------------------------- host-side launch helpers
thread_local std::string g_last_error;

constexpr const char* kRowFwdName = "k_row_fwd";
constexpr const char* kPsfRowsName = "k_psf_rows";
constexpr const char* kColName = "k_col";
constexpr const char* kRowInvName = "k_row_inv";
constexpr const char* kRowInvFwdName = "k_row_invfwd";
constexpr const char* kGalRegName = "k_gal_reg";
constexpr const char* kGalInitName = "k_gal_init";
constexpr const char* kGalSmallName = "k_gal_small";
constexpr const char* kGalSmallInitName = "k_gal_small_init";

inline int fail(int code, const char* msg) {
    g_last_error = msg;
    return code;
}
inline int fail(int code, const std::string& msg) {
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
int g_prof_level = 0;  // 0 off, 1 whole operations (op_*), 2 operations + every kernel launch
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
    ProfScope(const std::string& name, hipStream_t s, int level = 2) : on(false), st(s) {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        if (g_prof_level < level) return;
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
    static int psf_rows(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kPsfRowsName, 0), st);
        const int bpg = (a.h / 2 + G::LPB - 1) / G::LPB;
        hipLaunchKernelGGL((k_psf_rows<L>), dim3(a.N * bpg), dim3(256), 0, st, a);
        return check_launch("k_psf_rows");
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
    static int psf_rows_state(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kPsfRowsName, 1), st);
        const int bpg = (a.h / 2 + G::LPB - 1) / G::LPB;
        hipLaunchKernelGGL((k_psf_rows<L, true>), dim3(a.N * bpg), dim3(256), 0, st, a);
        return check_launch("k_psf_rows");
    }
    template <bool FIRST, bool LAST>
    static int gal_small_v(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kGalSmallName, FIRST + 2 * LAST), st);
        if constexpr (L == 48)  // packed row spectra in LDS, 8 x 6 line plan (k_gal_small_p)
            hipLaunchKernelGGL((k_gal_small_p<L, 8, 6, FIRST, LAST>), dim3(a.N), dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL((k_gal_small<L, FIRST, LAST>), dim3(a.N), dim3(256), 0, st, a);
        return check_launch("k_gal_small");
    }
    static int gal_small_init(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kGalSmallInitName, 0), st);
        hipLaunchKernelGGL((k_gal_small_init<L>), dim3(a.N), dim3(256), 0, st, a);
        return check_launch("k_gal_small_init");
    }
    static int gal_small(const Args& a, hipStream_t st) {
        if (a.first) return a.last ? gal_small_v<true, true>(a, st) : gal_small_v<true, false>(a, st);
        return a.last ? gal_small_v<false, true>(a, st) : gal_small_v<false, false>(a, st);
    }
    static int gal_reg(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kGalRegName, a.first + 2 * a.last), st);
        hipLaunchKernelGGL((k_gal_reg<L>), dim3(a.N), dim3(RegGeo<L>::THREADS), 0, st, a);
        return check_launch("k_gal_reg");
    }
    static int pois_a(const Args& a, hipStream_t st) {
        ProfScope ps(nm("k_pois_a", a.first + 2 * a.last), st);
        hipLaunchKernelGGL((k_gal_reg<L, true>), dim3(a.N), dim3(RegGeo<L>::THREADS), 0, st, a);
        return check_launch("k_gal_reg<POIS>");
    }
    static int pois_b(const Args& a, int init, hipStream_t st) {
        ProfScope ps(nm("k_pois_b", init), st);
        hipLaunchKernelGGL((k_pois_b<L>), dim3(a.N), dim3(RegGeo<L>::THREADS), 0, st, a, init);
        return check_launch("k_pois_b");
    }
    static int gal_reg_init_pois(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kGalInitName, 5), st);
        hipLaunchKernelGGL((k_gal_reg_init<L, true>), dim3(a.N), dim3(RegGeo<L>::THREADS), 0, st, a);
        return check_launch("k_gal_reg_init<POIS>");
    }
    static int rl_reg(const Args& a, int n_iters, hipStream_t st) {
        ProfScope ps(nm("k_rl_reg", 0), st);
        hipLaunchKernelGGL((k_rl_reg<L>), dim3(a.N), dim3(RegGeo<L>::THREADS), 0, st, a, n_iters);
        return check_launch("k_rl_reg");
    }
    static int gal_reg_init(const Args& a, hipStream_t st) {
        ProfScope ps(nm(kGalInitName, 4), st);
        hipLaunchKernelGGL((k_gal_reg_init<L>), dim3(a.N), dim3(RegGeo<L>::THREADS), 0, st, a);
        return check_launch("k_gal_reg_init");
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

// ---------------------------------------------------------------- Infinity-Cache pipelining
// A multi-kernel operation runs over the batch in chunks of G galaxies; consecutive chunks go to
// g_pipe_streams internal HIP streams, forked from and joined back into the caller's stream with
// events (the call stays ordered on - and graph-capturable through - the caller's stream).  Each
// internal stream owns a region of the workspace, so a chunk's spectra stay resident in the 256 MiB
// Infinity Cache between its kernels while the other streams keep the chip full (measured at 256^2:
// one ADMM iteration 7-11 % faster than one pass over the batch; plain sequential chunks on one
// stream were slower than one pass because small grids fill and drain).
size_t g_chunk_bytes = size_t(96) << 20;  // workspace (spectra) bytes per chunk; 0 = one pass
int g_pipe_streams = 2;                   // measured best at 256^2: 2 streams x 96 MiB (186 galaxies)
constexpr int kMaxPipe = 8;
int g_fused = 1;  // Gaussian iterations (and Poisson ones at 256^2 / L <= 112): 1 = the one-launch kernels; 0 = chained
int g_fused_rl = 1;    // Richardson-Lucy at 256^2: 1 = k_rl_reg (whole loop per galaxy), 0 = chunked chain
// gd_subnet_rhos_psf: one fused launch per galaxy up to this batch (one round of workgroups on the 256 CUs:
// 60.5 vs 75.5 us at 256 x 48^2), else the feature kernel + batched MLP (1024: 173 vs 212 us; 4096: 584 vs
// 818 us fused - each fused workgroup re-reads the MLP weights, and 129 VGPRs allow one per CU)
int g_subnet_fused_max = 256;
int g_sri_map = 0;  // k_subnet_rhos_init's block -> (role, galaxy) map (tools/kbench_small)
int g_fused_init = 1;  // Gaussian init (256^2: k_psf_rows<STATE> + k_gal_reg_init) and the other one-launch inits: 1 on; 0 = chunked
// 256^2 Gaussian: the whole-galaxy kernels (k_gal_reg, k_psf_rows + k_gal_reg_init) from this batch up; smaller batches
// run the chained row / column kernels, whose many small workgroups use the CUs a one-workgroup-per-galaxy launch of
// N < 256 leaves idle (r06j: N = 1 2.1x, 8 2.1x, 32 1.62x, 64 1.28x faster chained; 128 1.17x, 256 1.82x faster fused).
// The Gaussian state layout is the same either way, so the choice is per call.
int g_fused_min_n = 96;
// the same for the Poisson two-pass at 256^2 (the state layout follows: 2 from this batch up, 3 below; r06k: the
// three-kernel chain 3.6x at N = 1, 1.86x at 64, 1.17x at 128 faster, the two-pass 1.25x at 256) and for k_rl_reg
// (the chunked chain 2.6x at N = 1, 1.46x at 64 faster; k_rl_reg 1.05x at 128, 2.0x at 256)
int g_pois2_min_n = 192;
int g_rl_min_n = 96;

// Eager pipelined operations fork onto the device's internal streams (PipeRes, shared by the host threads, one
// operation at a time under its mutex).  Under stream capture (mode 2, gd_set_capture_pipeline) an operation
// forks onto streams of the CALLING HOST THREAD instead (CapRes): those streams join the capture and stay in it
// until hipStreamEndCapture, so they must never be the streams another thread's eager calls enqueue on.  Each
// captured operation takes its fork / join events from a ring of kCapSets sets, so no event is recorded twice
// inside one captured forward.
constexpr int kCapSets = 64;
struct PipeRes {
    bool ok = false;
    hipStream_t st[kMaxPipe];
    hipEvent_t fork;
    hipEvent_t join[kMaxPipe];
    // held from the fork record to the last join wait of one pipelined call: the fork / join events and
    // the internal streams are per device, so concurrent callers (host threads) enqueue one at a time
    std::mutex mu;
};
PipeRes g_pipe[64];
std::mutex g_pipe_mu;
struct CapRes {
    hipStream_t st[kMaxPipe];
    hipEvent_t cfork[kCapSets];
    hipEvent_t cjoin[kCapSets][kMaxPipe];
    int cpos = 0;
};
// per host thread and device, created at the thread's first pipelined capture; never freed (a thread's streams and
// events outlive it: destroying them from a thread-exit handler can race the runtime's own teardown)
thread_local CapRes* t_cap[64];

thread_local int g_capture_pipe_override = -1;  // gd_set_capture_pipeline (per host thread)
inline int capture_pipeline_mode() {
    // default 0 (chunks in sequence on the capturing stream): a fork from a stream that itself joined the capture
    // through an event onto internal streams crashed the ROCm 7 runtime inside hipStreamEndCapture;
    // callers that fork from the capturing stream itself (gdeconv.graphs.GraphedForward) opt in to 2
    static const int mode = [] {
        const char* e = std::getenv("GD_CAPTURE_PIPELINE");
        const int m = e ? std::atoi(e) : 0;
        return m == 2 ? 2 : 0;
    }();
    return g_capture_pipe_override >= 0 ? g_capture_pipe_override : mode;
}

inline CapRes* cap_res() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    if (t_cap[dev]) return t_cap[dev];
    CapRes* r = new CapRes();
    for (int i = 0; i < kMaxPipe; ++i)
        if (hipStreamCreateWithFlags(&r->st[i], hipStreamNonBlocking) != hipSuccess) return nullptr;
    for (int c = 0; c < kCapSets; ++c) {
        if (hipEventCreateWithFlags(&r->cfork[c], hipEventDisableTiming) != hipSuccess) return nullptr;
        for (int i = 0; i < kMaxPipe; ++i)
            if (hipEventCreateWithFlags(&r->cjoin[c][i], hipEventDisableTiming) != hipSuccess) return nullptr;
    }
    t_cap[dev] = r;
    return r;
}

inline PipeRes* pipe_res() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    PipeRes& r = g_pipe[dev];
    if (!r.ok) {
        for (int i = 0; i < kMaxPipe; ++i) {
            if (hipStreamCreateWithFlags(&r.st[i], hipStreamNonBlocking) != hipSuccess) return nullptr;
            if (hipEventCreateWithFlags(&r.join[i], hipEventDisableTiming) != hipSuccess) return nullptr;
        }
        if (hipEventCreateWithFlags(&r.fork, hipEventDisableTiming) != hipSuccess) return nullptr;
        r.ok = true;
    }
    return &r;
}

template <int L>
constexpr bool has_fused() { return L == 256; }

inline Args offset_args(const Args& a, int g0, int n, int H, int W) {
    Args b = a;
    b.N = n;
    const size_t img = (size_t)g0 * H * W;
    const size_t spec = (size_t)g0 * (W / 2 + 1) * H;
    if (b.otf && !b.otf_bcast) b.otf += spec;
    if (b.s_hh) b.s_hh += spec;
    if (b.s_g) b.s_g += spec;
    if (b.s_u1) b.s_u1 += spec;
    if (b.s_w) b.s_w += spec;
    if (b.ltl) b.ltl += (long long)g0 * a.ltl_gstride;
    if (b.Tw) b.Tw += 2 * spec;   // full-batch workspace layouts [N][2][K][L]
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
    return b;  // T is set per chunk to its stream's workspace region
}

// f(const Args& chunk, hipStream_t stream) enqueues one chunk's kernels on `stream`.
template <typename F>
int for_chunks_hw(const Args& a, int H, int W, hipStream_t st, F&& f) {
    const size_t tgal = (size_t)2 * (W / 2 + 1) * H * sizeof(float2);  // workspace per galaxy
    int G = a.N;
    if (g_chunk_bytes) {
        const size_t g = g_chunk_bytes / tgal;
        G = (int)(g < 1 ? 1 : (g > (size_t)a.N ? (size_t)a.N : g));
    }
    if (G >= a.N) return f(a, st);
    int S = g_pipe_streams < kMaxPipe ? g_pipe_streams : kMaxPipe;
    if (S > a.N / G) S = a.N / G;  // regions must fit the caller's workspace
    // Under stream capture (GD_CAPTURE_PIPELINE, or gd_set_capture_pipeline per host thread): 0 (default) = the
    // chunks in sequence on the capturing stream; 2 = pipelined over the calling thread's capture streams, each
    // operation's fork / join on its own event set from the ring.  Round 5 (profiles/r05_capture_*): the round-4 crash
    // inside hipStreamEndCapture (4096 x 160^2, profiles/r04dbg_160_graph_crash.txt) came with a fork from a stream
    // that itself joined the capture through an event (ADMMState.init_concurrent's side stream) onto internal streams;
    // forked from the capturing stream itself, mode 2 captures, instantiates and replays bit-identically.  The same
    // fork / join in plain HIP (tools/capture_probe.hip) does not crash.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    const bool capturing = S > 1 && hipStreamIsCapturing(st, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
    if (capturing && capture_pipeline_mode() != 2) S = 1;
    PipeRes* r = (S > 1 && !capturing) ? pipe_res() : nullptr;
    CapRes* cr = (S > 1 && capturing) ? cap_res() : nullptr;
    if (!r && !cr) S = 1;
    std::unique_lock<std::mutex> lk;
    if (r) lk = std::unique_lock<std::mutex>(r->mu);
    hipEvent_t fork = nullptr;
    hipEvent_t* join = nullptr;
    hipStream_t* streams = nullptr;
    if (S > 1) {
        if (cr) {
            const int c = cr->cpos;
            cr->cpos = (c + 1) % kCapSets;
            fork = cr->cfork[c];
            join = cr->cjoin[c];
            streams = cr->st;
        } else {
            fork = r->fork;
            join = r->join;
            streams = r->st;
        }
        if (hipEventRecord(fork, st) != hipSuccess) return fail(GD_ERR_HIP, "pipeline fork");
        for (int i = 0; i < S; ++i)
            if (hipStreamWaitEvent(streams[i], fork, 0) != hipSuccess) return fail(GD_ERR_HIP, "pipeline fork");
    }
    int rc = GD_OK;
    for (int g0 = 0, c = 0; g0 < a.N && rc == GD_OK; g0 += G, ++c) {
        const int n = (a.N - g0 < G) ? a.N - g0 : G;
        Args b = offset_args(a, g0, n, H, W);
        b.T = a.T + (size_t)(c % S) * G * 2 * (W / 2 + 1) * H;
        rc = f(b, S > 1 ? streams[c % S] : st);
    }
    if (S > 1) {
        for (int i = 0; i < S; ++i) {
            if (hipEventRecord(join[i], streams[i]) != hipSuccess || hipStreamWaitEvent(st, join[i], 0) != hipSuccess)
                return fail(GD_ERR_HIP, "pipeline join");
        }
    }
    return rc;
}
template <typename F>
int for_chunks(const Args& a, int L, hipStream_t st, F&& f) {
    return for_chunks_hw(a, L, L, st, std::forward<F>(f));
}

#ifndef GD_REG_REV
#define GD_REG_REV 1
#endif
#ifndef GD_POIS_SMALL
#define GD_POIS_SMALL 1  // 1: Poisson iterations at L <= 112 in one launch (k_pois_small); 0: the three-kernel chain
#endif
// Poisson state layouts (gd_admm_state_layout): 3 = [OTF | u1 | w] with w = v1 - 0 after the init; 4 = the same
// buffers, the init SPLIT (w slot = H x0 until iteration 0 forms w1): the fused small path (L <= 112 square, fused
// init and iterations on) - the init then reads no rho and runs beside the SubNet
inline bool pois_split(int H, int W) {
    return GD_POIS_SMALL && g_fused && g_fused_init && H == W &&
           (H == 32 || H == 48 || H == 64 || H == 80 || H == 96 || H == 112);
}
template <int L>
int pois_small_init_launch(const Args& a, hipStream_t st) {
    using PL = PoisSmallPlan<L>;
    ProfScope ps("k_pois_small_init<" + std::to_string(L) + ">", st);
    if (pois_split(L, L)) hipLaunchKernelGGL((k_pois_small_init<L, PL::TP, PL::TQ, PL::NT, true>), dim3(a.N), dim3(PL::NT), 0, st, a);
    else hipLaunchKernelGGL((k_pois_small_init<L, PL::TP, PL::TQ, PL::NT, false>), dim3(a.N), dim3(PL::NT), 0, st, a);
    return check_launch("k_pois_small_init");
}
template <int L>
int pois_small_launch(const Args& a, hipStream_t st) {
    using PL = PoisSmallPlan<L>;
    static const std::string names[4] = {"k_pois_small<" + std::to_string(L) + ",MID>", "k_pois_small<" + std::to_string(L) + ",FIRST>",
                                         "k_pois_small<" + std::to_string(L) + ",LAST>",
                                         "k_pois_small<" + std::to_string(L) + ",FIRST_LAST>"};
    const bool first = a.first && pois_split(L, L);  // iteration 0 after a SPLIT init forms w1
    ProfScope ps(names[first + 2 * a.last], st);
    if (first) {
        if (a.last) hipLaunchKernelGGL((k_pois_small<L, PL::TP, PL::TQ, PL::NT, true, true>), dim3(a.N), dim3(PL::NT), 0, st, a);
        else hipLaunchKernelGGL((k_pois_small<L, PL::TP, PL::TQ, PL::NT, false, true>), dim3(a.N), dim3(PL::NT), 0, st, a);
    } else {
        if (a.last) hipLaunchKernelGGL((k_pois_small<L, PL::TP, PL::TQ, PL::NT, true>), dim3(a.N), dim3(PL::NT), 0, st, a);
        else hipLaunchKernelGGL((k_pois_small<L, PL::TP, PL::TQ, PL::NT, false>), dim3(a.N), dim3(PL::NT), 0, st, a);
    }
    return check_launch("k_pois_small");
}

// Operation bodies, templated on L.
#ifndef GD_MID_EXTRA
#define GD_MID_EXTRA 1  // 1: k_gal_mid / k_gal_mid_init for the compile-time sizes 96 and 128 too (r04midextra_ab.txt: iteration
                        // 0.346 -> 0.314 / 0.604 -> 0.469 ms, init 0.81 -> 0.43 / 1.00 -> 0.99 ms); k_gal_small stays at 64^2 (0.095 vs 0.168)
#endif
template <int L>
int gal_mid_launch_t(const Args& a, hipStream_t st);
template <int L>
int gal_mid_init_launch_t(const Args& a, hipStream_t st);
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
    // Poisson in two whole-galaxy passes per iteration at 256^2 (gd_poisreg.hpp): the Gaussian init's
    // |H|^2, x0 -> zin and F(x0) with the OTF in the G slot, then pass B with u2 = 0 (w1, W~1)
    static int admm_init_pois2(Args a0, hipStream_t st0) {
        if (g_fused_init && a0.h <= 64) {
            GD_TRY(Lc::psf_rows_state(a0, st0));
            GD_TRY(Lc::gal_reg_init_pois(a0, st0));
        } else {
            GD_TRY(for_chunks(a0, L, st0, [&](const Args& a, hipStream_t st) {
                Args b = a;
                GD_TRY(Lc::template rf<RF_YA>(b, st));
                GD_TRY(Lc::psf_rows(b, st));
                GD_TRY(Lc::template col<C_G_INIT>(b, st));  // llh = Poisson: stores H, not G
                b.o0 = a.o2;
                b.t_slot = 1;
                GD_TRY(Lc::template rif<RIF_CLAMP>(b, st));
                return Lc::template col<C_G_W1>(b, st);     // F(x0) -> the W~ slot (iteration 0 forms W~1)
            }));
        }
        Args b = a0;
        b.s_x = a0.s_w;  // H X := H F(x0), left in the W slot by the init
        return Lc::pois_b(b, 1, st0);
    }
    static int admm_iter_pois2(Args a, hipStream_t st0) {
        // a.a0 = z, a.o0 = zin | out (pass A); a.o1 = w (pass B, in place)
        GD_TRY(Lc::pois_a(a, st0));
        if (a.last) return GD_OK;
        return Lc::pois_b(a, 0, st0);
    }
    static int admm_init(Args a0, hipStream_t st0) {
        // Poisson: a.o0 = u1, a.o1 = w, a.o2 = zin (x0)
        if constexpr (L <= 112) {
            if (GD_POIS_SMALL && g_fused_init) return pois_small_init_launch<L>(a0, st0);  // one launch
        }
        return for_chunks(a0, L, st0, [&](const Args& a, hipStream_t st) {
            Args b = a;
            GD_TRY(Lc::template rf<RF_PSF_Y>(b, st));
            GD_TRY(Lc::template col<C_OTF_INIT>(b, st));
            b.o0 = a.o2;  // RIF_CLAMP writes x0 -> zin
            GD_TRY(Lc::template rif<RIF_CLAMP>(b, st));
            GD_TRY(Lc::template col<C_CONV>(b, st));
            return Lc::template ri<RI_INIT>(a, st);
        });
    }
    static int admm_init_gauss(Args a0, hipStream_t st0) {
        // Gaussian state |H|^2, G and iteration 0's W~; x0 -> zin (a.o2)
        if constexpr (GD_MID_EXTRA && (L == 96 || L == 128)) {
            if (g_fused && g_fused_init) return gal_mid_init_launch_t<L>(a0, st0);  // k_gal_mid_init
        }
        if constexpr (L <= 96) {
            if (g_fused) return Lc::gal_small_init(a0, st0);  // both spectra in LDS, one pass
        }
        if constexpr (has_fused<L>()) {
            if (g_fused_init && a0.h <= 64 && a0.N >= g_fused_min_n) {  // whole-galaxy passes, no workspace: PSF rows -> U1 slot, init, W~
                GD_TRY(Lc::psf_rows_state(a0, st0));
                return Lc::gal_reg_init(a0, st0);
            }
        }
        return for_chunks(a0, L, st0, [&](const Args& a, hipStream_t st) {
            Args b = a;
            GD_TRY(Lc::template rf<RF_YA>(b, st));
            GD_TRY(Lc::psf_rows(b, st));  // PSF row spectra -> slot 1 (free until RIF_CLAMP)
            GD_TRY(Lc::template col<C_G_INIT>(b, st));
            b.o0 = a.o2;    // RIF_CLAMP writes x0 -> zin and its row spectra -> slot 1
            b.t_slot = 1;
            GD_TRY(Lc::template rif<RIF_CLAMP>(b, st));
            return Lc::template col<C_G_W1>(b, st);
        });
    }
    static int admm_iter_gauss(Args a, hipStream_t st0) {
        // a.a0 = z; spectral state updated in place; a.o0 = zin (or the output on the last iteration)
        if constexpr (has_fused<L>()) {
            if (g_fused && a.N >= g_fused_min_n) return Lc::gal_reg(a, st0);  // one pass, no workspace
        }
        if constexpr (GD_MID_EXTRA && (L == 96 || L == 128)) {
            if (g_fused) return gal_mid_launch_t<L>(a, st0);  // k_gal_mid
        }
        if constexpr (L <= 128) {
            if (g_fused) return Lc::gal_small(a, st0);  // whole spectrum in LDS, one pass
        }
        return for_chunks(a, L, st0, [&](const Args& b, hipStream_t st) {
            GD_TRY(Lc::template rf<RF_ONE>(b, st));
            if (b.first)
                GD_TRY(b.last ? Lc::template col<C_G_ITER_FL>(b, st) : Lc::template col<C_G_ITER_F>(b, st));
            else
                GD_TRY(b.last ? Lc::template col<C_G_ITER_L>(b, st) : Lc::template col<C_G_ITER>(b, st));
            return Lc::template ri<RI_OUT1>(b, st);
        });
    }
    static int admm_iter(Args a0, hipStream_t st0) {
        // Poisson: a.a0 = z, a.a1 = u1 (RF reads), a.a2 = w; RI: a.o0 = u1, a.o1 = w, a.o2 = zin / out
        if constexpr (L <= 112) {
            if (GD_POIS_SMALL && g_fused) return pois_small_launch<L>(a0, st0);  // one workgroup per galaxy
        }
        return for_chunks(a0, L, st0, [&](const Args& a, hipStream_t st) {
            GD_TRY(Lc::template rf<RF_ITER>(a, st));
            GD_TRY(Lc::template col<C_ITER>(a, st));
            return Lc::template ri<RI_ITER>(a, st);
        });
    }
    static int wiener(Args a0, hipStream_t st0) {
        return for_chunks(a0, L, st0, [&](const Args& a, hipStream_t st) {
            GD_TRY(Lc::template rf<RF_PSF_RAW>(a, st));
            GD_TRY(Lc::template col<C_WIENER>(a, st));
            return Lc::template ri<RI_OUT1>(a, st);
        });
    }
    static int tikhonov(Args a0, hipStream_t st0) {
        return for_chunks(a0, L, st0, [&](const Args& a, hipStream_t st) {
            GD_TRY(Lc::template rf<RF_PSF_YAR>(a, st));
            GD_TRY(Lc::template col<C_TIKHONOV>(a, st));
            return Lc::template ri<RI_OUT1>(a, st);
        });
    }
    // UnrolledADMMGaussian on the 2x-padded grid (this L = 2 x image side); one pass over the batch
    static int gx_init(Args a, hipStream_t st) {
        GD_TRY(Lc::template rf<RF_PSF_YPAD>(a, st));
        GD_TRY(Lc::template col<C_GX_INIT>(a, st));
        return Lc::template ri<RI_CROP>(a, st);
    }
    static int gx_x(Args a, hipStream_t st) {
        GD_TRY(Lc::template rf<RF_PADV>(a, st));
        GD_TRY(Lc::template col<C_GX>(a, st));
        return Lc::template ri<RI_CROP>(a, st);
    }
    static int gx_x_bwd(Args a, hipStream_t st) {
        GD_TRY(Lc::template rf<RF_PAD2>(a, st));
        GD_TRY(Lc::template col<C_GX_BWD>(a, st));
        return Lc::template ri<RI_CROP_BWD>(a, st);
    }
    static int power(Args a, hipStream_t st) {
        GD_TRY(Lc::template rf<RF_ONE>(a, st));
        return Lc::template col<C_POWER>(a, st);
    }
    static int richardson_lucy(Args a0, int n_iters, hipStream_t st0) {
        if constexpr (has_fused<L>()) {
            if (g_fused_rl && n_iters > 0 && a0.N >= g_rl_min_n) {
                // the OTF (chunked psf_to_otf), then every galaxy's whole loop in one launch
                GD_TRY(for_chunks(a0, L, st0, [&](const Args& a, hipStream_t st) { return psf_to_otf(a, st); }));
                return Lc::rl_reg(a0, n_iters, st0);
            }
        }
        // a.o0 = x (output, also the iterate); otf kept in a.otf.  The whole iteration loop runs per
        // chunk, so x, y, the OTF and the chunk's spectra stay cache-resident across all n_iters.
        return for_chunks(a0, L, st0, [&](const Args& a, hipStream_t st) {
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

// the launch the runtime-planned Gaussian iteration uses at 160^2 (GOps::admm_iter_gauss)
// the square sizes with a fused one-workgroup Gaussian iteration and init (k_gal_mid, k_gal_mid_init): L = 16 TQ,
// lines of 16 lanes (a divisor of the wave) x TQ points (radix 5, 7, 9 = 3 x 3, 10), the packed half spectrum and
// 32 lines' exchange areas in LDS (144^2: 126 KiB, 160^2: 147 KiB)
inline bool mid_size(int H, int W) { return H == W && (H == 80 || H == 112 || H == 144 || H == 160); }
// threads per workgroup: 80, 96 and 112^2 (38 / 52 / 67 KiB of LDS at 256 threads) take 256, so two galaxies share a CU
// (the prefetching k_gal_mid holds ~210 VGPRs: two waves per SIMD); 144 / 160^2 fill the LDS with one galaxy and
// take 512 (at 256 threads they ran 0.66 / 0.77 ms per iteration against 0.60 / 0.73, r04midnt_ab.txt), as does 128^2
#ifndef GD_MID_BIG_THREADS
#define GD_MID_BIG_THREADS 512  // k_gal_mid / k_gal_mid_init workgroup above 112^2
#endif
#ifndef GD_MID_SMALL_THREADS
#define GD_MID_SMALL_THREADS 256  // ... at 80, 96 and 112^2
#endif
template <int L>
constexpr int mid_threads() { return L <= 112 ? GD_MID_SMALL_THREADS : GD_MID_BIG_THREADS; }
template <int L>
int gal_mid_launch_t(const Args& a, hipStream_t st) {
    constexpr int NT = mid_threads<L>(), TP = 16, TQ = L / 16;
    static const std::string names[4] = {"k_gal_mid<" + std::to_string(L) + ",MID>", "k_gal_mid<" + std::to_string(L) + ",FIRST>",
                                         "k_gal_mid<" + std::to_string(L) + ",LAST>",
                                         "k_gal_mid<" + std::to_string(L) + ",FIRST_LAST>"};
    ProfScope ps(names[a.first + 2 * a.last], st);
    if (a.first) {
        if (a.last) hipLaunchKernelGGL((k_gal_mid<L, TP, TQ, NT, true, true>), dim3(a.N), dim3(NT), 0, st, a);
        else hipLaunchKernelGGL((k_gal_mid<L, TP, TQ, NT, true, false>), dim3(a.N), dim3(NT), 0, st, a);
    } else {
        if (a.last) hipLaunchKernelGGL((k_gal_mid<L, TP, TQ, NT, false, true>), dim3(a.N), dim3(NT), 0, st, a);
        else hipLaunchKernelGGL((k_gal_mid<L, TP, TQ, NT, false, false>), dim3(a.N), dim3(NT), 0, st, a);
    }
    return check_launch("k_gal_mid");
}
template <int L>
int gal_mid_init_launch_t(const Args& a, hipStream_t st) {
    constexpr int NT = mid_threads<L>();
    ProfScope ps("k_gal_mid_init<" + std::to_string(L) + ">", st);
    hipLaunchKernelGGL((k_gal_mid_init<L, 16, L / 16, NT>), dim3(a.N), dim3(NT), 0, st, a);
    return check_launch("k_gal_mid_init");
}
inline int gal_mid_launch(const Args& a, hipStream_t st) {
    switch (a.gH) {
        case 80: return gal_mid_launch_t<80>(a, st);
        case 112: return gal_mid_launch_t<112>(a, st);
        case 144: return gal_mid_launch_t<144>(a, st);
        default: return gal_mid_launch_t<160>(a, st);
    }
}
inline int gal_mid_init_launch(const Args& a, hipStream_t st) {
    switch (a.gH) {
        case 80: return gal_mid_init_launch_t<80>(a, st);
        case 112: return gal_mid_init_launch_t<112>(a, st);
        case 144: return gal_mid_init_launch_t<144>(a, st);
        default: return gal_mid_init_launch_t<160>(a, st);
    }
}

#include "gd_generic.hpp"  // GOps: the same operations for any other H x W (runtime-planned line FFTs)

inline bool specialised_size(int H, int W) {
    if (H != W) return false;
    switch (H) {
        case 32: case 48: case 64: case 96: case 128: case 256: return true;
        default: return false;
    }
}

// Square 32/48/64/96/128/256 -> the compile-time-planned Ops<L>; any other H x W in [2, 1024]^2 -> GOps
template <template <int> class OP, typename F>
int dispatch(int H, int W, F&& f) {
    if (H == W) {
        switch (H) {
            case 32: return f(OP<32>{});
            case 48: return f(OP<48>{});
            case 64: return f(OP<64>{});
            case 96: return f(OP<96>{});
            case 128: return f(OP<128>{});
            case 256: return f(OP<256>{});
            default: break;
        }
    }
    if (gen::size_ok(H, W)) return f(GOps{});
    return fail(GD_ERR_UNSUPPORTED, "unsupported image size (H and W must be in [2, 1024])");
}

inline int check_shape(int N, int H, int W) {
    if (N < 0) return fail(GD_ERR_ARG, "negative batch");
    if (!specialised_size(H, W) && !gen::size_ok(H, W))
        return fail(GD_ERR_UNSUPPORTED, "unsupported image size (H and W must be in [2, 1024])");
    return GD_OK;
}

inline int check_psf(int h, int w, int H, int W) {
    if (h != w) return fail(GD_ERR_ARG, "psf must be square (psf_to_otf uses ker.shape[2] for both axes)");
    if (h <= 0 || (h & 1)) return fail(GD_ERR_ARG, "psf side must be even (odd sizes fail in the reference's quadrant copy)");
    if (h > H || h > W) return fail(GD_ERR_ARG, "psf larger than the image");
    return GD_OK;
}

inline Args base_args(int N, void* ws, int H, int W) {
    Args a;
    std::memset(&a, 0, sizeof(a));
    a.N = N;
    a.T = reinterpret_cast<float2*>(ws);
    a.gH = H;
    a.gW = W;
    a.alpha = GalScalar{nullptr, 0};
    a.rho1 = a.rho2 = a.rho2n = a.alpha;
    return a;
}

}  // namespace gd

using namespace gd;
#ifndef GD_KERNELS_ONLY  // tools/*.hip build single kernels without the host library

// ====================================================================== C ABI
extern "C" {

int gd_abi_version(void) { return GD_ABI_VERSION; }

// bumped whenever a kernel's memory traffic changes; PMC summaries are stamped with it so a stale
// profile is never reported against a different engine
const char* gd_engine_rev(void) { return "r06.2"; }

// the source hash __graft_entry__.build() computed (gdeconv._lib.source_hash); the "gdsrc:" marker lets the
// build find it in the binary without loading it
#ifndef GD_SRC_HASH
#define GD_SRC_HASH "unknown"
#endif
static const char g_src_hash_marker[] = "gdsrc:" GD_SRC_HASH;
const char* gd_engine_src_hash(void) { return g_src_hash_marker + 6; }

int gd_hip_runtime_version(void) {
    int v = 0;
    if (hipRuntimeGetVersion(&v) != hipSuccess) return fail(GD_ERR_HIP, "hipRuntimeGetVersion");
    return v;
}

const char* gd_last_error(void) { return g_last_error.c_str(); }

int gd_supported_size(int H, int W) {
    if (specialised_size(H, W)) return 1;   // compile-time-planned kernels
    return gen::size_ok(H, W) ? 2 : 0;      // runtime-planned kernels (gd_generic.hpp)
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
    GD_TRY(check_psf(h, w, H, W));
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H, W);
    a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.otf = reinterpret_cast<float2*>(otf_half);
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::psf_to_otf(a, (hipStream_t)stream); });
}

int gd_conv_fft_batch(const void* otf_half, int conj, const float* x, float* out, int N, int H, int W,
                      void* ws, void* stream) {
    return gd_conv_fft_batch_strided(otf_half, (long long)(W / 2 + 1) * H, conj, x, out, N, H, W, ws, stream);
}

int gd_conv_fft_batch_strided(const void* otf_half, long long otf_gstride, int conj, const float* x, float* out,
                              int N, int H, int W, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (otf_gstride != 0 && otf_gstride != (long long)(W / 2 + 1) * H)
        return fail(GD_ERR_ARG, "otf_gstride must be 0 (one shared OTF) or (W/2+1)*H");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H, W);
    a.otf = reinterpret_cast<float2*>(const_cast<void*>(otf_half));
    a.otf_bcast = otf_gstride == 0;
    a.a0 = x; a.o0 = out;
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::conv(a, conj, (hipStream_t)stream); });
}

int gd_rfft2(const float* x, void* spec, int N, int H, int W, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (N == 0) return GD_OK;
    Args a = base_args(N, spec, H, W);  // spectrum lives in image slot 0 of a T-shaped buffer
    a.a0 = x;
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::rfft2(a, (hipStream_t)stream); });
}

int gd_irfft2(void* spec, float* x, int N, int H, int W, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (N == 0) return GD_OK;
    Args a = base_args(N, spec, H, W);
    a.o0 = x;
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::irfft2(a, (hipStream_t)stream); });
}

// Gap between the Gaussian state's slots at 256^2 (bytes).  The slots are N K L complex apart, a multiple of 8 MiB
// at 256^2 (N = 4096: 2^30 + 2^23 bytes), so one galaxy's |H|^2, G, U1 and W~ bins, which k_gal_reg streams
// together, sat at the same offset modulo every HBM interleave period; 256 KiB between the slots spreads them
// (tools/kbench_reg.hip KB_PAD in the engine layout: MID 1.597 -> 1.565-1.575 ms, profiles/r05_place_ab.txt).
constexpr size_t kStateSlotGap = 256 * 1024;
inline size_t state_slot_gap(int H, int W, int llh) { return (llh == GD_LLH_GAUSSIAN && H == 256 && W == 256) ? kStateSlotGap : 0; }

size_t gd_admm_state_bytes(int N, int H, int W, int llh) {
    if (!gd_supported_size(H, W) || N <= 0) return 0;
    const size_t spec = (size_t)N * (W / 2 + 1) * H * sizeof(float2), img = (size_t)N * H * W * sizeof(float);
    if (llh == GD_LLH_GAUSSIAN)  // |H|^2 padded to 8-byte alignment, the slot gaps
        return (spec / 8 + 1) / 2 * 8 + 3 * spec + 3 * state_slot_gap(H, W, llh);
    // Poisson: [otf | u1 | w] (three-kernel chain); at 256^2 also room for the two-pass layout
    // [(|H|^2) | H | U1 | F(w) | H X] + w (bind_state picks the layout from gd_set_fused_iteration)
    return (H == 256 && W == 256) ? std::max(spec + 2 * img, spec / 2 + 4 * spec + img) : spec + 2 * img;
}

namespace {
bool pois_two_pass(int N, int H, int W, int llh) {
    return llh == GD_LLH_POISSON && H == 256 && W == 256 && g_fused != 0 && N >= g_pois2_min_n;
}
// state layout - Gaussian: [|H|^2 (fp32) | conj(H)F(y/alpha) | F(u1) | conj(H)F(v-u2)] (spectral; at 256^2 with
// kStateSlotGap bytes between the slots);
// Poisson: [otf | u1 | w]
void bind_state(Args& a, void* state, int N, int H, int W, int llh) {
    const size_t spec = (size_t)N * (W / 2 + 1) * H;
    float2* base = reinterpret_cast<float2*>(state);
    if (pois_two_pass(N, H, W, llh)) {
        a.s_hh = reinterpret_cast<float*>(base);
        float2* c = base + spec / 2;
        a.s_g = c;                 // the OTF H
        a.s_u1 = c + spec;
        a.s_w = c + 2 * spec;      // F(w), w = v - u2 (pass B -> pass A, which multiplies by conj(H))
        a.s_x = c + 3 * spec;      // H X (pass A -> pass B)
        a.o1 = reinterpret_cast<float*>(c + 4 * spec);  // w = v - u2 (spatial)
        return;
    }
    if (llh == GD_LLH_GAUSSIAN) {
        const size_t gap = state_slot_gap(H, W, llh) / sizeof(float2);
        a.s_hh = reinterpret_cast<float*>(base);
        float2* c = base + (spec + 1) / 2 + gap;  // |H|^2: spec floats, rounded up to whole float2
        a.s_g = c;
        a.s_u1 = c + spec + gap;
        a.s_w = c + 2 * (spec + gap);
    } else {
        a.otf = base;
        float* u1 = reinterpret_cast<float*>(base + spec);
        a.o0 = u1;                       // u1 (spatial)
        a.o1 = u1 + (size_t)N * H * W;   // w = v - u2 (spatial)
    }
}
}  // namespace

int gd_admm_state_layout(int N, int H, int W, int llh) {
    if (!gd_supported_size(H, W)) return GD_ERR_UNSUPPORTED;
    if (N < 0) return GD_ERR_ARG;
    if (llh == GD_LLH_GAUSSIAN) return 1;
    if (llh != GD_LLH_POISSON) return GD_ERR_ARG;
    return pois_two_pass(N, H, W, llh) ? 2 : (pois_split(H, W) ? 4 : 3);
}

int gd_admm_init_reads_rho(int H, int W, int llh) {
    if (!gd_supported_size(H, W)) return GD_ERR_UNSUPPORTED;
    if (llh == GD_LLH_GAUSSIAN) return 0;  // iteration 0 forms W~1 (w1_value)
    if (llh != GD_LLH_POISSON) return GD_ERR_ARG;
    return pois_split(H, W) ? 0 : 1;       // layout 4: iteration 0 forms w1 (k_pois_small<FIRST>)
}

int gd_admm_init(const float* y, const float* psf, long long psf_gstride, int h, int w,
                 const float* alpha, long long alpha_stride, const float* rho2, long long rho2_stride,
                 int llh, int N, int H, int W, void* state, float* zin, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H, W));
    if (llh != GD_LLH_GAUSSIAN && llh != GD_LLH_POISSON) return fail(GD_ERR_ARG, "llh must be Gaussian or Poisson");
    if (llh == GD_LLH_POISSON && rho2 == nullptr && !pois_split(H, W))
        return fail(GD_ERR_ARG, "the Poisson init takes the first V step: it needs rho2");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H, W);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.alpha = GalScalar{alpha, alpha_stride};
    a.rho2n = GalScalar{rho2, rho2_stride};
    a.llh = llh;
    bind_state(a, state, N, H, W, llh);
    a.o2 = zin;
    ProfScope ps("op_admm_init<" + std::to_string(H) + "," + std::to_string(llh) + ">", (hipStream_t)stream, 1);
    if (llh == GD_LLH_GAUSSIAN)
        return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::admm_init_gauss(a, (hipStream_t)stream); });
    if (pois_two_pass(N, H, W, llh)) return Ops<256>::admm_init_pois2(a, (hipStream_t)stream);
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::admm_init(a, (hipStream_t)stream); });
}

int gd_admm_iter(const float* y, const float* z, float* zin_or_out, const float* alpha, long long alpha_stride,
                 const float* rho1, long long rho1_stride, const float* rho2, long long rho2_stride,
                 const float* rho2_next, long long rho2_next_stride, int llh, int iter, int last, int N, int H,
                 int W, void* state, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (llh != GD_LLH_GAUSSIAN && llh != GD_LLH_POISSON) return fail(GD_ERR_ARG, "llh must be Gaussian or Poisson");
    if (N == 0) return GD_OK;
    if (!last && rho2_next == nullptr) return fail(GD_ERR_ARG, "rho2_next required unless last");
    Args a = base_args(N, ws, H, W);
    a.y = y;
    bind_state(a, state, N, H, W, llh);
    a.alpha = GalScalar{alpha, alpha_stride};
    a.rho1 = GalScalar{rho1, rho1_stride};
    a.rho2 = GalScalar{rho2, rho2_stride};
    a.rho2n = GalScalar{rho2_next ? rho2_next : rho2, rho2_next ? rho2_next_stride : rho2_stride};
    a.llh = llh;
    a.last = last;
    a.first = iter == 0;
    // k_gal_reg's galaxy order alternates from launch to launch (the init runs forward; Poisson's pass B forward,
    // pass A reversed), so a launch starts on the galaxies the previous one finished with - their state, z and
    // zin are the last ~256 MB of traffic, still in the Infinity Cache (GD_REG_REV)
    a.rev = GD_REG_REV ? (llh == GD_LLH_POISSON ? 1 : (iter % 2 == 0)) : 0;
    ProfScope ps("op_admm_iter<" + std::to_string(H) + "," + std::to_string(llh) + ">", (hipStream_t)stream, 1);
    if (llh == GD_LLH_GAUSSIAN) {
        a.a0 = z;
        a.o0 = zin_or_out;
        return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::admm_iter_gauss(a, (hipStream_t)stream); });
    }
    if (pois_two_pass(N, H, W, llh)) {
        a.a0 = z;
        a.o0 = zin_or_out;
        return Ops<256>::admm_iter_pois2(a, (hipStream_t)stream);
    }
    // Poisson: spatial u1 / w (RF reads z, u1, w; RI writes u1, w and zin_or_out)
    a.a0 = z; a.a1 = a.o0; a.a2 = a.o1;
    a.o2 = zin_or_out;
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::admm_iter(a, (hipStream_t)stream); });
}

int gd_admm_iter_v(const long long* v) {
    if (v == nullptr) return fail(GD_ERR_ARG, "gd_admm_iter_v: null argument vector");
    const auto p = [v](int i) { return reinterpret_cast<void*>(static_cast<intptr_t>(v[i])); };
    return gd_admm_iter(static_cast<const float*>(p(0)), static_cast<const float*>(p(1)), static_cast<float*>(p(2)),
                        static_cast<const float*>(p(3)), v[4], static_cast<const float*>(p(5)), v[6],
                        static_cast<const float*>(p(7)), v[8], static_cast<const float*>(p(9)), v[10], (int)v[11],
                        (int)v[12], (int)v[13], (int)v[14], (int)v[15], (int)v[16], p(17), p(18), p(19));
}

int gd_wiener(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
              long long alpha_stride, float* x, int N, int H, int W, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H, W));
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H, W);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.alpha = GalScalar{alpha, alpha_stride};
    a.o0 = x;
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::wiener(a, (hipStream_t)stream); });
}

int gd_richardson_lucy(const float* y, const float* psf, long long psf_gstride, int h, int w, int n_iters,
                       float* x, int N, int H, int W, void* otf_half, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H, W));
    if (n_iters < 0) return fail(GD_ERR_ARG, "n_iters must be >= 0");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H, W);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.otf = reinterpret_cast<float2*>(otf_half);
    a.o0 = x;
    ProfScope ps("op_rl<" + std::to_string(H) + ",0>", (hipStream_t)stream, 1);
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::richardson_lucy(a, n_iters, (hipStream_t)stream); });
}

int gd_tikhonov(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
                long long alpha_stride, const float* lam, long long lam_stride, const float* ltl,
                long long ltl_gstride, float* x, int N, int H, int W, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H, W));
    if (lam == nullptr) return fail(GD_ERR_ARG, "lam required");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H, W);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.alpha = GalScalar{alpha, alpha_stride};
    a.rho1 = GalScalar{lam, lam_stride};
    a.ltl = ltl; a.ltl_gstride = ltl_gstride;
    a.o0 = x;
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::tikhonov(a, (hipStream_t)stream); });
}

int gd_filter_power(const float* filt, float* power_half, int N, int H, int W, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, H, W);
    a.a0 = filt;
    a.s_hh = power_half;
    return dispatch<Ops>(H, W, [&](auto op) { return decltype(op)::power(a, (hipStream_t)stream); });
}

namespace {
int check_gx(int N, int H, int W) {
    if (N < 0) return fail(GD_ERR_ARG, "negative batch");
    // pad_double (utils/utils_torch.py:11-13) doubles even sides only (an odd side gives a 2H - 1 grid
    // whose crop_half no longer matches the image in the reference); H != W pads each side on its own
    // (a 2H x 2W grid: the runtime-planned path, which sizes the padding per axis)
    if (H % 2 || W % 2 || !gd_supported_size(2 * H, 2 * W) || (specialised_size(2 * H, 2 * W) && H % 4))
        return fail(GD_ERR_UNSUPPORTED, "UnrolledADMMGaussian: images of even sides 2 .. 2048 (2x padded grid)");
    return GD_OK;
}
// half spectrum of the 2H x 2W grid, [N][W + 1][2H] (complex elements)
size_t gx_spec_elems(int N, int H, int W) { return (size_t)N * (W + 1) * (2 * H); }
void bind_gx_state(Args& a, void* state, int N, int H, int W) {
    const size_t spec = gx_spec_elems(N, H, W);
    a.s_hh = reinterpret_cast<float*>(state);
    a.s_g = reinterpret_cast<float2*>(state) + spec / 2;
}
}  // namespace

size_t gd_gx_state_bytes(int N, int H, int W) {
    if (check_gx(N, H, W) != GD_OK || N <= 0) return 0;
    return gx_spec_elems(N, H, W) * (sizeof(float) + sizeof(float2));
}

size_t gd_gx_spec_bytes(int N, int H, int W) {
    if (check_gx(N, H, W) != GD_OK || N <= 0) return 0;
    return gx_spec_elems(N, H, W) * sizeof(float2);
}

int gd_gx_init(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
               long long alpha_stride, int N, int H, int W, void* state, float* z0, void* ws, void* stream) {
    GD_TRY(check_gx(N, H, W));
    if (h != H || w != W) return fail(GD_ERR_ARG, "UnrolledADMMGaussian pads the PSF like the image: psf must be H x W");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, 2 * H, 2 * W);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.pw = w == h ? 0 : w;  // H x W (non-square: the runtime-planned path places it per axis)
    a.alpha = GalScalar{alpha, alpha_stride};
    bind_gx_state(a, state, N, H, W);
    a.o0 = z0;
    return dispatch<Ops>(2 * H, 2 * W, [&](auto op) { return decltype(op)::gx_init(a, (hipStream_t)stream); });
}

int gd_gx_xupdate(const float* z, float* u, const float* x_prev, const float* rho, long long rho_stride,
                  const float* rho_prev, long long rho_prev_stride, float* x, float* zin, void* xspec,
                  int N, int H, int W, void* state, void* ws, void* stream) {
    GD_TRY(check_gx(N, H, W));
    if (x_prev && (!u || !rho_prev)) return fail(GD_ERR_ARG, "the fused dual update needs u and rho_prev");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, 2 * H, 2 * W);
    bind_gx_state(a, state, N, H, W);
    a.a0 = z; a.a1 = u; a.a2 = x_prev; a.o1 = u;
    a.rho1 = GalScalar{rho, rho_stride};
    a.rho2 = GalScalar{rho_prev ? rho_prev : rho, rho_prev ? rho_prev_stride : rho_stride};
    a.s_w = reinterpret_cast<float2*>(xspec);
    a.o0 = x; a.o2 = zin;
    return dispatch<Ops>(2 * H, 2 * W, [&](auto op) { return decltype(op)::gx_x(a, (hipStream_t)stream); });
}

int gd_gx_xupdate_backward(const float* grad_x, const float* z, const float* rho, long long rho_stride,
                           const void* xspec, float* grad_z, float* grad_u, float* grad_rho_part, int N, int H,
                           int W, void* state, void* ws, void* stream) {
    GD_TRY(check_gx(N, H, W));
    if (!xspec) return fail(GD_ERR_ARG, "backward needs the forward's saved spectrum");
    if (N == 0) return GD_OK;
    Args a = base_args(N, ws, 2 * H, 2 * W);
    bind_gx_state(a, state, N, H, W);
    a.a0 = grad_x; a.a1 = z;
    a.rho1 = GalScalar{rho, rho_stride};
    a.s_w = reinterpret_cast<float2*>(const_cast<void*>(xspec));
    a.o0 = grad_z; a.o1 = grad_u; a.o2 = grad_rho_part;
    return dispatch<Ops>(2 * H, 2 * W, [&](auto op) { return decltype(op)::gx_x_bwd(a, (hipStream_t)stream); });
}

int gd_filter_power_taps(const int* rc, const float* vals, int ntaps, float* power_half, int H, int W,
                         void* stream) {
    if (H <= 0 || W <= 0 || H > 4096 || W > 4096) return fail(GD_ERR_UNSUPPORTED, "image sides must be in [1, 4096]");
    if (ntaps < 0 || (ntaps > 0 && (!rc || !vals))) return fail(GD_ERR_ARG, "bad tap list");
    const int K = W / 2 + 1;
    hipLaunchKernelGGL(k_sparse_power, dim3((K * H + 255) / 256), dim3(256), 0, (hipStream_t)stream, rc, vals, ntaps,
                       power_half, H, W, K);
    return check_launch("k_sparse_power");
}

int gd_profile_enable(int level) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_level = level < 0 ? 0 : level;
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

int gd_set_capture_pipeline(int mode) {
    // (GD_ERR_ARG is -1, the "no override" value: an invalid mode answers GD_ERR_UNSUPPORTED)
    if (mode != -1 && mode != 0 && mode != 2) return fail(GD_ERR_UNSUPPORTED, "capture pipeline mode must be -1, 0 or 2");
    const int old = g_capture_pipe_override;
    g_capture_pipe_override = mode;
    return old;
}

int gd_set_pipeline_streams(int streams) {
    const int old = g_pipe_streams;
    if (streams >= 1) g_pipe_streams = streams < kMaxPipe ? streams : kMaxPipe;
    return old;
}

int gd_set_fused_init(int on) {
    if (on != 0 && on != 1) return fail(GD_ERR_ARG, "gd_set_fused_init: 0 or 1");
    const int old = g_fused_init;
    g_fused_init = on;
    return old;
}

int gd_set_fused_rl(int on) {
    if (on != 0 && on != 1) return fail(GD_ERR_ARG, "gd_set_fused_rl: 0 or 1");
    const int old = g_fused_rl;
    g_fused_rl = on;
    return old;
}

int gd_set_fused_min_batch(int op, int n) {
    int* t = op == GD_LLH_GAUSSIAN ? &g_fused_min_n : op == GD_LLH_POISSON ? &g_pois2_min_n : op == 2 ? &g_rl_min_n : nullptr;
    if (!t) return fail(GD_ERR_ARG, "gd_set_fused_min_batch: op must be 0 (Gaussian), 1 (Poisson) or 2 (Richardson-Lucy)");
    const int old = *t;
    if (n >= 0) *t = n;
    return old;
}

int gd_set_subnet_fused_max(int n) {
    const int old = g_subnet_fused_max;
    if (n >= 0) g_subnet_fused_max = n;
    return old;
}

int gd_set_fused_iteration(int on) {
    if (on != 0 && on != 1) return fail(GD_ERR_ARG, "gd_set_fused_iteration: 0 or 1");
    const int old = g_fused;
    g_fused = on;
    return old;
}

// the batched SubNet MLP over N feature vectors (MFMA chains, or k_subnet_mlp: bit-identical rhos)
static int subnet_mlp(const float* feat, const float* mlp_params, const float* alpha, long long alpha_stride, float* rhos,
                      int n_out, int N, hipStream_t stream) {
    ProfScope ps("k_subnet_mlp<128,0>", stream, 1);
    if (GD_MLP_MFMA) {
        hipLaunchKernelGGL(gd::subnet::k_subnet_mlp_mfma, dim3((N + gd::subnet::kMG - 1) / gd::subnet::kMG),
                           dim3(gd::subnet::kMlpThreads), 0, stream, feat, mlp_params, alpha, alpha_stride, rhos, n_out, N);
        return check_launch("k_subnet_mlp_mfma");
    }
    hipLaunchKernelGGL(gd::subnet::k_subnet_mlp, dim3((N + gd::subnet::kMlpG - 1) / gd::subnet::kMlpG),
                       dim3(gd::subnet::kMlpThreads), 0, stream, feat, mlp_params, alpha, alpha_stride, rhos, n_out, N);
    return check_launch("k_subnet_mlp");
}

int gd_subnet_param_count(void) { return gd::subnet::kParams; }

int gd_subnet_mlp_param_count(int n_out) {
    return (n_out >= 1 && n_out <= gd::subnet::kMaxOut) ? gd::subnet::mlp_param_count(n_out) : 0;
}

int gd_subnet_rhos(const void* otf128_half, const float* params, const float* mlp_params, const float* alpha,
                   long long alpha_stride, float* feat, float* rhos, int n_out, int N, void* stream) {
    if (N < 0) return fail(GD_ERR_ARG, "negative batch");
    if (n_out < 1 || n_out > gd::subnet::kMaxOut) return fail(GD_ERR_ARG, "n_out must be in [1, 64]");
    if (N == 0) return GD_OK;
    GD_TRY(gd_subnet_features(otf128_half, params, feat, N, stream));
    return subnet_mlp(feat, mlp_params, alpha, alpha_stride, rhos, n_out, N, (hipStream_t)stream);
}

int gd_subnet_rhos_psf(const float* psf, long long psf_gstride, int h, const float* params, const float* mlp_params,
                       const float* alpha, long long alpha_stride, float* feat, float* rhos, int n_out, int N,
                       void* stream) {
    if (N < 0) return fail(GD_ERR_ARG, "negative batch");
    if (n_out < 1 || n_out > gd::subnet::kMaxOut) return fail(GD_ERR_ARG, "n_out must be in [1, 64]");
    if (h < 2 || h > gd::subnet::kPsfMaxH || (h & 1)) return fail(GD_ERR_UNSUPPORTED, "PSF side must be even and <= 64");
    if (N == 0) return GD_OK;
    if (N <= g_subnet_fused_max) {  // features + MLP per galaxy in one workgroup (bit-identical rhos)
        ProfScope ps("k_subnet_rhos<128,2>", (hipStream_t)stream, 1);
        hipLaunchKernelGGL(gd::subnet::k_subnet_rhos_psf, dim3(N), dim3(gd::subnet::kThreads), 0, (hipStream_t)stream,
                           psf, psf_gstride, h, params, mlp_params, alpha, alpha_stride, rhos, n_out, N);
        return check_launch("k_subnet_rhos_psf");
    }
    {
        ProfScope ps("k_subnet_features<128,1>", (hipStream_t)stream, 1);
        hipLaunchKernelGGL(gd::subnet::k_subnet_features_psf, dim3(N), dim3(gd::subnet::kThreads), 0,
                           (hipStream_t)stream, psf, psf_gstride, h, params, feat, N);
        GD_TRY(check_launch("k_subnet_features_psf"));
    }
    return subnet_mlp(feat, mlp_params, alpha, alpha_stride, rhos, n_out, N, (hipStream_t)stream);
}

int gd_admm_init_subnet_supported(int N, int H, int W, int h, int w, int llh, int n_out) {
    if (H != W || !(H == 32 || H == 48 || H == 64) || !g_fused) return 0;
    if (llh != GD_LLH_GAUSSIAN && !(llh == GD_LLH_POISSON && pois_split(H, W))) return 0;
    if (h != w || h < 2 || (h & 1) || h > gd::subnet::kPsfMaxH || h > H) return 0;
    return N >= 1 && N <= g_subnet_fused_max && n_out >= 1 && n_out <= gd::subnet::kMaxOut;
}

int gd_admm_init_subnet(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
                        long long alpha_stride, int llh, int N, int H, int W, void* state, float* zin,
                        const float* params, const float* mlp_params, float* rhos, int n_out, void* ws, void* stream) {
    GD_TRY(check_shape(N, H, W));
    GD_TRY(check_psf(h, w, H, W));
    if (!gd_admm_init_subnet_supported(N, H, W, h, w, llh, n_out))
        return fail(GD_ERR_UNSUPPORTED, "gd_admm_init_subnet: not fusable here (gd_admm_init_subnet_supported)");
    Args a = base_args(N, ws, H, W);
    a.y = y; a.psf = psf; a.psf_gstride = psf_gstride; a.h = h;
    a.alpha = GalScalar{alpha, alpha_stride};
    a.llh = llh;
    bind_state(a, state, N, H, W, llh);
    a.o2 = zin;
    ProfScope ps("op_admm_init_subnet<" + std::to_string(H) + "," + std::to_string(llh) + ">", (hipStream_t)stream, 1);
    const int map = g_sri_map;
    const dim3 grid(map == 1 ? 2 * ((N + 7) / 8 * 8) : 2 * N), block(gd::subnet::kThreads);
#define GD_SRI_LAUNCH(LL)                                                                                            \
    hipLaunchKernelGGL(k_subnet_rhos_init<LL>, grid, block, 0, (hipStream_t)stream, a, psf, psf_gstride, h, params, \
                       mlp_params, alpha, alpha_stride, rhos, n_out, map)
    if (H == 32) GD_SRI_LAUNCH(32);
    else if (H == 48) GD_SRI_LAUNCH(48);
    else GD_SRI_LAUNCH(64);
#undef GD_SRI_LAUNCH
    return check_launch("k_subnet_rhos_init");
}

int gd_subnet_features(const void* otf128_half, const float* params, float* feat, int N, void* stream) {
    if (N < 0) return fail(GD_ERR_ARG, "negative batch");
    if (N == 0) return GD_OK;
    ProfScope ps("k_subnet_features<128,0>", (hipStream_t)stream, 1);
    hipLaunchKernelGGL(gd::subnet::k_subnet_features, dim3(N), dim3(gd::subnet::kThreads), 0, (hipStream_t)stream,
                       reinterpret_cast<const float2*>(otf128_half), params, feat, N);
    return check_launch("k_subnet_features");
}

}  // extern "C"

#include "gd_ingest.hpp"  // host-side packed-batch reader (C ABI gd_pack_*)
#endif  // GD_KERNELS_ONLY
