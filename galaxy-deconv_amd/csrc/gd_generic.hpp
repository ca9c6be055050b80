// gd_generic.hpp - the runtime-size path: any H x W image with 2 <= H, W <= 4096, square or not.
//
// The specialised sizes (square 32, 48, 64, 96, 128, 256) run the compile-time-planned kernels of
// gd_engine.hip.  Every other size the reference's torch.fft path accepts (utils/utils_torch.py:22-27,
// 46-50, 79-92 work for any H x W) runs here, with the SAME operation chains (row forward -> column
// pass -> row inverse, the chunked pipeline of for_chunks) and the same per-bin / per-pixel arithmetic,
// on a line FFT planned at run time:
//
//  * Stockham autosort, mixed radix: n = 4^a 2^b 3^c 5^d p1 p2 ... (radix 2, 3, 4, 5 as explicit butterflies,
//    any other prime factor as a symmetric odd-prime DFT stage, odd_prime_stage), all lines of a workgroup
//    transformed in LDS, ping-pong between two line buffers, one barrier per stage;
//  * twiddles W_n^k = exp(-2 pi i k / n) for k < n computed per workgroup in double (sincospi) and
//    rounded once into an LDS table - no device-side plan buffers, so the C ABI keeps its "no internal
//    allocation, graph-capturable" contract;
//  * row kernels pack two rows of one image into one complex line (the same packing rule as the
//    specialised kernels: rows of one image share its scale); an odd H pads its last pair with a zero
//    row that is never stored; columns are contiguous in the transposed half-spectrum layout
//    [N][W/2+1][H], so column lines load and store coalesced.
//
// Dynamic LDS per workgroup: (n + 2 lines n) float2 <= 64 KiB for lines of n <= 1638 points; longer lines (up to 4096,
// the gfx950 CU's whole 160 KiB for a two-image workgroup) take the larger budget, one workgroup per CU.
#pragma once

namespace gen {

// per axis: a two-image workgroup (one line each, plus the ping-pong buffers) needs 5 n float2 of LDS
constexpr int kMaxLen = 4096;      // 5 n float2 in the CU's 160 KiB
constexpr int kSmallLen = 1638;    // 5 n float2 in 64 KiB: the budget of every line up to here (rounds 1-5 unchanged)
constexpr int kMaxStages = 16;
constexpr int kThreads = 256;
constexpr int kLdsFloat2 = 8192;   // 64 KiB
constexpr int kLdsFloat2Big = 20480;  // 160 KiB (gfx950 LDS per CU)
constexpr int kMaxLines = 16;

struct Axis {
    int n, ns;
    int r[kMaxStages];
};
struct Dims {
    int H, W, K;  // rows, columns, K = W/2 + 1 half-spectrum columns
    Axis row;     // length W
    Axis col;     // length H
};

__host__ __device__ inline int lines_for(int n) {
    const int l = ((n <= kSmallLen ? kLdsFloat2 : kLdsFloat2Big) - n) / (2 * n);
    return l < 1 ? 1 : (l > kMaxLines ? kMaxLines : l);
}
// row pairs per workgroup per image (NI images), and columns per workgroup (NIC lines per column)
__host__ __device__ inline int row_pairs(int NI, int W) {
    const int p = lines_for(W) / NI;
    return p < 1 ? 1 : p;
}
__host__ __device__ inline int col_cols(int NIC, int H) {
    const int c = lines_for(H) / NIC;
    return c < 1 ? 1 : c;
}
inline size_t lds_bytes(int n, int lines) { return (size_t)(n + 2 * lines * n) * sizeof(float2); }

inline Axis make_axis(int n) {
    Axis ax;
    std::memset(&ax, 0, sizeof(ax));
    ax.n = n;
    int m = n;
    while (m % 4 == 0) { ax.r[ax.ns++] = 4; m /= 4; }
    while (m % 2 == 0) { ax.r[ax.ns++] = 2; m /= 2; }
    for (int p = 3; p * p <= m; p += 2)
        while (m % p == 0) { ax.r[ax.ns++] = p; m /= p; }
    if (m > 1) ax.r[ax.ns++] = m;
    return ax;
}

inline bool size_ok(int H, int W) { return H >= 2 && W >= 2 && H <= kMaxLen && W <= kMaxLen; }

// ---------------------------------------------------------------- device: twiddles and line FFTs
__device__ inline void fill_tw(float2* tw, int n) {
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        double s, c;
        sincospi(-2.0 * (double)k / (double)n, &s, &c);
        tw[k] = make_float2((float)c, (float)s);
    }
}
__device__ __forceinline__ float2 twv(const float2* tw, int e, bool inv) {
    const float2 w = tw[e];
    return inv ? make_float2(w.x, -w.y) : w;
}

// A Stockham stage of odd prime radix r >= 7 (butterfly i of each line reads x[i + t m], t < r, and
// writes y[(i - i mod p) r + i mod p + q p]), as the symmetric form of the DFT: with the stage twiddles
// applied, a_t = x_t W_n^{t e1}, and b_t = a_t + a_{r-t}, d_t = a_t - a_{r-t} (t = 1 .. h = (r-1)/2),
//     X_0 = a_0 + sum_t b_t,   X_q, X_{r-q} = A_q -+ i B_q  (forward; inverse +-),
//     A_q = a_0 + sum_t b_t cos(2 pi q t / r),   B_q = sum_t d_t sin(2 pi q t / r).
// h^2 real-coefficient terms per butterfly instead of r^2 complex ones, and every output a sum of h terms,
// split over two accumulators: ~1/4 of the FMAs of a direct DFT and ~3x less rounding growth (a direct
// DFT of 61 or 97 points was 2.4-3.4x further from fp64 than the reference's FFT,
// tests/test_gpu_pixel_parity.py).  Two phases, both spread over the workgroup: the (butterfly, pair)
// items form b_t, d_t in place (each butterfly owns its r inputs), then the (butterfly, q) items sum.
__device__ void odd_prime_stage(float2* x, float2* y, int n, int r, int m, int p, int ts, const float2* tw, int nl,
                                bool inv) {
    const int h = (r - 1) >> 1;
    for (int idx = threadIdx.x; idx < nl * m * h; idx += blockDim.x) {
        const int bi = idx / h, t = idx - bi * h + 1;
        const int line = bi / m, i = bi - line * m;
        const int e1 = (i % p) * ts;  // < m: t e1 < n
        float2* xs = x + line * n + i;
        float2 at = xs[t * m], ar = xs[(r - t) * m];
        if (e1) {
            at = cmul(at, twv(tw, t * e1, inv));
            ar = cmul(ar, twv(tw, (r - t) * e1, inv));
        }
        xs[t * m] = cadd(at, ar);
        xs[(r - t) * m] = csub(at, ar);
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nl * m * (h + 1); idx += blockDim.x) {
        const int bi = idx / (h + 1), q = idx - bi * (h + 1);
        const int line = bi / m, i = bi - line * m;
        const int k = i % p;
        const float2* xs = x + line * n + i;
        float2* ys = y + line * n + (i - k) * r + k;
        const float2 a0 = xs[0];
        if (q == 0) {
            float2 s0 = a0, s1 = make_float2(0.f, 0.f);
            for (int t = 1; t <= h; t += 2) {
                s0 = cadd(s0, xs[t * m]);
                if (t + 1 <= h) s1 = cadd(s1, xs[(t + 1) * m]);
            }
            ys[0] = cadd(s0, s1);
            continue;
        }
        float2 A0 = a0, A1 = make_float2(0.f, 0.f), B0 = A1, B1 = A1;
        const int step = q * m;  // W_r^{q t} = W_n^{(q t mod r) m}
        int e = 0;
        for (int t = 1; t <= h; ++t) {
            e += step;
            if (e >= n) e -= n;
            const float2 w = tw[e];          // (cos, -sin) of 2 pi (q t mod r) / r
            const float c = w.x, sn = -w.y;
            const float2 b = xs[t * m], d = xs[(r - t) * m];
            if (t & 1) {
                A0 = make_float2(fmaf(b.x, c, A0.x), fmaf(b.y, c, A0.y));
                B0 = make_float2(fmaf(d.x, sn, B0.x), fmaf(d.y, sn, B0.y));
            } else {
                A1 = make_float2(fmaf(b.x, c, A1.x), fmaf(b.y, c, A1.y));
                B1 = make_float2(fmaf(d.x, sn, B1.x), fmaf(d.y, sn, B1.y));
            }
        }
        const float2 A = cadd(A0, A1), B = cadd(B0, B1);
        // forward X_q = A - i B, X_{r-q} = A + i B (inverse: the other way round)
        const float2 mi = make_float2(A.x + B.y, A.y - B.x), pl = make_float2(A.x - B.y, A.y + B.x);
        ys[q * p] = inv ? pl : mi;
        ys[(r - q) * p] = inv ? mi : pl;
    }
}

// nl lines of length ax.n, contiguous in x ([line][n]); y is scratch of the same size.  Returns the
// buffer holding the result (x or y).  Stage with radix r after p points combined: butterfly i < n/r
// reads x[i + q n/r], twiddles by W_{p r}^{q (i mod p)}, DFT_r, writes y[(i - i mod p) r + i mod p + q p].
__device__ float2* fft_lines(float2* x, float2* y, const Axis& ax, const float2* tw, int nl, bool inv) {
    const int n = ax.n;
    int p = 1;
    for (int s = 0; s < ax.ns; ++s) {
        const int r = ax.r[s], m = n / r, ts = m / p;
        if (r > 5) {
            odd_prime_stage(x, y, n, r, m, p, ts, tw, nl, inv);
        } else {
            for (int idx = threadIdx.x; idx < nl * m; idx += blockDim.x) {
                const int line = idx / m, i = idx - line * m;
                const int k = i % p;
                const float2* xs = x + line * n + i;
                float2* ys = y + line * n + (i - k) * r + k;
                const int e1 = k * ts;  // < n / r
                if (r == 2) {
                    const float2 a0 = xs[0], a1 = cmul(xs[m], twv(tw, e1, inv));
                    ys[0] = cadd(a0, a1);
                    ys[p] = csub(a0, a1);
                } else if (r == 4) {
                    const float2 a0 = xs[0], a1 = cmul(xs[m], twv(tw, e1, inv)), a2 = cmul(xs[2 * m], twv(tw, 2 * e1, inv)),
                                 a3 = cmul(xs[3 * m], twv(tw, 3 * e1, inv));
                    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3);
                    const float2 d = csub(a1, a3);
                    const float2 t3 = inv ? make_float2(-d.y, d.x) : make_float2(d.y, -d.x);  // (a1 - a3) (-+i)
                    ys[0] = cadd(t0, t2);
                    ys[p] = cadd(t1, t3);
                    ys[2 * p] = csub(t0, t2);
                    ys[3 * p] = csub(t1, t3);
                } else if (r == 3) {
                    const float2 a0 = xs[0], a1 = cmul(xs[m], twv(tw, e1, inv)), a2 = cmul(xs[2 * m], twv(tw, 2 * e1, inv));
                    const float2 sm = cadd(a1, a2), df = csub(a1, a2);
                    const float2 t = make_float2(a0.x - 0.5f * sm.x, a0.y - 0.5f * sm.y);
                    const float c3 = 0.866025403784438646763723f;                 // sin(2 pi / 3)
                    // forward: W = -1/2 - i sqrt(3)/2;  -i c3 (a1 - a2) for X1, +i c3 (a1 - a2) for X2
                    const float2 u = inv ? make_float2(-c3 * df.y, c3 * df.x) : make_float2(c3 * df.y, -c3 * df.x);
                    ys[0] = cadd(a0, sm);
                    ys[p] = cadd(t, u);
                    ys[2 * p] = csub(t, u);
                } else {  // r == 5
                    const float2 a0 = xs[0], a1 = cmul(xs[m], twv(tw, e1, inv)), a2 = cmul(xs[2 * m], twv(tw, 2 * e1, inv)),
                                 a3 = cmul(xs[3 * m], twv(tw, 3 * e1, inv)), a4 = cmul(xs[4 * m], twv(tw, 4 * e1, inv));
                    const float c1 = 0.309016994374947424102f, c2 = -0.809016994374947424102f;  // cos(2pi/5), cos(4pi/5)
                    const float s1 = 0.951056516295153572116f, s2 = 0.587785252292473129169f;   // sin(2pi/5), sin(4pi/5)
                    const float2 b1 = cadd(a1, a4), b2 = cadd(a2, a3), d1 = csub(a1, a4), d2 = csub(a2, a3);
                    const float2 t1 = make_float2(a0.x + c1 * b1.x + c2 * b2.x, a0.y + c1 * b1.y + c2 * b2.y);
                    const float2 t2 = make_float2(a0.x + c2 * b1.x + c1 * b2.x, a0.y + c2 * b1.y + c1 * b2.y);
                    const float2 u1 = make_float2(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y);
                    const float2 u2 = make_float2(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y);
                    // forward: X1 = t1 - i u1, X4 = t1 + i u1, X2 = t2 - i u2, X3 = t2 + i u2 (inverse: i -> -i)
                    const float2 iu1 = inv ? make_float2(-u1.y, u1.x) : make_float2(u1.y, -u1.x);
                    const float2 iu2 = inv ? make_float2(-u2.y, u2.x) : make_float2(u2.y, -u2.x);
                    ys[0] = cadd(a0, cadd(b1, b2));
                    ys[p] = cadd(t1, iu1);
                    ys[2 * p] = cadd(t2, iu2);
                    ys[3 * p] = csub(t2, iu2);
                    ys[4 * p] = csub(t1, iu1);
                }
            }
        }
        __syncthreads();
        float2* t = x;
        x = y;
        y = t;
        p *= r;
    }
    return x;
}

// ---------------------------------------------------------------- device: sources and sinks
// psf_to_otf's placement (utils/utils_torch.py:82-88) on an H x W grid: padded pixel (r, c) holds PSF
// pixel ((r + h/2) mod H, (c + h/2) mod W) when both are < h, zero elsewhere.  An h x pw PSF (a.pw != 0:
// UnrolledADMMGaussian's image-size kernel of a non-square image, pad_double + ifftshift at
// models/unrolled_admm_gaussian.py:122) is centred per axis: column offset pw/2, columns < pw.
__device__ __forceinline__ float gpsf(const Args& a, int g, int r, int c, int H, int W) {
    const int pw = a.pw ? a.pw : a.h;
    int i = r + (a.h >> 1), jj = c + (pw >> 1);
    if (i >= H) i -= H;
    if (jj >= W) jj -= W;
    if (i >= a.h || jj >= pw) return 0.0f;
    return a.psf[(long long)g * a.psf_gstride + (long long)i * pw + jj];
}

// the row-forward producers of gd_engine.hip's rf_source4, one pixel at a time
template <int MODE>
__device__ __forceinline__ float gsrc(const Args& a, const Dims& d, int g, int im, int r, int c) {
    const size_t pix = ((size_t)g * d.H + r) * d.W + c;
    if constexpr (MODE == RF_ITER) {
        if (im == 0) return a.a0[pix] - a.a1[pix];   // z - u1
        return a.a2[pix];                            // w = v - u2
    } else if constexpr (MODE == RF_PSF || MODE == RF_PSF_Y || MODE == RF_PSF_YP || MODE == RF_PSF_RAW ||
                         MODE == RF_PSF_YAR) {
        if (im == 0) return gpsf(a, g, r, c, d.H, d.W);
        const float y = a.y[pix];
        if constexpr (MODE == RF_PSF_RAW) return y;
        if constexpr (MODE == RF_PSF_YAR) return y / a.alpha(g);
        const float yp = fmaxf(y, 0.f);
        if constexpr (MODE == RF_PSF_YP) {
            a.o0[pix] = yp;                          // Richardson-Lucy x0 = max(y, 0)
            return yp;
        } else {
            return yp / a.alpha(g);                  // max(y, 0) / alpha
        }
    } else if constexpr (MODE == RF_PADV || MODE == RF_PSF_YPAD || MODE == RF_PAD2) {
        // UnrolledADMMGaussian: Sh x Sw sources at the origin of the 2Sh x 2Sw grid (gd_engine.hip RF_PAD*)
        const int Sh = d.H / 2, Sw = d.W / 2;
        if constexpr (MODE == RF_PSF_YPAD) {
            if (im == 0) return gpsf(a, g, r, c, d.H, d.W);
        }
        if (r >= Sh || c >= Sw) return 0.f;
        const size_t p = ((size_t)g * Sh + r) * Sw + c;
        if constexpr (MODE == RF_PSF_YPAD) {
            return fmaxf(a.y[p], 0.f);
        } else if constexpr (MODE == RF_PAD2) {
            return (im == 0 ? a.a0 : a.a1)[p];
        } else {
            const float z = a.a0[p];
            float u = a.a1 ? a.a1[p] : 0.f;
            if (a.a2) {
                u = u + a.rho2(g) * (a.a2[p] - z);   // u + rho_prev (x_prev - z), in place
                a.o1[p] = u;
            }
            return a.rho1(g) * z - u;
        }
    } else if constexpr (MODE == RF_ONE) {
        return a.a0[pix];
    } else if constexpr (MODE == RF_YA) {
        return fmaxf(a.y[pix], 0.f) / a.alpha(g);
    } else {
        return (im == 0 ? a.a0 : a.a1)[pix];
    }
}

// rows 2 pr, 2 pr + 1 of image im (pr = p0 + mm) -> line im pb + mm; the spectra of each image's rows
// from the packed line spectra C: row 2m (C + conj D)/2, row 2m+1 (C - conj D)/(2i), D = C[(W - k) mod W]
__device__ __forceinline__ void gsplit_store(const Args& a, const Dims& d, const float2* res, int g, int p0, int pb,
                                             int nl) {
    const int H = d.H, W = d.W, K = d.K;
    float2* T = a.Tw ? a.Tw : a.T;
    for (int e = threadIdx.x; e < nl * K; e += blockDim.x) {
        const int mm = e % pb, t = e / pb;
        const int k = t % K, im = t / K;
        const int r0 = 2 * (p0 + mm);
        if (r0 >= H) continue;
        const int line = im * pb + mm;
        const float2 C = res[line * W + k], D = res[line * W + (k == 0 ? 0 : W - k)];
        const size_t o = tidx(g, im + a.t_slot, k, r0, K, H);
        T[o] = make_float2(0.5f * (C.x + D.x), 0.5f * (C.y - D.y));
        if (r0 + 1 < H) T[o + 1] = make_float2(0.5f * (C.y + D.y), 0.5f * (D.x - C.x));
    }
}

// the Hermitian-extended packed line R_even + i R_odd of rows 2 pr, 2 pr + 1 of image slot im
__device__ __forceinline__ void ggather(const Args& a, const Dims& d, float2* x, int g, int p0, int pb, int nl) {
    const int H = d.H, W = d.W, K = d.K;
    for (int e = threadIdx.x; e < nl * K; e += blockDim.x) {
        const int mm = e % pb, t = e / pb;
        const int k = t % K, im = t / K;
        const int r0 = 2 * (p0 + mm), r1 = r0 + 1;
        float2 Re = make_float2(0.f, 0.f), Ro = Re;
        if (r0 < H) Re = a.T[tidx(g, im, k, r0, K, H)];
        if (r1 < H) Ro = a.T[tidx(g, im, k, r1, K, H)];
        const bool self = (k == 0) || (2 * k == W);  // self-conjugate bins: real parts only (irfft)
        if (self) {
            Re.y = 0.f;
            Ro.y = 0.f;
        }
        const int line = im * pb + mm;
        x[line * W + k] = make_float2(Re.x - Ro.y, Re.y + Ro.x);
        if (!self) x[line * W + (W - k)] = make_float2(Re.x + Ro.y, Ro.x - Re.y);
    }
}

// ---------------------------------------------------------------- RF: row forward
template <int MODE>
__global__ __launch_bounds__(kThreads) void k_gen_rf(Args a, Dims d) {
    constexpr int NI = RfTraits<MODE>::NI;
    extern __shared__ __attribute__((aligned(16))) float2 gsm[];
    const int H = d.H, W = d.W;
    const int pb = row_pairs(NI, W), nl = NI * pb;
    const int bpg = ((H + 1) / 2 + pb - 1) / pb;
    const int g = blockIdx.x / bpg, p0 = (blockIdx.x - g * bpg) * pb;
    float2* tw = gsm;
    float2* x = gsm + W;
    float2* y = x + nl * W;
    fill_tw(tw, W);
    for (int e = threadIdx.x; e < nl * W; e += blockDim.x) {
        const int line = e / W, c = e - line * W;
        const int im = line / pb, r0 = 2 * (p0 + line - im * pb);
        const float v0 = r0 < H ? gsrc<MODE>(a, d, g, im, r0, c) : 0.f;
        const float v1 = r0 + 1 < H ? gsrc<MODE>(a, d, g, im, r0 + 1, c) : 0.f;
        x[e] = make_float2(v0, v1);
    }
    __syncthreads();
    const float2* res = fft_lines(x, y, d.row, tw, nl, false);
    gsplit_store(a, d, res, g, p0, pb, nl);
}

// ---------------------------------------------------------------- C: column pass
// Generic C_G_INIT takes the OTF column from slot 0 (RF_PSF_Y: the placed PSF) and F(max(y,0)/alpha)
// from slot 1 (the specialised kernels build the OTF from k_psf_rows' compact rows instead).
template <int MODE>
struct GColTraits {
    static constexpr bool IN2 = ColTraits<MODE>::IN2 || MODE == C_G_INIT;
};

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_gen_col(Args a, Dims d) {
    using TR = ColTraits<MODE>;
    constexpr int NIC = GColTraits<MODE>::IN2 ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) float2 gsm[];
    const int H = d.H, W = d.W, K = d.K;
    const int cb = col_cols(NIC, H), nl = NIC * cb;
    const int NK = a.N * K, f0 = blockIdx.x * cb;
    float2* tw = gsm;
    float2* x = gsm + H;
    float2* y = x + nl * H;
    fill_tw(tw, H);
    for (int e = threadIdx.x; e < nl * H; e += blockDim.x) {
        const int line = e / H, ky = e - line * H;
        const int im = line / cb, f = f0 + line - im * cb;
        float2 v = make_float2(0.f, 0.f);
        if (f < NK) {
            const int g = f / K, kx = f - g * K;
            v = a.T[tidx(g, MODE == C_G_W1 ? 1 : im, kx, ky, K, H)];  // C_G_W1: x0's row spectra in slot 1
        }
        x[e] = v;
    }
    __syncthreads();
    float2* P = TR::FWD ? fft_lines(x, y, d.col, tw, nl, false) : x;
    float2* O = (P == x) ? y : x;
    const float inv_n = float(1.0 / ((double)H * (double)W));
    constexpr bool giter = (MODE == C_G_ITER || MODE == C_G_ITER_F || MODE == C_G_ITER_L || MODE == C_G_ITER_FL);
    constexpr bool gfirst = (MODE == C_G_ITER_F || MODE == C_G_ITER_FL);
    constexpr bool glast = (MODE == C_G_ITER_L || MODE == C_G_ITER_FL);
    float* part = reinterpret_cast<float*>(O);  // C_GX_BWD: per-bin d/drho terms [cb][H]
    for (int e = threadIdx.x; e < cb * H; e += blockDim.x) {
        const int cc = e / H, ky = e - cc * H, f = f0 + cc;
        if (f >= NK) {
            if constexpr (MODE == C_GX_BWD) part[e] = 0.f;
            continue;
        }
        const int g = f / K, kx = f - g * K;
        const size_t ob = ((size_t)g * K + kx) * H, o = ob + ky;
        float2& Pv = P[cc * H + ky];
        float2 Qv = make_float2(0.f, 0.f);
        if constexpr (NIC == 2) Qv = P[(cb + cc) * H + ky];
        float2 Hk = make_float2(0.f, 0.f);
        if constexpr (TR::LOAD_OTF) Hk = a.otf[(a.otf_bcast ? (size_t)kx * H : ob) + ky];
        if constexpr (TR::STORE_OTF || MODE == C_WIENER || MODE == C_TIKHONOV) Hk = Pv;
        if constexpr (TR::STORE_OTF) a.otf[o] = Hk;
        if constexpr (MODE == C_ITER) {
            // runtime X_Update (models/Unrolled_ADMM.py:315-319): X = (rho1 F(z-u1) + rho2 conj(H) F(w)) / lhs
            const float r1 = a.rho1(g), r2 = a.rho2(g);
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float lhs = r1 * HtH + r2;
            const float2 HtW = cmulc(Qv, Hk);
            const float2 rhs = make_float2(r1 * Pv.x + r2 * HtW.x, r1 * Pv.y + r2 * HtW.y);
            const float2 X = make_float2(rhs.x / lhs, rhs.y / lhs);
            Pv = cscale(X, inv_n);
            P[(cb + cc) * H + ky] = cscale(cmul(Hk, X), inv_n);
        } else if constexpr (MODE == C_OTF_INIT) {
            // init_l2 (models/Unrolled_ADMM.py:170-175): conj(H) F(y/alpha) / (|H|^2 + 1/alpha)
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float lhs = HtH + 1.0f / a.alpha(g);
            const float2 rhs = cmulc(Qv, Hk);
            Pv = cscale(make_float2(rhs.x / lhs, rhs.y / lhs), inv_n);
        } else if constexpr (MODE == C_G_INIT) {
            // init_l2 + the Gaussian constants |H|^2, G = conj(H) F(y/alpha); X0 = G / (|H|^2 + 1/alpha)
            const float2 Hk2 = Pv;
            const float hh = Hk2.x * Hk2.x + Hk2.y * Hk2.y;
            const float2 Gk = cmulc(Qv, Hk2);
            a.s_hh[o] = hh;
            a.s_g[o] = Gk;
            const float lhs = hh + 1.0f / a.alpha(g);
            Pv = cscale(make_float2(Gk.x / lhs, Gk.y / lhs), inv_n);
        } else if constexpr (giter) {
            // the Gaussian iteration on spectra (gauss_math, shared with every specialised kernel)
            const float hh = a.s_hh[o];
            const float2 Gk = (glast && !gfirst) ? make_float2(0.f, 0.f) : a.s_g[o];
            const float2 U1 = gfirst ? make_float2(0.f, 0.f) : a.s_u1[o];
            float2 Wt = a.s_w[o];
            if constexpr (gfirst) Wt = w1_value(hh, Gk, Wt, a.rho2(g));  // the slot holds F(x0)
            float2 U1o, Wo;
            Pv = gauss_math<glast>(hh, Gk, U1, Wt, Pv, a.rho1(g), a.rho2(g), glast ? 0.f : a.rho2n(g), inv_n, U1o, Wo);
            if constexpr (!glast) {
                a.s_u1[o] = U1o;
                a.s_w[o] = Wo;
            }
        } else if constexpr (MODE == C_G_W1) {
            // F(x0) -> the W~ slot: iteration 0 forms W~ = conj(H) V1 (the first V step,
            // models/Unrolled_ADMM.py:335-336) from it (w1_value), so the init reads no rho
            a.s_w[o] = Pv;
        } else if constexpr (MODE == C_WIENER) {
            // models/Wiener.py:16-18: conj(H) F(y) / (|H|^2 + 350/alpha)
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float div = HtH + 350.0f / a.alpha(g);
            const float2 num = cmulc(Qv, Hk);
            Pv = cscale(make_float2(num.x / div, num.y / div), inv_n);
        } else if constexpr (MODE == C_TIKHONOV) {
            // models/Tikhonet.py:19-29: conj(H) F(y/alpha) / (|H|^2 + lam [|L|^2])
            const float lam = a.rho1(g);
            const float HtH = Hk.x * Hk.x + Hk.y * Hk.y;
            const float div = a.ltl ? HtH + lam * a.ltl[(size_t)g * a.ltl_gstride + (size_t)kx * H + ky] : HtH + lam;
            const float2 num = cmulc(Qv, Hk);
            Pv = cscale(make_float2(num.x / div, num.y / div), inv_n);
        } else if constexpr (MODE == C_GX_INIT) {
            // UnrolledADMMGaussian (models/unrolled_admm_gaussian.py:111-127)
            const float2 Hk2 = Pv;
            const float hh = Hk2.x * Hk2.x + Hk2.y * Hk2.y;
            const float2 Gk = cmulc(Qv, Hk2);
            a.s_hh[o] = hh;
            a.s_g[o] = Gk;
            const float lhs = hh + 1.0f / a.alpha(g);
            Pv = cscale(make_float2(Gk.x / lhs, Gk.y / lhs), inv_n);
        } else if constexpr (MODE == C_GX) {
            // XUpdateGaussian (:89-93): X = (Ht Y + F(rho z - u)) / (rho + HtH)
            const float lhs = a.rho1(g) + a.s_hh[o];
            const float2 rhs = cadd(a.s_g[o], Pv);
            const float2 X = make_float2(rhs.x / lhs, rhs.y / lhs);
            if (a.s_w) a.s_w[o] = X;
            Pv = cscale(X, inv_n);
        } else if constexpr (MODE == C_GX_BWD) {
            // adjoint of the X update; d/drho over the full spectrum (bins other than kx = 0, W/2 twice)
            const float D = a.rho1(g) + a.s_hh[o];
            const float2 X = a.s_w[o];
            const float2 dd = csub(Qv, X);
            const float wk = (kx == 0 || 2 * kx == W) ? 1.f : 2.f;
            part[e] = wk * (Pv.x * dd.x + Pv.y * dd.y) / D;
            Pv = cscale(make_float2(Pv.x / D, Pv.y / D), inv_n);
        } else if constexpr (MODE == C_POWER) {
            a.s_hh[o] = Pv.x * Pv.x + Pv.y * Pv.y;
        } else if constexpr (MODE == C_OTF_CONV) {
            Pv = cscale(cmul(Qv, Hk), inv_n);
        } else if constexpr (MODE == C_CONV) {
            Pv = cscale(cmul(Pv, Hk), inv_n);
        } else if constexpr (MODE == C_CONVC) {
            Pv = cscale(cmulc(Pv, Hk), inv_n);
        } else if constexpr (MODE == C_CONV2) {
            Pv = cscale(cmul(Pv, Hk), inv_n);
            P[(cb + cc) * H + ky] = cscale(cmul(Qv, Hk), inv_n);
        } else if constexpr (MODE == C_INV) {
            Pv = cscale(Pv, inv_n);
        }
    }
    __syncthreads();
    if constexpr (MODE == C_GX_BWD) {
        if ((int)threadIdx.x < cb && f0 + (int)threadIdx.x < NK) {  // fixed-order sum per column
            const int f = f0 + threadIdx.x;
            float s = 0.f;
            for (int ky = 0; ky < H; ++ky) s += part[threadIdx.x * H + ky];
            a.o2[f] = s * inv_n;  // [N][K]: f = g K + kx
        }
        __syncthreads();
    }
    if constexpr (MODE == C_FWD) {
        for (int e = threadIdx.x; e < cb * H; e += blockDim.x) {
            const int cc = e / H, ky = e - cc * H, f = f0 + cc;
            if (f < NK) a.T[tidx(f / K, 0, f % K, ky, K, H)] = P[e];
        }
    } else if constexpr (TR::HAS_OUT) {
        const int nout = TR::OUT2 ? 2 * cb : cb;
        const float2* R = fft_lines(P, O, d.col, tw, nout, true);
        for (int e = threadIdx.x; e < nout * H; e += blockDim.x) {
            const int line = e / H, ky = e - line * H;
            const int im = line / cb, f = f0 + line - im * cb;
            if (f < NK) a.T[tidx(f / K, im, f % K, ky, K, H)] = R[e];
        }
    }
}

// ---------------------------------------------------------------- RI: row inverse + sink
template <int MODE>
__global__ __launch_bounds__(kThreads) void k_gen_ri(Args a, Dims d) {
    constexpr int NI = RiTraits<MODE>::NI;
    extern __shared__ __attribute__((aligned(16))) float2 gsm[];
    const int H = d.H, W = d.W, K = d.K;
    const int pb = row_pairs(NI, W), nl = NI * pb;
    const int bpg = ((H + 1) / 2 + pb - 1) / pb;
    const int g = blockIdx.x / bpg, p0 = (blockIdx.x - g * bpg) * pb;
    float2* tw = gsm;
    float2* x = gsm + W;
    float2* y = x + nl * W;
    fill_tw(tw, W);
    ggather(a, d, x, g, p0, pb, nl);
    __syncthreads();
    const float2* res = fft_lines(x, y, d.row, tw, nl, true);
    float al = 1.f, r2n = 1.f, div = 1.f;
    if constexpr (MODE == RI_ITER || MODE == RI_INIT) {
        al = a.alpha(g);
        if (!(MODE == RI_ITER && a.last)) r2n = a.rho2n(g);
    }
    if constexpr (MODE == RI_RL_FINAL) div = a.otf[(size_t)g * K * H].x;  // conv(Ht, ones) = H(0,0)
    const bool poisson = a.llh == GD_LLH_POISSON;
    // this block's rows 2 p0 .. 2 (p0 + pb) - 1 of each image: value (rr odd ? imag : real) of line rr/2
    for (int e = threadIdx.x; e < 2 * pb * W; e += blockDim.x) {
        const int rr = e / W, c = e - rr * W, r = 2 * p0 + rr;
        if (r >= H) continue;
        const float2 v0 = res[(rr >> 1) * W + c];
        const float X = (rr & 1) ? v0.y : v0.x;
        if constexpr (MODE == RI_CROP || MODE == RI_CROP_BWD) {
            const int Sh = H / 2, Sw = W / 2;
            if (r >= Sh || c >= Sw) continue;
            const size_t p = ((size_t)g * Sh + r) * Sw + c;
            if constexpr (MODE == RI_CROP) {
                a.o0[p] = X;                                               // x (or z0 = init_l2)
                if (a.o2) a.o2[p] = a.rho1(g) * X + (a.a1 ? a.a1[p] : 0.f);  // rho x + u (:142)
            } else {
                const float rho = a.rho1(g);
                a.o0[p] = rho * X;                                         // dz = rho dv
                a.o1[p] = -X;                                              // du = -dv
            }
            continue;
        }
        const size_t pix = ((size_t)g * H + r) * W + c;
        if constexpr (MODE == RI_ITER) {
            // models/Unrolled_ADMM.py:207-215 (x = image 0, conv(H, x) = image 1)
            const float2 v1 = res[(pb + (rr >> 1)) * W + c];
            const float hx = (rr & 1) ? v1.y : v1.x;
            if (a.last) {
                a.o2[pix] = poisson ? X * al : X;
            } else {
                const float u1 = (a.o0[pix] + X) - a.a0[pix];           // u1 + x - z
                const float u2 = hx - a.o1[pix];                         // u2 + conv(H,x) - v  (w = v - u2)
                const float vn = v_step(a.llh, hx + u2, fmaxf(a.y[pix], 0.f), r2n, al);
                a.o0[pix] = u1;
                a.o1[pix] = vn - u2;
                a.o2[pix] = X + u1;                                      // next denoiser input
            }
        } else if constexpr (MODE == RI_INIT) {
            a.o1[pix] = v_step(a.llh, X + 0.0f, fmaxf(a.y[pix], 0.f), r2n, al);
            a.o0[pix] = 0.f;
        } else if constexpr (MODE == RI_OUT1) {
            a.o0[pix] = X;
        } else if constexpr (MODE == RI_OUT2) {
            const float2 v1 = res[(pb + (rr >> 1)) * W + c];
            a.o0[pix] = X;
            a.o1[pix] = (rr & 1) ? v1.y : v1.x;
        } else if constexpr (MODE == RI_RL_FINAL) {
            a.o0[pix] = a.o0[pix] * X / div;                             // x * numerator / divisor
        }
    }
}

// ---------------------------------------------------------------- RIF: row inverse -> pointwise -> row forward
template <int MODE>
__device__ __forceinline__ float gif_point(const Args& a, size_t pix, float re, float div) {
    if constexpr (MODE == RIF_CLAMP) {
        const float p = fminf(fmaxf(re, 0.f), 1.f);  // torch.clamp(x0, 0, 1)
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

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_gen_rif(Args a, Dims d) {
    extern __shared__ __attribute__((aligned(16))) float2 gsm[];
    const int H = d.H, W = d.W, K = d.K;
    const int pb = row_pairs(1, W), nl = pb;
    const int bpg = ((H + 1) / 2 + pb - 1) / pb;
    const int g = blockIdx.x / bpg, p0 = (blockIdx.x - g * bpg) * pb;
    float2* tw = gsm;
    float2* x = gsm + W;
    float2* y = x + nl * W;
    fill_tw(tw, W);
    ggather(a, d, x, g, p0, pb, nl);
    __syncthreads();
    float2* res = fft_lines(x, y, d.row, tw, nl, true);
    float div = 1.f;
    if constexpr (MODE == RIF_RL_UPDATE) div = a.otf[(size_t)g * K * H].x;
    for (int e = threadIdx.x; e < nl * W; e += blockDim.x) {
        const int mm = e / W, c = e - mm * W;
        const int r0 = 2 * (p0 + mm);
        float2 v = res[e];
        const size_t pix = ((size_t)g * H + r0) * W + c;
        v.x = r0 < H ? gif_point<MODE>(a, pix, v.x, div) : 0.f;
        v.y = r0 + 1 < H ? gif_point<MODE>(a, pix + W, v.y, div) : 0.f;
        res[e] = v;
    }
    __syncthreads();
    const float2* out = fft_lines(res, res == x ? y : x, d.row, tw, nl, false);
    gsplit_store(a, d, out, g, p0, pb, nl);
}

// ---------------------------------------------------------------- host: launches and operations
struct GLaunch {
    static Dims dims(const Args& a) {
        Dims d;
        d.H = a.gH;
        d.W = a.gW;
        d.K = a.gW / 2 + 1;
        d.row = make_axis(d.W);
        d.col = make_axis(d.H);
        return d;
    }
    static std::string nm(const char* k, int mode, const Dims& d) {
        return std::string(k) + "<" + std::to_string(d.H) + "x" + std::to_string(d.W) + "," + std::to_string(mode) + ">";
    }
    // dynamic LDS above 64 KiB (lines longer than kSmallLen) must be allowed per kernel before its launch; set once
    // per kernel and size (normally at an eager call, before any stream capture of the same operation)
    static int allow_lds(const void* k, size_t bytes) {
        if (bytes <= 65536) return GD_OK;
        static std::mutex mu;
        static std::map<const void*, size_t> allowed;
        std::lock_guard<std::mutex> lk(mu);
        size_t& have = allowed[k];
        if (have >= bytes) return GD_OK;
        if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
            return fail(GD_ERR_HIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
        have = bytes;
        return GD_OK;
    }
    static int row_grid(int NI, const Args& a, const Dims& d) {
        const int pb = row_pairs(NI, d.W);
        return a.N * (((d.H + 1) / 2 + pb - 1) / pb);
    }
    template <int MODE>
    static int rf(const Args& a, hipStream_t st) {
        const Dims d = dims(a);
        constexpr int NI = RfTraits<MODE>::NI;
        ProfScope ps(nm("k_gen_rf", MODE, d), st);
        const size_t lb = lds_bytes(d.W, NI * row_pairs(NI, d.W));
        GD_TRY(allow_lds(reinterpret_cast<const void*>(&k_gen_rf<MODE>), lb));
        hipLaunchKernelGGL((k_gen_rf<MODE>), dim3(row_grid(NI, a, d)), dim3(kThreads), lb, st, a, d);
        return check_launch("k_gen_rf");
    }
    template <int MODE>
    static int col(const Args& a, hipStream_t st) {
        const Dims d = dims(a);
        constexpr int NIC = GColTraits<MODE>::IN2 ? 2 : 1;
        const int cb = col_cols(NIC, d.H);
        ProfScope ps(nm("k_gen_col", MODE, d), st);
        const size_t lb = lds_bytes(d.H, NIC * cb);
        GD_TRY(allow_lds(reinterpret_cast<const void*>(&k_gen_col<MODE>), lb));
        hipLaunchKernelGGL((k_gen_col<MODE>), dim3((a.N * d.K + cb - 1) / cb), dim3(kThreads), lb, st, a, d);
        return check_launch("k_gen_col");
    }
    template <int MODE>
    static int ri(const Args& a, hipStream_t st) {
        const Dims d = dims(a);
        constexpr int NI = RiTraits<MODE>::NI;
        ProfScope ps(nm("k_gen_ri", MODE, d), st);
        const size_t lb = lds_bytes(d.W, NI * row_pairs(NI, d.W));
        GD_TRY(allow_lds(reinterpret_cast<const void*>(&k_gen_ri<MODE>), lb));
        hipLaunchKernelGGL((k_gen_ri<MODE>), dim3(row_grid(NI, a, d)), dim3(kThreads), lb, st, a, d);
        return check_launch("k_gen_ri");
    }
    template <int MODE>
    static int rif(const Args& a, hipStream_t st) {
        const Dims d = dims(a);
        ProfScope ps(nm("k_gen_rif", MODE, d), st);
        const size_t lb = lds_bytes(d.W, row_pairs(1, d.W));
        GD_TRY(allow_lds(reinterpret_cast<const void*>(&k_gen_rif<MODE>), lb));
        hipLaunchKernelGGL((k_gen_rif<MODE>), dim3(row_grid(1, a, d)), dim3(kThreads), lb, st, a, d);
        return check_launch("k_gen_rif");
    }
};

}  // namespace gen

// The operations of Ops<L> for a runtime H x W (a.gH x a.gW), same chains, same workspace layout.
struct GOps {
    using Lc = gen::GLaunch;
    template <typename F>
    static int chunks(const Args& a, hipStream_t st, F&& f) {
        return for_chunks_hw(a, a.gH, a.gW, st, std::forward<F>(f));
    }
    static int psf_to_otf(Args a, hipStream_t st) {
        GD_TRY(Lc::rf<RF_PSF>(a, st));
        return Lc::col<C_OTF>(a, st);
    }
    static int conv(Args a, int conj, hipStream_t st) {
        GD_TRY(Lc::rf<RF_ONE>(a, st));
        GD_TRY(conj ? Lc::col<C_CONVC>(a, st) : Lc::col<C_CONV>(a, st));
        return Lc::ri<RI_OUT1>(a, st);
    }
    static int rfft2(Args a, hipStream_t st) {
        GD_TRY(Lc::rf<RF_ONE>(a, st));
        return Lc::col<C_FWD>(a, st);
    }
    static int irfft2(Args a, hipStream_t st) {
        GD_TRY(Lc::col<C_INV>(a, st));
        return Lc::ri<RI_OUT1>(a, st);
    }
    static int admm_init(Args a0, hipStream_t st0) {
        // Poisson: a.o0 = u1, a.o1 = w, a.o2 = zin (x0); 80^2 / 112^2 in one launch (k_pois_small_init)
        if (GD_POIS_SMALL && g_fused_init && a0.gH == a0.gW && (a0.gH == 80 || a0.gH == 112) && a0.pw == 0)
            return a0.gH == 80 ? pois_small_init_launch<80>(a0, st0) : pois_small_init_launch<112>(a0, st0);
        return chunks(a0, st0, [&](const Args& a, hipStream_t st) {
            Args b = a;
            GD_TRY(Lc::rf<RF_PSF_Y>(b, st));
            GD_TRY(Lc::col<C_OTF_INIT>(b, st));
            b.o0 = a.o2;  // RIF_CLAMP writes x0 -> zin
            GD_TRY(Lc::rif<RIF_CLAMP>(b, st));
            GD_TRY(Lc::col<C_CONV>(b, st));
            return Lc::ri<RI_INIT>(a, st);
        });
    }
    static int admm_init_gauss(Args a0, hipStream_t st0) {
        // Gaussian state |H|^2, G and iteration 0's W~; x0 -> zin (a.o2)
        // 80 / 112 / 144 / 160: one launch, one workgroup per galaxy (k_gal_mid_init: the same state as this chain)
        // (one predicate for every mid size, compile-time 96 / 128 included: both switches on)
        if (GD_MID_FUSED && g_fused && g_fused_init && mid_size(a0.gH, a0.gW) && a0.pw == 0) return gal_mid_init_launch(a0, st0);
        return chunks(a0, st0, [&](const Args& a, hipStream_t st) {
            Args b = a;
            GD_TRY(Lc::rf<RF_PSF_Y>(b, st));  // placed PSF -> slot 0, max(y,0)/alpha -> slot 1
            GD_TRY(Lc::col<C_G_INIT>(b, st));
            b.o0 = a.o2;    // RIF_CLAMP writes x0 -> zin and its row spectra -> slot 1
            b.t_slot = 1;
            GD_TRY(Lc::rif<RIF_CLAMP>(b, st));
            return Lc::col<C_G_W1>(b, st);
        });
    }
    static int admm_iter_gauss(Args a, hipStream_t st0) {
        // 80 / 112 / 144 / 160: the whole iteration in one workgroup per galaxy (k_gal_mid; the same state layout and per-bin
        // arithmetic as this chain)
        if (GD_MID_FUSED && g_fused && mid_size(a.gH, a.gW)) return gal_mid_launch(a, st0);
        return chunks(a, st0, [&](const Args& b, hipStream_t st) {
            GD_TRY(Lc::rf<RF_ONE>(b, st));
            if (b.first)
                GD_TRY(b.last ? Lc::col<C_G_ITER_FL>(b, st) : Lc::col<C_G_ITER_F>(b, st));
            else
                GD_TRY(b.last ? Lc::col<C_G_ITER_L>(b, st) : Lc::col<C_G_ITER>(b, st));
            return Lc::ri<RI_OUT1>(b, st);
        });
    }
    static int admm_iter(Args a0, hipStream_t st0) {
        // Poisson at 80^2 / 112^2: one workgroup per galaxy (k_pois_small: the same state as this chain)
        if (GD_POIS_SMALL && g_fused && a0.gH == a0.gW && (a0.gH == 80 || a0.gH == 112))
            return a0.gH == 80 ? pois_small_launch<80>(a0, st0) : pois_small_launch<112>(a0, st0);
        return chunks(a0, st0, [&](const Args& a, hipStream_t st) {
            GD_TRY(Lc::rf<RF_ITER>(a, st));
            GD_TRY(Lc::col<C_ITER>(a, st));
            return Lc::ri<RI_ITER>(a, st);
        });
    }
    static int wiener(Args a0, hipStream_t st0) {
        return chunks(a0, st0, [&](const Args& a, hipStream_t st) {
            GD_TRY(Lc::rf<RF_PSF_RAW>(a, st));
            GD_TRY(Lc::col<C_WIENER>(a, st));
            return Lc::ri<RI_OUT1>(a, st);
        });
    }
    static int tikhonov(Args a0, hipStream_t st0) {
        return chunks(a0, st0, [&](const Args& a, hipStream_t st) {
            GD_TRY(Lc::rf<RF_PSF_YAR>(a, st));
            GD_TRY(Lc::col<C_TIKHONOV>(a, st));
            return Lc::ri<RI_OUT1>(a, st);
        });
    }
    static int gx_init(Args a, hipStream_t st) {
        GD_TRY(Lc::rf<RF_PSF_YPAD>(a, st));
        GD_TRY(Lc::col<C_GX_INIT>(a, st));
        return Lc::ri<RI_CROP>(a, st);
    }
    static int gx_x(Args a, hipStream_t st) {
        GD_TRY(Lc::rf<RF_PADV>(a, st));
        GD_TRY(Lc::col<C_GX>(a, st));
        return Lc::ri<RI_CROP>(a, st);
    }
    static int gx_x_bwd(Args a, hipStream_t st) {
        GD_TRY(Lc::rf<RF_PAD2>(a, st));
        GD_TRY(Lc::col<C_GX_BWD>(a, st));
        return Lc::ri<RI_CROP_BWD>(a, st);
    }
    static int power(Args a, hipStream_t st) {
        GD_TRY(Lc::rf<RF_ONE>(a, st));
        return Lc::col<C_POWER>(a, st);
    }
    static int richardson_lucy(Args a0, int n_iters, hipStream_t st0) {
        return chunks(a0, st0, [&](const Args& a, hipStream_t st) {
            GD_TRY(Lc::rf<RF_PSF_YP>(a, st));
            if (n_iters <= 0) return GD_OK;
            GD_TRY(Lc::col<C_OTF_CONV>(a, st));
            for (int it = 0; it < n_iters; ++it) {
                if (it > 0) GD_TRY(Lc::col<C_CONV>(a, st));
                GD_TRY(Lc::rif<RIF_RL_RATIO>(a, st));
                GD_TRY(Lc::col<C_CONVC>(a, st));
                if (it + 1 < n_iters)
                    GD_TRY(Lc::rif<RIF_RL_UPDATE>(a, st));
                else
                    GD_TRY(Lc::ri<RI_RL_FINAL>(a, st));
            }
            return GD_OK;
        });
    }
};
