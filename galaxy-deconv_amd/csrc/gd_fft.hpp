// Device-side FFT building blocks for gfx950 (CDNA4), fp32.
//
//  * DFT<N, INV>      : in-register mixed-radix (2/3/4) Cooley-Tukey on N complex values, every
//                       twiddle a compile-time constant (computed in double, rounded once).
//  * line_fft<L, INV> : length-L complex FFT spread over F1 lanes of ONE wave (the "line"), each
//                       lane holding F2 = L/F1 points.  Four-step: DFT-F2 in registers, twiddle
//                       W_L^{n1 k1} from an LDS table, one LDS transpose inside the wave, DFT-F1
//                       in registers.  Lane j holds x[j + F1*r] (r = 0..F2-1) on entry and
//                       X[j + F1*r] on exit, so a forward transform, a pointwise spectral op and an
//                       inverse transform chain with no extra data movement.
//  Requirements: F1 | F2 (so stage B is balanced), F1 <= 64, line lanes contiguous in one wave.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

namespace gd {

// ---------------------------------------------------------------- compile-time trigonometry
constexpr double kPi = 3.14159265358979323846264338327950288;

constexpr double cx_sin(double x) {  // |x| <= pi; Taylor to far below double eps
    double term = x, sum = x;
    for (int i = 1; i < 40; ++i) {
        term *= -x * x / ((2.0 * i) * (2.0 * i + 1.0));
        sum += term;
    }
    return sum;
}
constexpr double cx_cos(double x) {
    double term = 1.0, sum = 1.0;
    for (int i = 1; i < 40; ++i) {
        term *= -x * x / ((2.0 * i - 1.0) * (2.0 * i));
        sum += term;
    }
    return sum;
}
// W_N^m = exp(-+2 pi i m / N) (forward: minus), angle reduced to [-pi, pi] before the series.
template <int N, int M, bool INV>
struct Twiddle {
    static constexpr int m = ((M % N) + N) % N;
    static constexpr int mr = (2 * m > N) ? m - N : m;  // in [-N/2, N/2]
    static constexpr double ang = (INV ? 2.0 : -2.0) * kPi * double(mr) / double(N);
    static constexpr float re = float(cx_cos(ang));
    static constexpr float im = float(cx_sin(ang));
};

// ---------------------------------------------------------------- complex helpers
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// a * conj(b)
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {
    return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 mul_mi(float2 a) {
    return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}

template <int N, int M, bool INV>
__device__ __forceinline__ float2 twmul(float2 v) {
    constexpr int m = ((M % N) + N) % N;
    if constexpr (m == 0) {
        return v;
    } else if constexpr (2 * m == N) {
        return make_float2(-v.x, -v.y);
    } else if constexpr (4 * m == N) {
        return mul_mi<INV>(v);
    } else if constexpr (4 * m == 3 * N) {
        return mul_mi<!INV>(v);
    } else {
        return cmul(v, make_float2(Twiddle<N, M, INV>::re, Twiddle<N, M, INV>::im));
    }
}

// ---------------------------------------------------------------- static_for
template <int I, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < E) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, E>(f);
    }
}

// ---------------------------------------------------------------- packed complex (VOP3P)
// The transforms compute on c2 = (re, im) in one aligned VGPR pair, so every complex add is one
// v_pk_add_f32.  The products whose operands need their halves swapped or negated (a variable complex
// multiply, multiplication by -+i inside an add) are written as single VOP3P instructions with op_sel /
// neg modifiers: left to the compiler, the scalar form was re-paired by the SLP vectoriser with ~100
// moves and sign xors per 256-point line (429 -> ~280 instructions per line FFT).
typedef float c2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ c2 tc2(float2 a) { return c2{a.x, a.y}; }
__device__ __forceinline__ float2 tf2(c2 a) { return make_float2(a.x, a.y); }
// two halves of a * b / a * conj(b), issued separately so that independent products interleave (a VOP3P
// result read by the next instruction costs an s_nop)
__device__ __forceinline__ c2 pmul_t(c2 a, c2 b) {
    c2 t;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(b));
    return t;
}
template <bool CONJ>
__device__ __forceinline__ c2 pmul_r(c2 a, c2 b, c2 t) {
    c2 r;
    if constexpr (CONJ)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    else
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;
}
// a * b
__device__ __forceinline__ c2 pmul(c2 a, c2 b) {
    c2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(b));          // (ay by, ay bx)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;                                                                                          // (ax bx - ay by, ax by + ay bx)
}
// a * conj(b)
__device__ __forceinline__ c2 pmulc(c2 a, c2 b) {
    c2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(b));          // (ay by, ay bx)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;                                                                                          // (ax bx + ay by, ay bx - ax by)
}
// b + (-i) s (forward) / b + i s (inverse), one instruction
#ifndef GD_FFT_ASM_MI
#define GD_FFT_ASM_MI 1
#endif
template <bool INV>
__device__ __forceinline__ c2 add_mi(c2 b, c2 s) {
    if constexpr (!GD_FFT_ASM_MI) return INV ? b + c2{-s.y, s.x} : b + c2{s.y, -s.x};  // folded to op_sel / neg
    c2 r;
    if constexpr (INV)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(b), "v"(s));
    else
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(b), "v"(s));
    return r;
}
// v * (re + i im) for compile-time constants (the compiler keeps (re, im) in an SGPR pair)
__device__ __forceinline__ c2 cmul_const(c2 v, float re, float im) {
    return __builtin_elementwise_fma(v.yy, c2{-im, re}, v.xx * c2{re, im});
}
template <bool INV>
__device__ __forceinline__ c2 vmul_mi(c2 a) {
    return INV ? c2{-a.y, a.x} : c2{a.y, -a.x};
}
template <int N, int M, bool INV>
__device__ __forceinline__ c2 vtwmul(c2 v) {
    constexpr int m = ((M % N) + N) % N;
    if constexpr (m == 0) {
        return v;
    } else if constexpr (2 * m == N) {
        return -v;
    } else if constexpr (4 * m == N) {
        return vmul_mi<INV>(v);
    } else if constexpr (4 * m == 3 * N) {
        return vmul_mi<!INV>(v);
    } else {
        return cmul_const(v, Twiddle<N, M, INV>::re, Twiddle<N, M, INV>::im);
    }
}

// ---------------------------------------------------------------- in-register DFTs
constexpr int first_factor(int n) {
    return (n % 4 == 0 && n != 4) ? 4 : (n % 2 == 0 ? 2 : (n % 3 == 0 ? 3 : (n % 5 == 0 ? 5 : 7)));
}

template <int N, bool INV>
struct DFT {
    static constexpr int A = first_factor(N);
    static constexpr int B = N / A;
    static_assert(A * B == N, "unsupported DFT size");
    // N = A*B, n = A*n2 + n1, k = k1 + B*k2
    __device__ __forceinline__ static void run(c2 (&x)[N]) {
        c2 t[A][B];
        static_for<0, A>([&](auto n1c) {
            constexpr int n1 = decltype(n1c)::value;
            c2 y[B];
            static_for<0, B>([&](auto n2c) { y[decltype(n2c)::value] = x[A * decltype(n2c)::value + n1]; });
            DFT<B, INV>::run(y);
            static_for<0, B>([&](auto k1c) {
                constexpr int k1 = decltype(k1c)::value;
                t[n1][k1] = vtwmul<N, n1 * k1, INV>(y[k1]);
            });
        });
        static_for<0, B>([&](auto k1c) {
            constexpr int k1 = decltype(k1c)::value;
            c2 z[A];
            static_for<0, A>([&](auto n1c) { z[decltype(n1c)::value] = t[decltype(n1c)::value][k1]; });
            DFT<A, INV>::run(z);
            static_for<0, A>([&](auto k2c) { x[k1 + B * decltype(k2c)::value] = z[decltype(k2c)::value]; });
        });
    }
    __device__ __forceinline__ static void run(float2 (&x)[N]) {
        c2 v[N];
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = tc2(x[i]);
        run(v);
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = tf2(v[i]);
    }
};

template <bool INV>
struct DFT<1, INV> {
    __device__ __forceinline__ static void run(c2 (&)[1]) {}
};

template <bool INV>
struct DFT<2, INV> {
    __device__ __forceinline__ static void run(c2 (&x)[2]) {
        const c2 a = x[0], b = x[1];
        x[0] = a + b;
        x[1] = a - b;
    }
};

template <bool INV>
struct DFT<3, INV> {
    __device__ __forceinline__ static void run(c2 (&x)[3]) {
        constexpr float s3 = 0.866025403784438646763723170752936183f;  // sqrt(3)/2
        const c2 t1 = x[1] + x[2];
        const c2 t2 = x[0] - 0.5f * t1;
        const c2 d = s3 * (x[1] - x[2]);
        // forward: X1 = t2 - i s3 d ; X2 = t2 + i s3 d
        x[0] = x[0] + t1;
        x[1] = add_mi<INV>(t2, d);
        x[2] = add_mi<!INV>(t2, d);
    }
};

template <bool INV>
struct DFT<5, INV> {
    // forward X1 = a1 - i b1, X4 = a1 + i b1, X2 = a2 - i b2, X3 = a2 + i b2 (c_k = cos(2 pi k / 5), s_k = sin)
    __device__ __forceinline__ static void run(c2 (&x)[5]) {
        constexpr float c1 = 0.309016994374947424102293417182819059f, c2k = -0.809016994374947424102293417182819059f;
        constexpr float s1 = 0.951056516295153572116439333379382143f, s2 = 0.587785252292473129168705954639072769f;
        const c2 t1 = x[1] + x[4], t2 = x[2] + x[3], t3 = x[1] - x[4], t4 = x[2] - x[3];
        const c2 a1 = x[0] + c1 * t1 + c2k * t2, a2 = x[0] + c2k * t1 + c1 * t2;
        const c2 b1 = s1 * t3 + s2 * t4, b2 = s2 * t3 - s1 * t4;
        x[0] = x[0] + t1 + t2;
        x[1] = add_mi<INV>(a1, b1);
        x[4] = add_mi<!INV>(a1, b1);
        x[2] = add_mi<INV>(a2, b2);
        x[3] = add_mi<!INV>(a2, b2);
    }
};

template <bool INV>
struct DFT<7, INV> {
    // the symmetric form (gd_generic.hpp's odd_prime_stage): b_t = x_t + x_{7-t}, d_t = x_t - x_{7-t};
    // forward X_q = A_q - i B_q, X_{7-q} = A_q + i B_q, A_q = x0 + sum_t c_{qt} b_t, B_q = sum_t s_{qt} d_t
    __device__ __forceinline__ static void run(c2 (&x)[7]) {
        constexpr float c1 = 0.623489801858733530525004884004239811f, c2k = -0.222520933956314404288902564496794759f,
                        c3 = -0.900968867902419126236102319507445051f;
        constexpr float s1 = 0.781831482468029808708444526674057750f, s2 = 0.974927912181823607018131682993931217f,
                        s3 = 0.433883739117558120475768332848358754f;
        const c2 b1 = x[1] + x[6], b2 = x[2] + x[5], b3 = x[3] + x[4];
        const c2 d1 = x[1] - x[6], d2 = x[2] - x[5], d3 = x[3] - x[4];
        const c2 a1 = x[0] + c1 * b1 + c2k * b2 + c3 * b3;
        const c2 a2 = x[0] + c2k * b1 + c3 * b2 + c1 * b3;
        const c2 a3 = x[0] + c3 * b1 + c1 * b2 + c2k * b3;
        const c2 e1 = s1 * d1 + s2 * d2 + s3 * d3;
        const c2 e2 = s2 * d1 - s3 * d2 - s1 * d3;
        const c2 e3 = s3 * d1 - s1 * d2 + s2 * d3;
        x[0] = x[0] + b1 + b2 + b3;
        x[1] = add_mi<INV>(a1, e1);
        x[6] = add_mi<!INV>(a1, e1);
        x[2] = add_mi<INV>(a2, e2);
        x[5] = add_mi<!INV>(a2, e2);
        x[3] = add_mi<INV>(a3, e3);
        x[4] = add_mi<!INV>(a3, e3);
    }
};

template <bool INV>
struct DFT<4, INV> {
    __device__ __forceinline__ static void run(c2 (&x)[4]) {
        const c2 a = x[0] + x[2], b = x[0] - x[2];
        const c2 c = x[1] + x[3], d = x[1] - x[3];
        x[0] = a + c;
        x[2] = a - c;
        x[1] = add_mi<INV>(b, d);
        x[3] = add_mi<!INV>(b, d);
    }
};

// ---------------------------------------------------------------- line plans
template <int L>
struct Plan;
template <> struct Plan<32>  { static constexpr int F1 = 4,  F2 = 8;  };
template <> struct Plan<48>  { static constexpr int F1 = 4,  F2 = 12; };
template <> struct Plan<64>  { static constexpr int F1 = 8,  F2 = 8;  };
template <> struct Plan<96>  { static constexpr int F1 = 4,  F2 = 24; };
template <> struct Plan<128> { static constexpr int F1 = 8,  F2 = 16; };
template <> struct Plan<256> { static constexpr int F1 = 16, F2 = 16; };

// LDS floats2 needed per line for the in-wave transpose (row pad of one element).
template <int L>
constexpr int xch_elems() { return Plan<L>::F1 * (Plan<L>::F2 + 1); }

// Memory ordering for an exchange whose lanes all sit in ONE wave: LDS requests of a wave are
// processed in order, so only the compiler needs fencing.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Transposing four-step line FFT, N = P Q on the first max(P, Q) lanes of a line (for plans whose lane
// count does not divide the points per lane, e.g. 48 = 8 x 6: eight lanes per line instead of four).
// In: lane j < P holds x[j + P r] in v[r], r < Q.  Out: lane l < Q holds X[l + Q k1] in v[k1], k1 < P.
// Stage A is a DFT-Q per lane and the twiddle W_N^{j k2}; stage B a DFT-P over the lanes for k2 = l,
// through the line's LDS area xch (P (Q + 1) float2).  The inverse of a forward (P, Q) transform is
// tline_fft<N, Q, P, true>, which takes the forward's output layout back to its input layout.  Lanes
// outside a stage's range compute on don't-care values and never write the exchange area.
template <int N, int P, int Q, bool INV>
__device__ __forceinline__ void tline_fft(float2 (&v)[(P > Q ? P : Q)], int j, float2* xch, const float2* tw) {
    static_assert(P * Q == N, "N = P Q");
    constexpr int LD = Q + 1;
    const int ja = j < P ? j : 0, jb = j < Q ? j : 0;
    c2 x[Q];
#pragma unroll
    for (int r = 0; r < Q; ++r) x[r] = tc2(v[r]);
    DFT<Q, INV>::run(x);
    c2 t[Q];
#pragma unroll
    for (int k2 = 1; k2 < Q; ++k2) t[k2] = pmul_t(x[k2], tc2(tw[ja * k2]));  // ja k2 < N: no wrap
#pragma unroll
    for (int k2 = 1; k2 < Q; ++k2) x[k2] = pmul_r<INV>(x[k2], tc2(tw[ja * k2]), t[k2]);
    if (j < P) {
#pragma unroll
        for (int k2 = 0; k2 < Q; ++k2) xch[j * LD + k2] = tf2(x[k2]);
    }
    wave_lds_sync();
    c2 z[P];
#pragma unroll
    for (int n1 = 0; n1 < P; ++n1) z[n1] = tc2(xch[n1 * LD + jb]);
    DFT<P, INV>::run(z);
#pragma unroll
    for (int k1 = 0; k1 < P; ++k1) v[k1] = tf2(z[k1]);
    wave_lds_sync();  // the area may be rewritten by the next transform of this wave
}

// Twiddle table W_L^m = exp(-2 pi i m / L), m in [0, L), computed in double, rounded once.
template <int L>
__device__ __forceinline__ void fill_twiddles(float2* tw, int tid, int nthreads) {
    for (int m = tid; m < L; m += nthreads) {
        double s, c;
        sincospi(-2.0 * double(m) / double(L), &s, &c);
        tw[m] = make_float2(float(c), float(s));
    }
}

// Length-L FFT over the F1 lanes of a line.  v[r] = x[j + F1*r] in, X[j + F1*r] out.
// xch: this line's private LDS exchange area (xch_elems<L>() float2); tw: twiddle table.
// Register-only 16 x 16 transpose across the 16 lanes of a line (F1 = F2 = 16): lane j holds v[k]
// = x_j[k] on entry and v[n] = x_n[j] on exit.  The register index a lane needs depends on the lane,
// so the data are rotated by the lane index (four conditional stages of v_cndmask), moved with DPP
// row rotations (uniform register index), and rotated back.  No LDS: for kernels whose LDS is
// occupied by data while they transform.
#ifndef GD_DPP_ROR_DIR
#define GD_DPP_ROR_DIR 1  // row_ror:r delivers lane (j - r) mod 16 to lane j
#endif
template <int R>
__device__ __forceinline__ float dpp_row_ror(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x120 + R, 0xF, 0xF, false));
}
#ifndef GD_DPP_INPLACE
#define GD_DPP_INPLACE 1  // in-place cycle walks (2 spare VGPRs) instead of full 16-element copies
#endif
template <int SGN, int B = 0>
__device__ __forceinline__ void lane_rotate16(float2 (&x)[16], int j) {  // x[k] <- x[(k + SGN j) mod 16]
    if constexpr (B < 4) {  // stage B: rotate by 2^B where bit B of j is set (compile-time indices)
        constexpr int d = 1 << B;
        const bool c = (j >> B) & 1;
#if GD_DPP_INPLACE
        // the rotation by d splits into d cycles of 16/d registers: walk each cycle in place, keeping
        // only its first (overwritten) element aside
        static_for<0, d>([&](auto sc) {
            constexpr int s0 = decltype(sc)::value;
            const float2 first = x[s0];
            static_for<0, 16 / d>([&](auto ic) {
                constexpr int k = (s0 + SGN * d * decltype(ic)::value + 64) & 15;
                constexpr int src = (k + SGN * d + 64) & 15;
                // values made opaque first: a select of two array elements would otherwise be folded
                // into a load from a selected address, i.e. a dynamically indexed array in scratch
                float2 pv = (src == s0) ? first : x[src], q = x[k];
                asm volatile("" : "+v"(pv.x), "+v"(pv.y), "+v"(q.x), "+v"(q.y));
                x[k] = c ? pv : q;
            });
        });
#else
        float2 t[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            float2 p = x[(k + SGN * d) & 15], q = x[k];
            asm volatile("" : "+v"(p.x), "+v"(p.y), "+v"(q.x), "+v"(q.y));
            t[k] = c ? p : q;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = t[k];
#endif
        lane_rotate16<SGN, B + 1>(x, j);
    }
}
// rounds R..15 of the transpose (forceinline recursion, not a lambda: arrays must stay in registers)
template <int R>
__device__ __forceinline__ void dpp_rounds(float2 (&z)[16], const float2 (&v)[16]) {
    if constexpr (R < 16) {
        constexpr int src = GD_DPP_ROR_DIR > 0 ? R : (16 - R) & 15;
        z[R] = make_float2(dpp_row_ror<R>(v[src].x), dpp_row_ror<R>(v[src].y));
        dpp_rounds<R + 1>(z, v);
    }
}
template <int R>
__device__ __forceinline__ void dpp_rounds_inplace(float2 (&v)[16]) {  // v[R] <- row_ror:R of v[R]
    if constexpr (R < 16) {
        v[R] = make_float2(dpp_row_ror<R>(v[R].x), dpp_row_ror<R>(v[R].y));
        dpp_rounds_inplace<R + 1>(v);
    }
}
__device__ __forceinline__ void transpose16_dpp(float2 (&v)[16], int j) {
    // w[c] = v[(c + j) mod 16]: round r then moves, with ONE register index for all lanes, element
    // j of lane j -/+ r (row_ror direction GD_DPP_ROR_DIR = +1 / -1)
    lane_rotate16<1>(v, j);
#if GD_DPP_INPLACE && GD_DPP_ROR_DIR > 0
    // round r in place: v[r] now holds lane j - r's element; want v[n1] = (that of lane n1), i.e.
    // index (j - n1) mod 16 -> a compile-time register renaming v[m] <- v[(16 - m) mod 16]
    dpp_rounds_inplace<1>(v);
#pragma unroll
    for (int m = 1; m < 8; ++m) {
        const float2 t = v[m];
        v[m] = v[16 - m];
        v[16 - m] = t;
    }
#else
    float2 z[16];
    z[0] = v[0];
    dpp_rounds<1>(z, v);
    // z[r] holds lane n1 = j -/+ r; want v[n1] = z[(+/-(j - n1)) mod 16]
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = z[GD_DPP_ROR_DIR > 0 ? (16 - m) & 15 : m];
#endif
    lane_rotate16<-1>(v, j);
}

// LEAN (F2 = 16 only): the 15 twiddles W^{j k1} come from 6 table entries, W^{j (a + 4b)} =
// W^{4jb} W^{ja} (one extra rounding on 9 of them), so a line needs 12 twiddle registers instead
// of 30 - for kernels that run at the 128-VGPR budget of 1024-thread workgroups.
// DPP: register transpose (transpose16_dpp) instead of the LDS exchange (xch unused), F1 = F2 = 16.
template <int L, bool INV, bool LEAN = false, bool DPP = false>
__device__ __forceinline__ void line_fft(float2 (&v)[Plan<L>::F2], int j, float2* xch, const float2* tw) {
    constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2, M = F2 / F1, LD = F2 + 1;
    static_assert(F2 % F1 == 0, "line plan needs F1 | F2");
    static_assert(!LEAN || F2 == 16, "lean twiddles are for 16 points per lane");
    static_assert(!DPP || (F1 == 16 && F2 == 16), "register transpose is for 16 x 16 lines");
    // stage A: DFT-F2 over n2 (lane j = n1), then twiddle W_L^{n1 k1} (the table holds the forward
    // twiddles; the inverse multiplies by their conjugates)
    if constexpr (DPP) {
        DFT<F2, INV>::run(v);
        if constexpr (LEAN) {
            float2 t1[4], t4[4];
#pragma unroll
            for (int i = 1; i < 4; ++i) {
                t1[i] = tw[j * i];
                t4[i] = tw[4 * j * i];
                if (INV) {
                    t1[i].y = -t1[i].y;
                    t4[i].y = -t4[i].y;
                }
            }
#pragma unroll
            for (int k1 = 1; k1 < F2; ++k1) {
                const int a = k1 & 3, b = k1 >> 2;
                const float2 w = a == 0 ? t4[b] : (b == 0 ? t1[a] : cmul(t4[b], t1[a]));
                v[k1] = cmul(v[k1], w);
            }
        } else {
#pragma unroll
            for (int k1 = 1; k1 < F2; ++k1) {
                float2 w = tw[j * k1];
                if (INV) w.y = -w.y;
                v[k1] = cmul(v[k1], w);
            }
        }
        transpose16_dpp(v, j);  // lane j: v[n1] = (element k1 = j of lane n1)
        DFT<F1, INV>::run(v);   // lane j holds X[j + F1 k2] in v[k2]
        return;
    }
    c2 x[F2];
#pragma unroll
    for (int i = 0; i < F2; ++i) x[i] = tc2(v[i]);
    DFT<F2, INV>::run(x);
    c2 w[F2], t[F2];
    if constexpr (LEAN) {
        c2 t1[4], t4[4];
#pragma unroll
        for (int i = 1; i < 4; ++i) {
            t1[i] = tc2(tw[j * i]);
            t4[i] = tc2(tw[4 * j * i]);
        }
        // W^{j (a + 4b)} = W^{4 j b} W^{j a}; the inverse multiplies by conj(t4 t1) = conj t4 conj t1
#pragma unroll
        for (int k1 = 1; k1 < F2; ++k1) {
            const int a = k1 & 3, b = k1 >> 2;
            if (a != 0 && b != 0) t[k1] = pmul_t(t4[b], t1[a]);
        }
#pragma unroll
        for (int k1 = 1; k1 < F2; ++k1) {
            const int a = k1 & 3, b = k1 >> 2;
            w[k1] = a == 0 ? t4[b] : (b == 0 ? t1[a] : pmul_r<false>(t4[b], t1[a], t[k1]));
        }
    } else {
#pragma unroll
        for (int k1 = 1; k1 < F2; ++k1) w[k1] = tc2(tw[j * k1]);  // j*k1 <= (F1-1)(F2-1) < L: no wrap
    }
#pragma unroll
    for (int k1 = 1; k1 < F2; ++k1) t[k1] = pmul_t(x[k1], w[k1]);
#pragma unroll
    for (int k1 = 1; k1 < F2; ++k1) x[k1] = pmul_r<INV>(x[k1], w[k1], t[k1]);
#pragma unroll
    for (int k1 = 0; k1 < F2; ++k1) xch[j * LD + k1] = tf2(x[k1]);
    wave_lds_sync();
    // stage B: lane j takes k1 = j + F1*m, all n1; DFT-F1 over n1
#pragma unroll
    for (int mm = 0; mm < M; ++mm) {
        c2 z[F1];
#pragma unroll
        for (int n1 = 0; n1 < F1; ++n1) z[n1] = tc2(xch[n1 * LD + j + F1 * mm]);
        DFT<F1, INV>::run(z);
#pragma unroll
        for (int k2 = 0; k2 < F1; ++k2) v[mm + M * k2] = tf2(z[k2]);
    }
    wave_lds_sync();  // the area may be rewritten by the next line_fft of this wave
}

// Two independent line FFTs of one line (F1 = F2 = 16), the same arithmetic as two line_fft<L, INV, LEAN> calls
// (bit-identical results) through ONE exchange area, interleaved so that each transform's LDS round trip is
// covered by the other's register work: stage A of v0, its exchange write and read issue; stage A of v1 while
// those reads are in flight; v1's exchange write (LDS requests of a wave are processed in order, so it lands
// after v0's reads); stage B of v0 while v1's reads are in flight; stage B of v1.  The twiddles are formed once.
template <int L, bool INV, bool LEAN = false>
__device__ __forceinline__ void line_fft2(float2 (&v0)[Plan<L>::F2], float2 (&v1)[Plan<L>::F2], int j, float2* xch,
                                          const float2* tw) {
    constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2, LD = F2 + 1;
    static_assert(F1 == 16 && F2 == 16, "paired line FFTs are for 16 x 16 lines");
    c2 w[F2], t[F2];
    if constexpr (LEAN) {
        c2 t1[4], t4[4];
#pragma unroll
        for (int i = 1; i < 4; ++i) {
            t1[i] = tc2(tw[j * i]);
            t4[i] = tc2(tw[4 * j * i]);
        }
#pragma unroll
        for (int k1 = 1; k1 < F2; ++k1) {
            const int a = k1 & 3, b = k1 >> 2;
            if (a != 0 && b != 0) t[k1] = pmul_t(t4[b], t1[a]);
        }
#pragma unroll
        for (int k1 = 1; k1 < F2; ++k1) {
            const int a = k1 & 3, b = k1 >> 2;
            w[k1] = a == 0 ? t4[b] : (b == 0 ? t1[a] : pmul_r<false>(t4[b], t1[a], t[k1]));
        }
    } else {
#pragma unroll
        for (int k1 = 1; k1 < F2; ++k1) w[k1] = tc2(tw[j * k1]);
    }
    auto stage_a = [&](float2 (&v)[F2]) {
        c2 x[F2];
#pragma unroll
        for (int i = 0; i < F2; ++i) x[i] = tc2(v[i]);
        DFT<F2, INV>::run(x);
        c2 u[F2];
#pragma unroll
        for (int k1 = 1; k1 < F2; ++k1) u[k1] = pmul_t(x[k1], w[k1]);
#pragma unroll
        for (int k1 = 1; k1 < F2; ++k1) x[k1] = pmul_r<INV>(x[k1], w[k1], u[k1]);
#pragma unroll
        for (int k1 = 0; k1 < F2; ++k1) v[k1] = tf2(x[k1]);
    };
    auto stage_b = [&](float2 (&v)[F2]) {
        c2 z[F1];
#pragma unroll
        for (int n1 = 0; n1 < F1; ++n1) z[n1] = tc2(v[n1]);
        DFT<F1, INV>::run(z);
#pragma unroll
        for (int k2 = 0; k2 < F1; ++k2) v[k2] = tf2(z[k2]);
    };
    stage_a(v0);
#pragma unroll
    for (int k1 = 0; k1 < F2; ++k1) xch[j * LD + k1] = v0[k1];
    wave_lds_sync();
#pragma unroll
    for (int n1 = 0; n1 < F1; ++n1) v0[n1] = xch[n1 * LD + j];
    stage_a(v1);
    wave_lds_sync();  // (program order: v0's reads before v1's writes to the same area)
#pragma unroll
    for (int k1 = 0; k1 < F2; ++k1) xch[j * LD + k1] = v1[k1];
    wave_lds_sync();
#pragma unroll
    for (int n1 = 0; n1 < F1; ++n1) v1[n1] = xch[n1 * LD + j];
    stage_b(v0);
    stage_b(v1);
    wave_lds_sync();  // the area may be rewritten by the next line_fft of this wave
}

}  // namespace gd
