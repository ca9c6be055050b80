// Register-resident whole-galaxy Gaussian iteration (k_gal_reg<256>).
//
// Same arithmetic, in the same order, as k_gal_iter (row FFTs of packed row pairs, column FFT +
// spectral update + inverse column FFT per slice of 64 columns, inverse row FFTs per half of the rows;
// results agree to rounding - the compiler contracts multiply-adds differently per kernel).  What
// changes is the geometry and where the galaxy waits between phases:
//   * 512 threads per workgroup (two waves per SIMD): a wave owns 256 VGPRs instead of 128;
//   * the column FFTs use register (DPP) transposes, so once a slice has been gathered into the lines'
//     registers the 135 KiB slice area S is free: slice B's row bins wait there during column A, and
//     column A's results during column B.  Nothing round-trips through global memory (k_gal_iter parks
//     2 x 131 KiB per galaxy in the output image: +23 % over the algorithmic 7.5 words per pixel);
//   * the state is read and written with 16-byte accesses in a column order matching the lines'
//     registers (GD_STATE_V4 below), with D groups of 4 bins in flight per wave during the update.
//
//   R  pair p = line + 32 q (q < 4) = rows 2p, 2p+1: z -> 4 packed row FFTs per line (LDS exchange)
//   A  slice A's bins (columns 0..63 and the mirrored bins) -> S; each line gathers columns line and
//      line + 32 (line 0 packs column 0 with the real Nyquist column L/2); slice B's bins -> S; column
//      FFTs, Gaussian update against |H|^2, G, U1, W~ (models/Unrolled_ADMM.py:207-213, DESIGN.md
//      section 2), inverse column FFTs
//   B  slice B's bins S -> registers -> slice layout in S, gather, column A's results -> S, the same
//      per column, column A's results back
//   I  per half of the rows: both slices' results -> S as row half spectra, 2 inverse row FFTs per
//      line, store zin = x + u1 (x on the last iteration)
// Included inside namespace gd by gd_engine.hip (uses its Args, state helpers and FFT lines).

// Values the compiler must materialise here: machine sinking would otherwise move the tail of a row
// FFT (whose outputs phase B consumes) past the phase barriers, into the column phases.
__device__ __forceinline__ void pin4(float2& a, float2& b, float2& c, float2& d) {
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(b.x), "+v"(b.y), "+v"(c.x), "+v"(c.y), "+v"(d.x), "+v"(d.y));
}
template <int N>
__device__ __forceinline__ void pin(float2 (&v)[N]) {
    static_assert(N % 4 == 0, "pin in fours");
#pragma unroll
    for (int i = 0; i < N; i += 4) pin4(v[i], v[i + 1], v[i + 2], v[i + 3]);
}

__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- 16-byte state access.  At 256^2 the Gaussian state's bins inside a column are stored in the
// order the column lines hold them, so a lane's bins are contiguous (gd_engine.hip: sidx_c / sidx_h,
// used by every kernel that touches this state): lane j's bins ky = j + 16 s at 32 (s >> 1) + 2 j +
// (s & 1) (complex arrays; two bins per 16-byte access) and 64 (s >> 2) + 4 j + (s & 3) (|H|^2; four
// bins per access).  Offsets within one galaxy's array, in elements:
__device__ __forceinline__ int soff_c(int kx, int m, int j) { return kx * 256 + 32 * m + 2 * j; }  // bins j + 16 (2m + e)
__device__ __forceinline__ int soff_h(int kx, int q, int j) { return kx * 256 + 64 * q + 4 * j; }  // bins j + 16 (4q + e)
__device__ __forceinline__ f4v ld4v(const void* p) { return *reinterpret_cast<const f4v*>(p); }
__device__ __forceinline__ f4v ld4s(const void* p) { return *reinterpret_cast<const f4v*>(p); }
// state / image stores are single-use per iteration: non-temporal (st_s, gd_engine.hip)
__device__ __forceinline__ void st4v(void* p, f4v v) { __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p)); }

// Poisson pass A's bin (the X update and u1's dual, models/Unrolled_ADMM.py:209, :212, on spectra).  The
// state holds H (the OTF, G slot) and W = F(w), w = v - u2 (written by pass B, unmultiplied), so pass A
// forms W~ = conj(H) W and |H|^2 (the init's arithmetic) itself: X = (rho1 (Z - U1) + rho2 W~) / (rho1
// |H|^2 + rho2), U1' = (U1 + X) - Z; returns (X + U1') / L^2 (next denoiser input) | X / L^2 (last);
// HXo = H X, pass B's only spectral input (pass B reads neither H nor X: one half spectrum less per
// iteration, and no second read of H for its W~)
__device__ __forceinline__ float2 pois_math(float2 Hk, float2 U1, float2 Wf, float2 Zk, float r1, float r2, float inv_n,
                                            float2& U1o, float2& HXo, bool last) {
    const float hh = Hk.x * Hk.x + Hk.y * Hk.y;
    const float2 Wt = cmulc(Wf, Hk);
    const float lhs = r1 * hh + r2;
    const float2 A = csub(Zk, U1);
    const float rl = __builtin_amdgcn_rcpf(lhs);
    const float2 X = make_float2((r1 * A.x + r2 * Wt.x) * rl, (r1 * A.y + r2 * Wt.y) * rl);
    HXo = cmul(Hk, X);
    if (last) return cscale(X, inv_n);
    const float2 U1n = csub(cadd(U1, X), Zk);
    U1o = U1n;
    return cscale(cadd(X, U1n), inv_n);
}

// the Nyquist column, one bin per thread (ky = tid)
template <int L, bool POIS = false>
__device__ __forceinline__ float2 gauss_bin4(const Args& a, int g, int ky, float2 Zk, float r1, float r2, float r2n,
                                             bool first, bool last) {
    constexpr float inv_n = float(1.0 / double(L * L));
    const size_t cb = ((size_t)g * (L / 2 + 1) + L / 2) * L;
    const int pc = sidx_c<L>(ky);
    if constexpr (POIS) {
        const float2 U1 = first ? make_float2(0.f, 0.f) : a.s_u1[cb + pc];
        float2 U1n, HXo;
        const float2 r = pois_math(a.s_g[cb + pc], U1, a.s_w[cb + pc], Zk, r1, r2, inv_n, U1n, HXo, last);
        if (!last) {
            st_s(a.s_u1 + cb + pc, U1n);
            st_s(a.s_x + cb + pc, HXo);
        }
        return r;
    }
    const float hh = a.s_hh[cb + sidx_h<L>(ky)];
    const float2 Gk = (last && !first) ? make_float2(0.f, 0.f) : a.s_g[cb + pc];
    const float2 U1 = first ? make_float2(0.f, 0.f) : a.s_u1[cb + pc];
    float2 Wt = a.s_w[cb + pc];
    if (first) Wt = w1_value(hh, Gk, Wt, r2);  // the slot holds F(x0) (w1_value)
    float2 U1n, Wn;
    const float2 r = gauss_math_rt(hh, Gk, U1, Wt, Zk, r1, r2, r2n, inv_n, U1n, Wn, last);
    if (!last) {
        st_s(a.s_u1 + cb + pc, U1n);
        st_s(a.s_w + cb + pc, Wn);
    }
    return r;
}

// A line's NC columns (C[u]: kx0 + kstep u) as one stream of 4 NC groups of 4 bins, the state loads
// of D groups ahead in flight while a group is computed (memory-level parallelism per wave).
#ifndef GD_REG_DEPTH
#define GD_REG_DEPTH 2
#endif
#ifndef GD_POIS_DEPTH
#define GD_POIS_DEPTH 2  // Poisson pass A
#endif

struct SGroup {
    f4v h, g[2], u[2], w[2];
};
template <int L, bool POIS = false>
__device__ __forceinline__ void sgroup_load(const Args& a, SGroup& G, size_t gb, int kx, int q, int j, bool first,
                                            bool last) {
    G.h = POIS ? f4v{0.f, 0.f, 0.f, 0.f} : ld4s(a.s_hh + gb + soff_h(kx, q, j));  // Poisson: |H|^2 from H
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const size_t off = gb + soff_c(kx, 2 * q + h, j);
        // Gaussian G (first: W~1 needs it; not on the last); Poisson: the OTF H (the G slot)
        G.g[h] = (!POIS && last && !first) ? f4v{0.f, 0.f, 0.f, 0.f} : ld4s(a.s_g + off);
        G.u[h] = first ? f4v{0.f, 0.f, 0.f, 0.f} : ld4s(a.s_u1 + off);
        G.w[h] = ld4s(a.s_w + off);
    }
}
// GD_REG_SPF: the first D groups of a slice's state are loaded BEFORE the slice's forward column FFTs
// (fused_prefetch4x), so their latency runs under the transforms instead of opening the update
#ifndef GD_REG_PAIR
#define GD_REG_PAIR 3  // k_gal_reg (Gaussian): bit 0: a slice's two forward column transforms as an interleaved pair
                       // (reg_fft2), bit 1: the inverse ones
#endif
#ifndef GD_POIS_PAIR
#define GD_POIS_PAIR 0  // GD_REG_PAIR for Poisson pass A as well
#endif
#ifndef GD_POIS_SPF
#define GD_POIS_SPF 1  // the same for Poisson pass A (234 VGPRs with it, 248 without; pass A 1.530 -> 1.508 ms)
#endif
#ifndef GD_REG_SPF
#define GD_REG_SPF 1
#endif
template <int L, int NC, bool POIS = false, int D = GD_REG_DEPTH>
__device__ __forceinline__ void fused_prefetch4x(const Args& a, SGroup (&P)[D], int g, int kx0, int kstep, int j, bool first,
                                                 bool last) {
    j = opaque(j);
    kx0 = opaque(kx0);
    const size_t gb = (size_t)g * (L / 2 + 1) * L;
#pragma unroll
    for (int t = 0; t < D && t < 4 * NC; ++t) sgroup_load<L, POIS>(a, P[t], gb, kx0 + kstep * (t / 4), t % 4, j, first, last);
    __builtin_amdgcn_sched_barrier(0);
}
template <int L, int NC, bool POIS = false, int D = GD_REG_DEPTH, bool PRE = false>
__device__ __forceinline__ void fused_update4x(const Args& a, float2 (&C)[NC][16], int g, int kx0, int kstep, int j,
                                               float r1, float r2, float r2n, bool first, bool last,
                                               const SGroup (*pre)[D] = nullptr) {
    constexpr float inv_n = float(1.0 / double(L * L));
    constexpr int NG = 4 * NC;
    j = opaque(j);
    kx0 = opaque(kx0);
    __builtin_amdgcn_sched_barrier(0);
    const size_t gb = (size_t)g * (L / 2 + 1) * L;
    SGroup G[NG];
#pragma unroll
    for (int t = 0; t < D && t < NG; ++t) {
        if constexpr (PRE) G[t] = (*pre)[t];
        else sgroup_load<L, POIS>(a, G[t], gb, kx0 + kstep * (t / 4), t % 4, j, first, last);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NG; ++t) {
        const int u = t / 4, q = t % 4;
        f4v uo[2], wo[2];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int h = e >> 1, c = 2 * (e & 1);
            float2 U1n, Wn;
            const float2 Gk = make_float2(G[t].g[h][c], G[t].g[h][c + 1]);
            float2 Wt = make_float2(G[t].w[h][c], G[t].w[h][c + 1]);
            if constexpr (POIS) {  // Gk carries H, Wt the unmultiplied F(w), Wn H X (pass B's input)
                C[u][4 * q + e] = pois_math(Gk, make_float2(G[t].u[h][c], G[t].u[h][c + 1]), Wt, C[u][4 * q + e],
                                            r1, r2, inv_n, U1n, Wn, last);
            } else {
                if (first) Wt = w1_value(G[t].h[e], Gk, Wt, r2);  // the slot holds F(x0) (w1_value)
                C[u][4 * q + e] = gauss_math_rt(G[t].h[e], Gk, make_float2(G[t].u[h][c], G[t].u[h][c + 1]), Wt,
                                                C[u][4 * q + e], r1, r2, r2n, inv_n, U1n, Wn, last);
            }
            uo[h][c] = U1n.x; uo[h][c + 1] = U1n.y;
            wo[h][c] = Wn.x; wo[h][c + 1] = Wn.y;
        }
        if (!last) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const size_t off = gb + soff_c(kx0 + kstep * u, 2 * q + h, j);
                st4v(a.s_u1 + off, uo[h]);
                st4v((POIS ? a.s_x : a.s_w) + off, wo[h]);
            }
        }
        if (t + D < NG) sgroup_load<L, POIS>(a, G[t + D], gb, kx0 + kstep * ((t + D) / 4), (t + D) % 4, j, first, last);
        __builtin_amdgcn_sched_barrier(0);
    }
}

#ifndef GD_REG_LEAN
#define GD_REG_LEAN 1  // 1: twiddles W^{j k1} synthesised from 6 table entries; 0: 15 table reads
#endif
template <int L, bool INV, bool DPP = false>
__device__ __forceinline__ void reg_fft(float2 (&v)[16], int j, float2* xch, const float2* tw) {
    line_fft<L, INV, GD_REG_LEAN != 0, DPP>(v, j, xch, tw);
}
// two independent lines' transforms interleaved through one exchange area (line_fft2; bit-identical to two reg_fft)
template <int L, bool INV>
__device__ __forceinline__ void reg_fft2(float2 (&v0)[16], float2 (&v1)[16], int j, float2* xch, const float2* tw) {
    line_fft2<L, INV, GD_REG_LEAN != 0>(v0, v1, j, xch, tw);
}

template <int L>
struct RegGeo {
    static constexpr int F1 = Plan<L>::F1, F2 = Plan<L>::F2, K = L / 2 + 1;
    static constexpr int THREADS = 512, LINES = THREADS / F1;  // 32 lines of 16 lanes
    static constexpr int NP = L / 2, PPL = NP / LINES;          // 128 row pairs, 4 per line
    static constexpr int KS = L / 4, CPL = KS / LINES;          // 64 columns per slice, 2 per line
    // slice layout [pair][SLD] (k_gal_iter's, one slot longer): an odd row stride puts the 16 rows a
    // line writes in phase I (column results -> row half spectra) on 16 distinct bank pairs (SLD = 132
    // put every fourth row on the same banks: 4-way conflicts on those stores)
    static constexpr int SLD = FusedGeo<L>::SLD + 1;
    static constexpr int XCH = xch_elems<L>();
    static constexpr int HPL = (NP / 2) / LINES;                // row pairs per line in a half of phase I
    static constexpr int U = cmax(NP * SLD, LINES * XCH);
    static constexpr int RB0 = KS / F1, RB1 = (L - KS) / F1;    // row registers [RB0, RB1] hold slice B
    // The column transforms use the lines' LDS exchange areas (S[0, LINES XCH)); above them, S holds
    // PK values per thread: slice B's row registers [RB0, RB0 + PXB) of every pair during column A,
    // column A's second column's results during column B.
    static constexpr int XA = LINES * XCH;
    static constexpr int PK = (U - XA) / THREADS;
    static constexpr int PXB = PK / PPL;
    static_assert(F1 == 16 && F2 == 16 && PPL == 4 && CPL == 2 && HPL == 2, "256 x 256 geometry");
    static_assert(SLD >= 2 * KS && SLD > L / 2, "row half spectra fit a slice row");
    static_assert(PK >= F2 && PXB >= 1 && RB0 + PXB <= RB1, "parking area above the exchange areas");
};

// Phase-locking: one galaxy per CU at a time, the same phase durations on every CU, so every launch starts with
// all 256 CUs loading z together (HBM saturated), then transforming together (HBM idle), and the lock decays only
// over ~6 of the launch's 16 rounds (round-5 phase trace of 4096 x 256^2: the first round takes 139 us per galaxy
// against ~100 later; profiles/r05_reg_lockstep.txt).  The first round's workgroups g < 256 therefore start in
// GD_STAGGER_N groups spread over the given microseconds (group g mod N waits (g mod N) / N of it; the z / y loads
// are issued before the wait, so their latency runs during it).  A/B at 4096 x 256^2 (profiles/r05_stagger_ab.txt):
// k_gal_reg MID 1.646-1.650 -> 1.624-1.631 ms, FIRST 1.41 -> 1.39 ms, LAST unchanged; k_gal_reg_init 1.365 -> 1.320-
// 1.337 ms; k_rl_reg unchanged (not applied).
#ifndef GD_REG_STAGGER
#define GD_REG_STAGGER 60  // k_gal_reg: total spread of the first round's start times, microseconds
#endif
#ifndef GD_INIT_STAGGER
#define GD_INIT_STAGGER 60  // k_gal_reg_init
#endif
#ifndef GD_RL_STAGGER
#define GD_RL_STAGGER 0  // k_rl_reg
#endif
#ifndef GD_STAGGER_N
#define GD_STAGGER_N 4  // groups of the first round (group k starts k / N of the spread late)
#endif
// Only when the launch spans more than one round of workgroups (N > 256 galaxies at one per CU): a single round has
// no later rounds to phase-lock, and its staggered groups would only start late.
#ifndef GD_STAGGER_MIN_N
#define GD_STAGGER_MIN_N 256  // launches of at most this many galaxies start unstaggered (0: every launch, round 5)
#endif
template <int US>
__device__ __forceinline__ void stagger_start(int g, int N) {
    if (US > 0 && N > GD_STAGGER_MIN_N && g < 256 && (g % GD_STAGGER_N) != 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long d = (unsigned long long)US * 100 * (g % GD_STAGGER_N) / GD_STAGGER_N;
        while (__builtin_amdgcn_s_memrealtime() - t0 < d) __builtin_amdgcn_s_sleep(32);
    }
}

// First / last iteration as uniform runtime flags (a.first, a.last), not template variants: the MID
// code's register allocation is spill-free, compile-time FIRST / LAST variants spilled 60-100 VGPRs.
// POIS: Poisson pass A (k_gal_reg<L, true>): the same skeleton with pois_math's update (no V step, no G;
// U1', X out) and the last output x * alpha (models/Unrolled_ADMM.py:215)
template <int L, bool POIS = false>
__global__ __launch_bounds__(512) void k_gal_reg(Args a) {
    using RG = RegGeo<L>;
    constexpr int F1 = RG::F1, F2 = RG::F2, KS = RG::KS, SLD = RG::SLD, LINES = RG::LINES, T = RG::THREADS;
    constexpr int RB0 = RG::RB0, RB1 = RG::RB1;
    constexpr float inv_n = float(1.0 / double(L * L));
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 S[RG::U];
    __shared__ float2 nyq[RG::NP];  // X_p[L/2] of every pair
    __shared__ float2 nyqc[L];      // the Nyquist column's spectrum, then its update
    __shared__ float2 nyqx[L];      // line 0's split scratch (S is occupied)
    __shared__ float nyqo[L];       // x(., L/2)
    const int tid = threadIdx.x, line = tid / F1, j = tid - line * F1;
    const int b = blockIdx.x, g = a.rev ? a.N - 1 - b : b;
    const bool l0 = (line == 0);
    float2* my = S + line * RG::XCH;
    fill_twiddles<L>(tw, tid, T);
    const float r1 = a.rho1(g), r2 = a.rho2(g);
    const bool first = __builtin_amdgcn_readfirstlane(a.first) != 0, last = __builtin_amdgcn_readfirstlane(a.last) != 0;
    const float r2n = (POIS || last) ? 0.f : a.rho2n(g);
    const float al = POIS ? a.alpha(g) : 1.f;
    GD_TRACE(0);

    // R
    float2 X[RG::PPL][F2];
    {
        const float* z = a.a0 + (size_t)g * L * L;
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q) {
            // opaque: no 64-bit row offset CSE'd with phase I's stores and kept live in between
            const float* r0 = z + (size_t)(2 * (opaque(line) + LINES * q)) * L + opaque(j);
#pragma unroll
            for (int r = 0; r < F2; ++r) X[q][r] = make_float2(ld_s(r0 + F1 * r), ld_s(r0 + L + F1 * r));
        }
    }
    stagger_start<GD_REG_STAGGER>(b, a.N);  // (z's loads are in flight meanwhile)
    __syncthreads();  // twiddles
    GD_TRACE(1);
#pragma unroll
    for (int q = 0; q < RG::PPL; ++q) {
        reg_fft<L, false>(X[q], opaque(j), my, tw);
        pin(X[q]);
        __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();  // exchange areas -> slice A
    GD_TRACE(2);

    // A: bins of columns 0..KS-1 and the Nyquist bins (k_gal_iter's slice layout)
#pragma unroll
    for (int q = 0; q < RG::PPL; ++q) {
        const int p = opaque(line) + LINES * q, jq = opaque(j);
        float2* row = S + p * SLD;
#pragma unroll
        for (int r = 0; r < F2; ++r) {
            const int k = jq + F1 * r;
            if (r < KS / F1) row[k] = X[q][r];                               // X_p[kx], kx = k
            if (r == 0 && jq == 0) row[KS] = X[q][r];                         // X_p[L - 0]
            if (r == L / 2 / F1 && jq == 0) nyq[p] = X[q][r];                 // X_p[L/2]
            if (r > (L - KS) / F1 || (r == (L - KS) / F1 && jq > 0)) row[KS + L - k] = X[q][r];  // X_p[L - kx]
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();
    float2 CA[RG::CPL][F2];  // columns line, line + LINES of slice A; later their results
#pragma unroll
    for (int u = 0; u < RG::CPL; ++u) fused_gather<L, SLD>(S, line + LINES * u, j, CA[u]);
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        const int y = j + F1 * s;
        const float2 w = nyq[y >> 1];
        if (l0) CA[0][s].y = (y & 1) ? w.y : w.x;  // line 0: column 0 + i column L/2
    }
    lds_barrier();  // slice A read -> exchange areas + parked slice B bins
    // slice B's row registers r in [RB0, RB0 + PXB) wait in S above the exchange areas (thread-contiguous)
    float2* park = S + RG::XA;
#pragma unroll
    for (int q = 0; q < RG::PPL; ++q)
#pragma unroll
        for (int r = RB0; r < RB0 + RG::PXB; ++r) park[(q * RG::PXB + r - RB0) * T + tid] = X[q][r];
    __builtin_amdgcn_sched_barrier(0);
    GD_TRACE(3);
    constexpr int DPT = POIS ? GD_POIS_DEPTH : GD_REG_DEPTH;
    constexpr bool SPF = GD_REG_SPF && (!POIS || GD_POIS_SPF);
    SGroup preA[DPT];
    if constexpr (SPF) fused_prefetch4x<L, RG::CPL, POIS, DPT>(a, preA, g, line, LINES, j, first, last);
    if constexpr ((GD_REG_PAIR & 1) != 0 && (!POIS || GD_POIS_PAIR)) {
        reg_fft2<L, false>(CA[0], CA[1], opaque(j), my, tw);
        __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
        for (int u = 0; u < RG::CPL; ++u) {
            reg_fft<L, false>(CA[u], opaque(j), my, tw);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (l0) {
#pragma unroll
        for (int s = 0; s < F2; ++s) nyqx[j + F1 * s] = CA[0][s];
        wave_lds_sync();
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            const int ky = j + F1 * s;
            const float2 z = CA[0][s], zm = nyqx[(L - ky) & (L - 1)];
            nyqc[ky] = make_float2(0.5f * (z.y + zm.y), 0.5f * (zm.x - z.x));
            CA[0][s] = make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
        }
    }
    lds_barrier();  // nyqc complete
    if (__builtin_amdgcn_readfirstlane(tid >> 6) < L / 64) {
        nyqc[tid] = gauss_bin4<L, POIS>(a, g, tid, nyqc[tid], r1, r2, r2n, first, last);
    }
    fused_update4x<L, RG::CPL, POIS, DPT, SPF>(a, CA, g, line, LINES, j, r1, r2, r2n, first, last, &preA);
    lds_barrier();  // Nyquist results
    GD_TRACE(4);
#pragma unroll
    for (int s = 0; s < F2; ++s) {
        const float2 cn = nyqc[j + F1 * s];
        if (l0) CA[0][s] = make_float2(CA[0][s].x - cn.y, CA[0][s].y + cn.x);
    }
    if constexpr ((GD_REG_PAIR & 2) != 0 && (!POIS || GD_POIS_PAIR)) {
        reg_fft2<L, true>(CA[0], CA[1], opaque(j), my, tw);
        __builtin_amdgcn_sched_barrier(0);
    } else
#pragma unroll
    for (int u = 0; u < RG::CPL; ++u) {
        reg_fft<L, true>(CA[u], opaque(j), my, tw);
        if (POIS) pin(CA[u]);  // Poisson pass A: spill-free with the inverses pinned
        __builtin_amdgcn_sched_barrier(0);
    }
    if (l0) {
#pragma unroll
        for (int s = 0; s < F2; ++s) nyqo[j + F1 * s] = CA[0][s].y;
    }
    // slice B's parked bins back (each thread its own: no barrier before), then the slice layout
#pragma unroll
    for (int q = 0; q < RG::PPL; ++q)
#pragma unroll
        for (int r = RB0; r < RB0 + RG::PXB; ++r) X[q][r] = park[(q * RG::PXB + r - RB0) * T + opaque(tid)];
    lds_barrier();  // parked bins read -> slice B
    GD_TRACE(5);

    // B: columns KS..2KS-1
#pragma unroll
    for (int q = 0; q < RG::PPL; ++q) {
        const int jq = opaque(j);
        float2* row = S + (opaque(line) + LINES * q) * SLD;
#pragma unroll
        for (int r = RB0; r <= RB1; ++r) {
            const int k = jq + F1 * r;
            if (r < 2 * KS / F1) row[k - KS] = X[q][r];                       // X_p[kx], kx = k
            if (r > L / 2 / F1 || (r == L / 2 / F1 && jq > 0)) {
                if (r < RB1 || jq == 0) row[L - k] = X[q][r];                 // X_p[L - kx] at KS + (kx - KS)
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();
    float2 CB[RG::CPL][F2];
#pragma unroll
    for (int u = 0; u < RG::CPL; ++u) fused_gather<L, SLD>(S, line + LINES * u, j, CB[u]);
    lds_barrier();  // slice B read -> exchange areas + parked column A results (second column)
#pragma unroll
    for (int s = 0; s < F2; ++s) park[s * T + tid] = CA[RG::CPL - 1][s];
    __builtin_amdgcn_sched_barrier(0);
    GD_TRACE(6);
    SGroup preB[DPT];
    if constexpr (SPF) fused_prefetch4x<L, RG::CPL, POIS, DPT>(a, preB, g, KS + line, LINES, j, first, last);
    if constexpr ((GD_REG_PAIR & 1) != 0 && (!POIS || GD_POIS_PAIR)) {
        reg_fft2<L, false>(CB[0], CB[1], opaque(j), my, tw);
        __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
        for (int u = 0; u < RG::CPL; ++u) {
            reg_fft<L, false>(CB[u], opaque(j), my, tw);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    fused_update4x<L, RG::CPL, POIS, DPT, SPF>(a, CB, g, KS + line, LINES, j, r1, r2, r2n, first, last, &preB);
    if constexpr ((GD_REG_PAIR & 2) != 0 && (!POIS || GD_POIS_PAIR)) {
        reg_fft2<L, true>(CB[0], CB[1], opaque(j), my, tw);
        __builtin_amdgcn_sched_barrier(0);
    } else
#pragma unroll
    for (int u = 0; u < RG::CPL; ++u) {
        reg_fft<L, true>(CB[u], opaque(j), my, tw);
        if (POIS) pin(CB[u]);
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int s = 0; s < F2; ++s) CA[RG::CPL - 1][s] = park[s * T + opaque(tid)];

    // I: half hf = rows [hf L/2, (hf+1) L/2): both slices' results -> S as row half spectra [yl][SLD]
    // (bins 0..L/2), inverse FFTs of the packed row pairs m = line + LINES w, store
    float* out = a.o0 + (size_t)g * L * L;
    static_for<0, 2>([&](auto hfc) {
        constexpr int hf = decltype(hfc)::value;
        lds_barrier();  // parked results / exchange areas -> row half spectra
        GD_TRACE(7 + hf);
#pragma unroll
        for (int s = hf * F2 / 2; s < (hf + 1) * F2 / 2; ++s) {
            float2* rr = S + (j + F1 * s - hf * L / 2) * SLD;
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) {
                const float2 c = CA[u][s];
                rr[line + LINES * u] = (u == 0 && l0) ? make_float2(c.x, 0.f) : c;  // column 0: real part
                rr[KS + line + LINES * u] = CB[u][s];
            }
        }
        for (int i = tid; i < L / 2; i += T) S[i * SLD + L / 2] = make_float2(nyqo[hf * L / 2 + i], 0.f);
        lds_barrier();
        float2 V[RG::HPL][F2];
#pragma unroll
        for (int w = 0; w < RG::HPL; ++w) {
            const int jj = opaque(j);
            const float2* re = S + (2 * (opaque(line) + LINES * w)) * SLD;
            const float2* ro = re + SLD;
#pragma unroll
            for (int r = 0; r < F2; ++r) {
                const int k = jj + F1 * r;
                float2 be, bo;
                if (k <= L / 2) {
                    be = re[k];
                    bo = ro[k];
                } else {
                    be = cconj(re[L - k]);
                    bo = cconj(ro[L - k]);
                }
                V[w][r] = make_float2(be.x - bo.y, be.y + bo.x);
            }
        }
        lds_barrier();  // row half spectra -> exchange areas
#pragma unroll
        for (int w = 0; w < RG::HPL; ++w) {
            reg_fft<L, true>(V[w], opaque(j), my, tw);
            // (the row pointer ahead of Poisson's scaling: formed after it, pass A spilled 4 VGPRs)
            float* o = out + (size_t)(hf * L / 2 + 2 * (opaque(line) + LINES * w)) * L + opaque(j);
            if constexpr (POIS) {
                if (last) {  // x * alpha for Poisson (:215)
#pragma unroll
                    for (int r = 0; r < F2; ++r) V[w][r] = make_float2(V[w][r].x * al, V[w][r].y * al);
                }
            }
#pragma unroll
            for (int r = 0; r < F2; ++r) {
                st_s(o + F1 * r, V[w][r].x);
                st_s(o + L + F1 * r, V[w][r].y);
            }
        }
    });
    drain_vm();  // the stores drain before the workgroup ends (measured free, r05: kept)
    __syncthreads();
    GD_TRACE(9);
}

// ==================================================================== fused Gaussian init at 256^2
// k_gal_reg_init: init_l2 (models/Unrolled_ADMM.py:170-175) and iteration 0's W~ (the first V step,
// :335-336, premultiplied by conj(H)) in ONE launch on k_gal_reg's skeleton, one 512-thread workgroup
// per galaxy (the arithmetic of k_col<C_G_INIT>, RIF_CLAMP and k_col<C_G_W1>, bin for bin):
//   R  max(y, 0) / alpha -> 4 packed row FFTs per line
//   A  per column of slice A: Y's column FFT; the OTF column from the PSF's compact row spectra
//      (k_psf_rows<L, true> left them in the U1 slot) and its FFT; |H|^2, G = conj(H) Y -> state,
//      X0 = G / (|H|^2 + 1/alpha); inverse column FFT
//   B  the same for slice B
//   I  per half of the rows: row IFFTs, x0 = clamp(., 0, 1) -> zin, and the clamped rows' FFTs again
//   W  F(x0)'s columns (slice A, slice B) -> the W~ slot; iteration 0 forms W~1 = (rho2 |H|^2 F(x0) +
//      G) / (1 + rho2) from it (w1_value: |H|^2 and G are not re-read here, no rho is read)
// Bytes per galaxy: y, zin (2 img) + |H|^2, G, F(x0) (2.5 half) + the PSF's compact rows (h (L/2 + 1)
// complex).  No parking, 16-byte state accesses.

// One column of the init (NC = 1 per call): |H|^2, G -> state; C <- X0 / L^2
template <int L, bool POIS = false>
__device__ __forceinline__ void init_update4(const Args& a, float2 (&C)[16], const float2 (&Hc)[16], int g, int kx,
                                             int j, float ial) {
    constexpr float inv_n = float(1.0 / double(L * L));
    j = opaque(j);
    kx = opaque(kx);
    __builtin_amdgcn_sched_barrier(0);
    const size_t gb = (size_t)g * (L / 2 + 1) * L;
    if constexpr (POIS) {  // Poisson two-pass: the OTF itself in the G slot (pass B needs H), stored first
#pragma unroll
        for (int m = 0; m < 8; ++m)
            *reinterpret_cast<f4v*>(a.s_g + gb + soff_c(kx, m, j)) =
                f4v{Hc[2 * m].x, Hc[2 * m].y, Hc[2 * m + 1].x, Hc[2 * m + 1].y};
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        f4v h4, g4[2];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int s = 4 * q + e, h = e >> 1, c = 2 * (e & 1);
            const float2 Hk = Hc[s];
            const float hh = Hk.x * Hk.x + Hk.y * Hk.y;  // init_bin's arithmetic
            const float2 Gk = cmulc(C[s], Hk);
            h4[e] = hh;
            g4[h][c] = Gk.x;
            g4[h][c + 1] = Gk.y;
            const float rl = __builtin_amdgcn_rcpf(hh + ial);  // lhs = HtH + 1/alpha; one reciprocal (1 ulp), not two divisions
            C[s] = cscale(make_float2(Gk.x * rl, Gk.y * rl), inv_n);
        }
        if constexpr (!POIS) {  // (Poisson: pass A derives |H|^2 from H)
            *reinterpret_cast<f4v*>(a.s_hh + gb + soff_h(kx, q, j)) = h4;
#pragma unroll
            for (int h = 0; h < 2; ++h) *reinterpret_cast<f4v*>(a.s_g + gb + soff_c(kx, 2 * q + h, j)) = g4[h];
        }
    }
}
// One column of F(x0) (C) into the W~ slot: iteration 0 forms W~1 from it (w1_value)
// POIS: H F(x0) instead (pass B<INIT>'s input, as pass A leaves H X for pass B); H is the G slot this
// thread wrote for the same column in the init's column pass
template <int L, bool POIS = false>
__device__ __forceinline__ void w1_update4(const Args& a, const float2 (&C)[16], int g, int kx, int j) {
    j = opaque(j);
    kx = opaque(kx);
    __builtin_amdgcn_sched_barrier(0);
    const size_t gb = (size_t)g * (L / 2 + 1) * L;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        float2 c0 = C[2 * m], c1 = C[2 * m + 1];
        if constexpr (POIS) {
            const f4v h = ld4v(a.s_g + gb + soff_c(kx, m, j));
            c0 = cmul(make_float2(h[0], h[1]), c0);
            c1 = cmul(make_float2(h[2], h[3]), c1);
        }
        st4v(a.s_w + gb + soff_c(kx, m, j), f4v{c0.x, c0.y, c1.x, c1.y});
    }
}
// The OTF column kx (FFT'd, LDS exchange) from the PSF's compact row spectra; line 0 (kx = 0, packed
// with the real Nyquist column) splits it and leaves the Nyquist column's spectrum in nyqh.
#ifndef GD_INIT_HPF
#define GD_INIT_HPF 1  // 1: a slice's OTF row values are loaded before its data columns' forward FFTs
#endif
template <int L>
__device__ __forceinline__ void init_otf_column(const Args& a, float2 (&Hc)[16], int g, int kx, int j, bool l0,
                                                float2* my, const float2* tw, float2* nyqh,
                                                const float2 (*h4)[4] = nullptr) {
    if (h4)
        init_hcol<L>(Hc, *h4);
    else
        init_hload<L>(a, Hc, g, kx, j);
    reg_fft<L, false>(Hc, opaque(j), my, tw);
    if (l0) {
#pragma unroll
        for (int s = 0; s < 16; ++s) my[j + 16 * s] = Hc[s];
        wave_lds_sync();
        float2 zm[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) zm[s] = my[(L - j - 16 * s) & (L - 1)];
        wave_lds_sync();
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const float2 z = Hc[s];
            nyqh[j + 16 * s] = make_float2(0.5f * (z.y + zm[s].y), 0.5f * (zm[s].x - z.x));
            Hc[s] = make_float2(0.5f * (z.x + zm[s].x), 0.5f * (z.y - zm[s].y));
        }
    }
}

#ifndef GD_INIT_DPP
#define GD_INIT_DPP 0  // 1: the init's line FFTs transpose in registers (DPP) instead of through the LDS exchange
#endif
#ifndef GD_INIT_PAIR
#define GD_INIT_PAIR 1  // bit 0: a slice's two data columns transformed as an interleaved pair (reg_fft2), bit 1: the
                        // phase I rows
#endif
// POIS: the Poisson two-pass init (k_gal_reg_init<L, true>): the same init_l2 and F(x0), but the OTF
// itself goes to the G slot (the Poisson V step reads y, not G); pass B then forms w1 and W~1.
template <int L, bool POIS = false>
__global__ __launch_bounds__(512) void k_gal_reg_init(Args a) {
    using RG = RegGeo<L>;
    constexpr int F1 = RG::F1, F2 = RG::F2, KS = RG::KS, SLD = RG::SLD, LINES = RG::LINES, T = RG::THREADS;
    constexpr int RB0 = RG::RB0, RB1 = RG::RB1;
    constexpr float inv_n = float(1.0 / double(L * L));
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 S[RG::U];
    __shared__ float2 nyq[RG::NP];  // X_p[L/2] of every pair
    __shared__ float2 nyqc[L];      // the Nyquist column's spectrum, then its update
    __shared__ float2 nyqh[L];      // the OTF's Nyquist column
    __shared__ float nyqo[L];       // x(., L/2)
    const int tid = threadIdx.x, line = tid / F1, j = tid - line * F1;
    const int g = blockIdx.x;
    const bool l0 = (line == 0);
    float2* my = S + line * RG::XCH;
    float2* park = S + RG::XA;
    fill_twiddles<L>(tw, tid, T);
    const float al = a.alpha(g);  // no rho: iteration 0 forms W~1 (Poisson: pass B<INIT> takes the V step)
    GD_TRACE(0);

    // R: max(y, 0) / alpha (RF_YA), as a multiply by the galaxy's 1/alpha (within an ulp of the division;
    // 128 IEEE divisions per lane were a third of this phase)
    const float ial = 1.0f / al;
    float2 X[RG::PPL][F2];
    {
        const float* y = a.y + (size_t)g * L * L;
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q) {
            const float* r0 = y + (size_t)(2 * (opaque(line) + LINES * q)) * L + opaque(j);
#pragma unroll
            for (int r = 0; r < F2; ++r) X[q][r] = make_float2(fmaxf(r0[F1 * r], 0.f) * ial, fmaxf(r0[L + F1 * r], 0.f) * ial);
        }
    }
    stagger_start<GD_INIT_STAGGER>(g, a.N);
    __syncthreads();  // twiddles
    GD_TRACE(1);
#pragma unroll
    for (int q = 0; q < RG::PPL; ++q) {
        reg_fft<L, false, GD_INIT_DPP != 0>(X[q], opaque(j), my, tw);
        pin(X[q]);
        __builtin_amdgcn_sched_barrier(0);
    }

    float2 CA[RG::CPL][F2], CB[RG::CPL][F2];
    // forward columns of the row spectra X: slice A into CA (and nyqc), slice B into CB
    // (phase_cols is shared with the W~ pass below; INIT: the X0 columns' update and inverse)
    auto slices = [&](auto initc) {
        constexpr bool INIT = decltype(initc)::value;
        constexpr int TB = INIT ? 2 : 9;  // trace stamp base
        lds_barrier();  // exchange areas -> slice A
        GD_TRACE(TB);
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q) {
            const int p = opaque(line) + LINES * q, jq = opaque(j);
            float2* row = S + p * SLD;
#pragma unroll
            for (int r = 0; r < F2; ++r) {
                const int k = jq + F1 * r;
                if (r < KS / F1) row[k] = X[q][r];
                if (r == 0 && jq == 0) row[KS] = X[q][r];
                if (r == L / 2 / F1 && jq == 0) nyq[p] = X[q][r];
                if (r > (L - KS) / F1 || (r == (L - KS) / F1 && jq > 0)) row[KS + L - k] = X[q][r];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        lds_barrier();
#pragma unroll
        for (int u = 0; u < RG::CPL; ++u) fused_gather<L, SLD>(S, line + LINES * u, j, CA[u]);
#pragma unroll
        for (int s = 0; s < F2; ++s) {
            const int y = j + F1 * s;
            const float2 w = nyq[y >> 1];
            if (l0) CA[0][s].y = (y & 1) ? w.y : w.x;
        }
        lds_barrier();  // slice A read -> exchange areas + parked slice B bins
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q)
#pragma unroll
            for (int r = RB0; r < RB0 + RG::PXB; ++r) park[(q * RG::PXB + r - RB0) * T + tid] = X[q][r];
        __builtin_amdgcn_sched_barrier(0);
        GD_TRACE(TB + 1);
        float2 hpA[RG::CPL][4];  // INIT: slice A's OTF row values, in flight during the data columns' FFTs
        if constexpr (INIT && GD_INIT_HPF && !POIS) {  // (the Poisson init spills with them)
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) init_hload4<L>(a, hpA[u], g, line + LINES * u, j);
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr ((GD_INIT_PAIR & 1) != 0 && !POIS) {  // (the Poisson init spills with it)
            reg_fft2<L, false>(CA[0], CA[1], opaque(j), my, tw);
            if (POIS) {
                pin(CA[0]);
                pin(CA[1]);
            }
            __builtin_amdgcn_sched_barrier(0);
        } else {
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) {
                reg_fft<L, false, GD_INIT_DPP != 0>(CA[u], opaque(j), my, tw);
                if (POIS) pin(CA[u]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (l0) {  // column 0 / Nyquist column split (the exchange area is free: the FFTs are done)
#pragma unroll
            for (int s = 0; s < F2; ++s) my[j + F1 * s] = CA[0][s];
            wave_lds_sync();
#pragma unroll
            for (int s = 0; s < F2; ++s) {
                const int ky = j + F1 * s;
                const float2 z = CA[0][s], zm = my[(L - ky) & (L - 1)];
                nyqc[ky] = make_float2(0.5f * (z.y + zm.y), 0.5f * (zm.x - z.x));
                CA[0][s] = make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
            }
            wave_lds_sync();
        }
        if constexpr (INIT) {
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) {
                float2 Hc[F2];
                init_otf_column<L>(a, Hc, g, line + LINES * u, j, l0 && u == 0, my, tw, nyqh,
                                   (GD_INIT_HPF && !POIS) ? &hpA[u] : nullptr);
                init_update4<L, POIS>(a, CA[u], Hc, g, line + LINES * u, j, ial);
                __builtin_amdgcn_sched_barrier(0);
            }
            lds_barrier();  // nyqc, nyqh complete
            if (__builtin_amdgcn_readfirstlane(tid >> 6) < L / 64)
                nyqc[tid] = init_bin<L>(a, ((size_t)g * RG::K + L / 2) * L + tid, nyqc[tid], nyqh[tid], al, inv_n, POIS);
            lds_barrier();  // Nyquist results
#pragma unroll
            for (int s = 0; s < F2; ++s) {
                const float2 cn = nyqc[j + F1 * s];
                if (l0) CA[0][s] = make_float2(CA[0][s].x - cn.y, CA[0][s].y + cn.x);
            }
            if constexpr ((GD_INIT_PAIR & 1) != 0 && !POIS) {  // (the Poisson init spills with it)
                reg_fft2<L, true>(CA[0], CA[1], opaque(j), my, tw);
                if (POIS) {
                    pin(CA[0]);
                    pin(CA[1]);
                }
                __builtin_amdgcn_sched_barrier(0);
            } else {
#pragma unroll
                for (int u = 0; u < RG::CPL; ++u) {
                    reg_fft<L, true, GD_INIT_DPP != 0>(CA[u], opaque(j), my, tw);
                    if (POIS) pin(CA[u]);  // the Poisson init: materialised here, spill-free
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (l0) {
#pragma unroll
                for (int s = 0; s < F2; ++s) nyqo[j + F1 * s] = CA[0][s].y;
            }
        } else {
            lds_barrier();  // nyqc complete
            if (__builtin_amdgcn_readfirstlane(tid >> 6) < L / 64)
                w1_bin<L>(a, ((size_t)g * RG::K + L / 2) * L + tid, nyqc[tid]);
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) w1_update4<L, POIS>(a, CA[u], g, line + LINES * u, j);
        }
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q)
#pragma unroll
            for (int r = RB0; r < RB0 + RG::PXB; ++r) X[q][r] = park[(q * RG::PXB + r - RB0) * T + opaque(tid)];
        lds_barrier();  // parked bins read -> slice B
        GD_TRACE(TB + 2);
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q) {
            const int jq = opaque(j);
            float2* row = S + (opaque(line) + LINES * q) * SLD;
#pragma unroll
            for (int r = RB0; r <= RB1; ++r) {
                const int k = jq + F1 * r;
                if (r < 2 * KS / F1) row[k - KS] = X[q][r];
                if (r > L / 2 / F1 || (r == L / 2 / F1 && jq > 0)) {
                    if (r < RB1 || jq == 0) row[L - k] = X[q][r];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        lds_barrier();
#pragma unroll
        for (int u = 0; u < RG::CPL; ++u) fused_gather<L, SLD>(S, line + LINES * u, j, CB[u]);
        lds_barrier();  // slice B read -> exchange areas (+ parked column A results)
        GD_TRACE(TB + 3);
        if constexpr (INIT) {
#pragma unroll
            for (int s = 0; s < F2; ++s) park[s * T + tid] = CA[RG::CPL - 1][s];
        }
        __builtin_amdgcn_sched_barrier(0);
        float2 hpB[RG::CPL][4];  // INIT: slice B's OTF row values, in flight during the data columns' FFTs
        if constexpr (INIT && GD_INIT_HPF && !POIS) {  // (the Poisson init spills with them)
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) init_hload4<L>(a, hpB[u], g, KS + line + LINES * u, j);
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr ((GD_INIT_PAIR & 1) != 0 && !POIS) {  // (the Poisson init spills with it)
            reg_fft2<L, false>(CB[0], CB[1], opaque(j), my, tw);
            __builtin_amdgcn_sched_barrier(0);
        } else {
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) {
                reg_fft<L, false, GD_INIT_DPP != 0>(CB[u], opaque(j), my, tw);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int u = 0; u < RG::CPL; ++u) {
            if constexpr (INIT) {
                float2 Hc[F2];
                init_otf_column<L>(a, Hc, g, KS + line + LINES * u, j, false, my, tw, nyqh,
                                   (GD_INIT_HPF && !POIS) ? &hpB[u] : nullptr);
                init_update4<L, POIS>(a, CB[u], Hc, g, KS + line + LINES * u, j, ial);
                reg_fft<L, true, GD_INIT_DPP != 0>(CB[u], opaque(j), my, tw);
                if (POIS) pin(CB[u]);
            } else {
                w1_update4<L, POIS>(a, CB[u], g, KS + line + LINES * u, j);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (INIT) {
#pragma unroll
            for (int s = 0; s < F2; ++s) CA[RG::CPL - 1][s] = park[s * T + opaque(tid)];
        }
    };
    slices(std::true_type{});

    // I: per half, row IFFTs -> x0 = clamp(., 0, 1) -> zin, then the clamped rows' FFTs (W~'s input);
    // pair m = line + LINES w of half hf is row pair p = 64 hf + m of the W~ pass (X[2 hf + w])
    float* out = a.o2 + (size_t)g * L * L;
    static_for<0, 2>([&](auto hfc) {
        constexpr int hf = decltype(hfc)::value;
        lds_barrier();  // parked results / exchange areas -> row half spectra
        GD_TRACE(6 + hf);
#pragma unroll
        for (int s = hf * F2 / 2; s < (hf + 1) * F2 / 2; ++s) {
            float2* rr = S + (j + F1 * s - hf * L / 2) * SLD;
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) {
                const float2 c = CA[u][s];
                rr[line + LINES * u] = (u == 0 && l0) ? make_float2(c.x, 0.f) : c;
                rr[KS + line + LINES * u] = CB[u][s];
            }
        }
        for (int i = tid; i < L / 2; i += T) S[i * SLD + L / 2] = make_float2(nyqo[hf * L / 2 + i], 0.f);
        lds_barrier();
#pragma unroll
        for (int w = 0; w < RG::HPL; ++w) {
            float2 (&V)[F2] = X[2 * hf + w];
            const int jj = opaque(j);
            const float2* re = S + (2 * (opaque(line) + LINES * w)) * SLD;
            const float2* ro = re + SLD;
#pragma unroll
            for (int r = 0; r < F2; ++r) {
                const int k = jj + F1 * r;
                float2 be, bo;
                if (k <= L / 2) {
                    be = re[k];
                    bo = ro[k];
                } else {
                    be = cconj(re[L - k]);
                    bo = cconj(ro[L - k]);
                }
                V[r] = make_float2(be.x - bo.y, be.y + bo.x);
            }
        }
        lds_barrier();  // row half spectra -> exchange areas
        auto clamp_store = [&](float2 (&V)[F2], int w) {
            float* o = out + (size_t)(hf * L / 2 + 2 * (opaque(line) + LINES * w)) * L + opaque(j);
#pragma unroll
            for (int r = 0; r < F2; ++r) {  // x0 = torch.clamp(x0, 0, 1) (RIF_CLAMP)
                V[r] = make_float2(fminf(fmaxf(V[r].x, 0.f), 1.f), fminf(fmaxf(V[r].y, 0.f), 1.f));
                o[F1 * r] = V[r].x;
                o[L + F1 * r] = V[r].y;
            }
        };
        if constexpr ((GD_INIT_PAIR & 2) != 0) {
            static_assert(RG::HPL == 2, "two row pairs per line and half");
            reg_fft2<L, true>(X[2 * hf], X[2 * hf + 1], opaque(j), my, tw);
            clamp_store(X[2 * hf], 0);
            clamp_store(X[2 * hf + 1], 1);
            reg_fft2<L, false>(X[2 * hf], X[2 * hf + 1], opaque(j), my, tw);  // F(x0) rows
            pin(X[2 * hf]);
            pin(X[2 * hf + 1]);
            __builtin_amdgcn_sched_barrier(0);
        } else {
#pragma unroll
            for (int w = 0; w < RG::HPL; ++w) {
                float2 (&V)[F2] = X[2 * hf + w];
                reg_fft<L, true, GD_INIT_DPP != 0>(V, opaque(j), my, tw);
                clamp_store(V, w);
                reg_fft<L, false, GD_INIT_DPP != 0>(V, opaque(j), my, tw);  // F(x0) rows
                pin(V);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    });

    // W: F(x0)'s columns -> W~ (no inverse)
    GD_TRACE(8);
    slices(std::false_type{});
    drain_vm();  // the stores drain before the workgroup ends (measured free, r05: kept)
    __syncthreads();
    GD_TRACE(13);
}
