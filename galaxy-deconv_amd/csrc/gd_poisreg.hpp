// Poisson ADMM at 256^2 in two whole-galaxy passes per iteration (models/Unrolled_ADMM.py:199-215 with
// V_Update_Poisson :326-328).  The Poisson V step (sqrt) keeps v, hence w = v - u2, in the image domain,
// so an iteration needs the spectra of two images and two inverse transforms: more than one CU holds
// at once.  Split where the data are smallest:
//   pass A  k_gal_reg<L, true> (gd_galreg.hpp): z -> Z;  W~ = conj(H) W;  X = (rho1 (Z - U1) + rho2 W~) /
//           (rho1 |H|^2 + rho2);  U1' = (U1 + X) - Z;  zin = F^-1(X + U1')  (last: x alpha);  H X -> the X slot
//   pass B  k_pois_b<L> (here): H X -> Hx (column then row inverses);  u2 = Hx - w;
//           v' = V(Hx + u2, y, rho2', alpha);  w' = v' - u2 -> out;  W' = F(w') -> state
// with U1 = F(u1) and W = F(w) kept as spectra (the linear steps :209, :212 on spectra, as the Gaussian
// engine does).  H (the OTF) is read once per iteration, by pass A, which multiplies W by conj(H) and X by
// H: pass B's only spectral input is H X and its only spectral output F(w').  Compulsory bytes per galaxy
// and iteration: pass A 2 img + 5 half, pass B 3 img + 2 half, against 10 img + 7 half through the
// workspace for the three-kernel chain (and 5 img + 8.5 half when pass B read H and X, and H twice).
// State at 256^2: [(|H|^2, unused) | H (the G slot) | U1 | W | H X] + w (image).
// The init (INIT = 1): k_gal_reg_init<L, true> leaves the OTF in the G slot and H F(x0) in the W slot;
// pass B with H X := H F(x0) and u2 = 0 forms w1 = v1 = V(H x0) and W1 = F(w1) (RI_INIT's arithmetic).
// Included inside namespace gd by gd_engine.hip (after gd_galreg.hpp).

#ifndef GD_POIS_PC
#define GD_POIS_PC 8  // pixels per row loaded together in pass B's V step
#endif
template <int L>
__global__ __launch_bounds__(512) void k_pois_b(Args a, int init_flag) {
    using RG = RegGeo<L>;
    constexpr int F1 = RG::F1, F2 = RG::F2, KS = RG::KS, SLD = RG::SLD, LINES = RG::LINES, T = RG::THREADS;
    constexpr int RB0 = RG::RB0, RB1 = RG::RB1, K = RG::K;
    constexpr float inv_n = float(1.0 / double(L * L));
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 S[RG::U];
    __shared__ float2 nyq[RG::NP];  // X_p[L/2] of every pair (W pass)
    __shared__ float2 nyqc[L];      // the Nyquist column's spectrum
    __shared__ float nyqo[L];       // Hx(., L/2)
    const int tid = threadIdx.x, line = tid / F1, j = tid - line * F1;
    const int g = blockIdx.x;
    const bool l0 = (line == 0);
    float2* my = S + line * RG::XCH;
    float2* park = S + RG::XA;
    fill_twiddles<L>(tw, tid, T);
    const float al = a.alpha(g), r2n = a.rho2n(g);
    const bool init = __builtin_amdgcn_readfirstlane(init_flag) != 0;
    const size_t gb = (size_t)g * K * L;
    const float* HXs = reinterpret_cast<const float*>(a.s_x);
    __syncthreads();  // twiddles
    GD_TRACE(0);

    // C1: column kx of H X / L^2 (pass A's product; 16-byte loads in the lines' register order); the next
    // column's loads are issued before this column's inverse FFT
    struct ColLd {
        f4v x[F2 / 2];
    };
    auto col_load = [&](ColLd& c, int kx) {
        kx = opaque(kx);
        const int jj = opaque(j);
#pragma unroll
        for (int m = 0; m < F2 / 2; ++m) c.x[m] = ld4v(HXs + 2 * (gb + soff_c(kx, m, jj)));
    };
    auto col_hx = [&](float2 (&C)[F2], const ColLd& c) {
#pragma unroll
        for (int m = 0; m < F2 / 2; ++m) {
            C[2 * m] = cscale(make_float2(c.x[m][0], c.x[m][1]), inv_n);
            C[2 * m + 1] = cscale(make_float2(c.x[m][2], c.x[m][3]), inv_n);
        }
    };
    float2 CA[RG::CPL][F2], CB[RG::CPL][F2];
    {
        ColLd ld;
        col_load(ld, line);
        __builtin_amdgcn_sched_barrier(0);
        static_for<0, 2 * RG::CPL>([&](auto ic) {
            constexpr int i = decltype(ic)::value;  // columns: CA[0], CA[1], CB[0], CB[1]
            float2 (&C)[F2] = i < RG::CPL ? CA[i] : CB[i - RG::CPL];
            col_hx(C, ld);
            if constexpr (i == 0) {
                if (l0) {  // line 0: column 0 + i (the Nyquist column L/2), both real after the inverse
                    ColLd nl;
                    col_load(nl, L / 2);
                    float2 Nc[F2];
                    col_hx(Nc, nl);
#pragma unroll
                    for (int s2 = 0; s2 < F2; ++s2) C[s2] = make_float2(C[s2].x - Nc[s2].y, C[s2].y + Nc[s2].x);
                }
            }
            if constexpr (i + 1 < 2 * RG::CPL)
                col_load(ld, (i + 1 < RG::CPL ? 0 : KS) + line + LINES * ((i + 1) % RG::CPL));
            __builtin_amdgcn_sched_barrier(0);
            reg_fft<L, true>(C, opaque(j), my, tw);
            pin(C);  // materialised here: spill-free (2 VGPRs spilled across phase I otherwise)
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    if (l0) {
#pragma unroll
        for (int s = 0; s < F2; ++s) nyqo[j + F1 * s] = CA[0][s].y;
    }
    GD_TRACE(1);
    // I: per half of the rows, row IFFT -> Hx; the V step and duals (RI_ITER / RI_INIT's arithmetic)
    // -> w' (out); w' rows FFT'd again into X (row pair p = 64 hf + m, X[2 hf + w])
    float2 X[RG::PPL][F2];
    const float* yg = a.y + (size_t)g * L * L;
    float* wg = a.o1 + (size_t)g * L * L;
    static_for<0, 2>([&](auto hfc) {
        constexpr int hf = decltype(hfc)::value;
        lds_barrier();  // exchange areas -> row half spectra
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
        if (tid < L / 2) S[tid * SLD + L / 2] = make_float2(nyqo[hf * L / 2 + tid], 0.f);
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
#pragma unroll
        for (int w = 0; w < RG::HPL; ++w) {
            float2 (&V)[F2] = X[2 * hf + w];
            reg_fft<L, true>(V, opaque(j), my, tw);
            const size_t ro0 = (size_t)(hf * L / 2 + 2 * (opaque(line) + LINES * w)) * L + opaque(j);
            // y and w in chunks of PC pixels per row, loaded together: the w stores may alias the y loads
            // for the compiler, which would otherwise serialise every pixel's loads behind the previous
            // pixel's store (one memory latency per pixel).  (Double-buffering the chunks, and loading the
            // first under the IFFT, spilled and measured slower: 1.48 -> 1.58 ms.)
            constexpr int PC = GD_POIS_PC;
#pragma unroll
            for (int r0 = 0; r0 < F2; r0 += PC) {
                float yv[PC][2], wv[PC][2];
#pragma unroll
                for (int r = 0; r < PC; ++r) {
                    yv[r][0] = yg[ro0 + F1 * (r0 + r)];
                    yv[r][1] = yg[ro0 + L + F1 * (r0 + r)];
                    wv[r][0] = init ? 0.f : wg[ro0 + F1 * (r0 + r)];
                    wv[r][1] = init ? 0.f : wg[ro0 + L + F1 * (r0 + r)];
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int r = 0; r < PC; ++r) {
                    float2 wn;
                    const float hx0 = V[r0 + r].x, hx1 = V[r0 + r].y;
                    const float y0 = fmaxf(yv[r][0], 0.f), y1 = fmaxf(yv[r][1], 0.f);
                    if (init) {  // RI_INIT: v1 = V(H x0 + 0), w1 = v1 (u2 = 0)
                        wn = make_float2(v_step(GD_LLH_POISSON, hx0 + 0.0f, y0, r2n, al),
                                         v_step(GD_LLH_POISSON, hx1 + 0.0f, y1, r2n, al));
                    } else {     // RI_ITER: u2 = u2 + Hx - v = Hx - w; v' = V(Hx + u2); w' = v' - u2
                        const float u20 = hx0 - wv[r][0], u21 = hx1 - wv[r][1];
                        wn = make_float2(v_step(GD_LLH_POISSON, hx0 + u20, y0, r2n, al) - u20,
                                         v_step(GD_LLH_POISSON, hx1 + u21, y1, r2n, al) - u21);
                    }
                    wg[ro0 + F1 * (r0 + r)] = wn.x;
                    wg[ro0 + L + F1 * (r0 + r)] = wn.y;
                    V[r0 + r] = wn;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            reg_fft<L, false>(V, opaque(j), my, tw);  // F(w') rows
            pin(V);
            __builtin_amdgcn_sched_barrier(0);
        }
        GD_TRACE(2 + hf);
    });

    // W: F(w')'s columns -> the W slot (unnormalised, as F(z) in pass A, which multiplies by conj(H))
    auto wt_store = [&](const float2 (&C)[F2], int kx) {
        kx = opaque(kx);
        const int jj = opaque(j);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < F2 / 2; ++m)
            st4v(a.s_w + gb + soff_c(kx, m, jj), f4v{C[2 * m].x, C[2 * m].y, C[2 * m + 1].x, C[2 * m + 1].y});
    };
    lds_barrier();  // exchange areas -> slice A
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
#pragma unroll
    for (int u = 0; u < RG::CPL; ++u) {
        reg_fft<L, false>(CA[u], opaque(j), my, tw);
        __builtin_amdgcn_sched_barrier(0);
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
    lds_barrier();  // nyqc complete
    if (__builtin_amdgcn_readfirstlane(tid >> 6) < L / 64) a.s_w[((size_t)g * K + L / 2) * L + sidx_c<L>(tid)] = nyqc[tid];
#pragma unroll
    for (int u = 0; u < RG::CPL; ++u) wt_store(CA[u], line + LINES * u);
    GD_TRACE(4);
#pragma unroll
    for (int q = 0; q < RG::PPL; ++q)
#pragma unroll
        for (int r = RB0; r < RB0 + RG::PXB; ++r) X[q][r] = park[(q * RG::PXB + r - RB0) * T + opaque(tid)];
    lds_barrier();  // parked bins read -> slice B
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
    lds_barrier();  // slice B read -> exchange areas
#pragma unroll
    for (int u = 0; u < RG::CPL; ++u) {
        reg_fft<L, false>(CB[u], opaque(j), my, tw);
        wt_store(CB[u], KS + line + LINES * u);
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    GD_TRACE(5);
}
