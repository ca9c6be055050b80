// Whole Richardson-Lucy loop per galaxy (k_rl_reg<256>): models/Richard_Lucy.py:10-24,
//   y = max(y, 0); x = y;  n x { Hx = conv(H, x); num = conv(conj H, y / Hx); x = x * num / div }
// with div = conv(conj H, ones) = H(0, 0) (real), one 512-thread workgroup per galaxy running ALL the
// iterations on k_gal_reg's skeleton (gd_galreg.hpp).  The chunked chain (C_CONV -> RIF_RL_RATIO ->
// C_CONVC -> RIF_RL_UPDATE, four launches and four half-spectrum round trips of the workspace per
// iteration) becomes, per iteration:
//   C1  columns of x's row spectra (in registers): FFT, * H / L^2, inverse FFT     (slices A, B)
//   I1  per half of the rows: row IFFT -> Hx; ratio = max(y, 0) / Hx; row FFT -> registers
//   C2  columns: FFT, * conj(H) / L^2, inverse FFT
//   I2  per half: row IFFT -> num; x = x * num / div -> out; row FFT -> registers (not after the last)
// The galaxy's spectra never leave the CU; per iteration it reads y, x and H twice (MALL-resident for
// the galaxies in flight) and writes x.  Arithmetic per bin / pixel as k_col<C_CONV / C_CONVC> and
// k_row_invfwd<RIF_RL_RATIO / RIF_RL_UPDATE>, except the ratio's division (rl_div: a reciprocal and one Newton
// step) and the update's 1 / div (one reciprocal per galaxy).
// Neither product carries the chain's 1 / L^2: Hx comes out L^2 too large, y / Hx L^2 too small, and the conj(H)
// pass's missing 1 / L^2 restores num (L^2 = 2^16: power-of-two scalings, no extra rounding; round 6: 2.6 % fewer
// VALU instructions, time unchanged - profiles/r06o_rl_ab.txt).
// The OTF (a.otf, [N][K][L], ky contiguous) is computed beforehand (psf_to_otf).
// Included inside namespace gd by gd_engine.hip (after gd_galreg.hpp).

#ifndef GD_RL_HPF
#define GD_RL_HPF 4  // bit 0 / bit 1: slice A's / B's OTF columns loaded before its forward column FFTs (latency hidden);
                      // bit 2: slice A's column 0 before the FFTs, column 1 right after them
#endif
#ifndef GD_RL_DPP
#define GD_RL_DPP 0  // 1: every line FFT transposes in registers (DPP) instead of through the LDS exchange
#endif
#ifndef GD_RL_PAIR
#define GD_RL_PAIR 3  // bit 0: slice A's two columns transformed as a pair (reg_fft2), bit 1: slice B's, bit 2: the rows
#endif
#ifndef GD_RL_FASTDIV
#define GD_RL_FASTDIV 1
#endif

// y / Hx without the IEEE division sequence (div_scale / div_fmas / div_fixup and denorm-mode toggles,
// ~10 instructions): reciprocal, then one Newton correction of the quotient (within an ulp of the
// division; the pixel loop runs 256 of these per lane per iteration)
__device__ __forceinline__ float rl_div(float y, float d) {
#if GD_RL_FASTDIV
    const float r = __builtin_amdgcn_rcpf(d);
    const float q = y * r;
    return __builtin_fmaf(__builtin_fmaf(-d, q, y), r, q);
#else
    return y / d;
#endif
}
template <int L>
__global__ __launch_bounds__(512) void k_rl_reg(Args a, int n_iters) {
    using RG = RegGeo<L>;
    constexpr int F1 = RG::F1, F2 = RG::F2, KS = RG::KS, SLD = RG::SLD, LINES = RG::LINES, T = RG::THREADS;
    constexpr int RB0 = RG::RB0, RB1 = RG::RB1, K = RG::K;
    __shared__ float2 tw[L];
    __shared__ __attribute__((aligned(16))) float2 S[RG::U];
    __shared__ float2 nyq[RG::NP];  // X_p[L/2] of every pair
    __shared__ float2 nyqc[L];      // the Nyquist column's spectrum (line 0's own bins)
    __shared__ float nyqo[L];       // the Nyquist column after the inverse (x(., L/2))
    const int tid0 = threadIdx.x;
    const int g = blockIdx.x;
    fill_twiddles<L>(tw, tid0, T);
    const float* yg = a.y + (size_t)g * L * L;
    float* xg = a.o0 + (size_t)g * L * L;
    const float2* Hg = a.otf + (size_t)g * K * L;
    // the OTF's Nyquist column (kx = L/2), constant over the iterations: read once into LDS, so that line 0 - the
    // only holder of that column's bins - forms its products alone (round 6: the two workgroup barriers and the
    // per-pass global loads of a four-wave product are gone, 121.9 -> 120.0 ms per 4096 x RL(100), bit-identical;
    // profiles/r06zj_rl_nyquist_ab.txt)
    __shared__ float2 hnyq[L];
    for (int e = tid0; e < L; e += T) hnyq[e] = Hg[(size_t)(L / 2) * L + e];
    const float div = Hg[0].x;  // conv(Ht, ones) = H(0, 0)
    const float idiv = 1.0f / div;
    const int tid = tid0;
    GD_TRACE(0);

    // R: x0 = max(y, 0) -> row FFTs of the packed row pairs p = line + LINES q
    float2 X[RG::PPL][F2];
    {
        const int line = tid / F1, j = tid - line * F1;
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q) {
            const float* r0 = yg + (size_t)(2 * (line + LINES * q)) * L + j;
#pragma unroll
            for (int r = 0; r < F2; ++r) X[q][r] = make_float2(fmaxf(r0[F1 * r], 0.f), fmaxf(r0[L + F1 * r], 0.f));
        }
        // x0 -> out: every iteration's update then reads x from there (the same thread's own pixels)
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q) {
            float* o0 = xg + (size_t)(2 * (line + LINES * q)) * L + j;
#pragma unroll
            for (int r = 0; r < F2; ++r) {
                o0[F1 * r] = X[q][r].x;
                o0[L + F1 * r] = X[q][r].y;
            }
        }
    }
    stagger_start<GD_RL_STAGGER>(g, a.N);
    __syncthreads();  // twiddles
    {
        const int line = tid / F1, j = tid - line * F1;
        float2* my = S + line * RG::XCH;
#pragma unroll
        for (int q = 0; q < RG::PPL; ++q) {
            reg_fft<L, false, GD_RL_DPP != 0>(X[q], opaque(j), my, tw);
            pin(X[q]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    GD_TRACE(1);

    for (int it = 0; it < n_iters; ++it) {
        // thread-derived values recomputed per iteration from an opaque copy (hoisted out of the loop,
        // the addresses derived from them would stay live across the whole iteration)
        const int tt = opaque(tid0), line = tt / F1, j = tt - line * F1;
        const bool l0 = (line == 0);
        float2* my = S + line * RG::XCH;
        float2* park = S + RG::XA;
        const bool last = it + 1 == n_iters;

        float2 CA[RG::CPL][F2], CB[RG::CPL][F2];
        // column pass: X's row spectra -> CA, CB (columns line + LINES u of slices A, B) and nyqo, each
        // column transformed, multiplied by H (CONJ: conj H) / L^2 and transformed back
        auto cols = [&](auto conjc) {
            constexpr bool CONJ = decltype(conjc)::value;
            auto hload = [&](float2 (&h)[F2], int kx) {
                const float2* Hc = Hg + (size_t)opaque(kx) * L + opaque(j);
#pragma unroll
                for (int s = 0; s < F2; ++s) h[s] = Hc[F1 * s];
            };
            auto happly = [&](float2 (&C)[F2], const float2 (&h)[F2]) {
#pragma unroll
                for (int s = 0; s < F2; ++s) {
                    const c2 c = tc2(C[s]), hh = tc2(h[s]);
                    C[s] = tf2(pmul_r<CONJ>(c, hh, pmul_t(c, hh)));
                }
            };
            auto hmul = [&](float2 (&C)[F2], int kx) {
                float2 h[F2];
                hload(h, kx);
                happly(C, h);
            };
            lds_barrier();  // exchange areas / row spectra -> slice A
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
                if (l0) CA[0][s].y = (y & 1) ? w.y : w.x;  // line 0: column 0 + i column L/2
            }
            lds_barrier();  // slice A read -> exchange areas + parked slice B bins
#pragma unroll
            for (int q = 0; q < RG::PPL; ++q)
#pragma unroll
                for (int r = RB0; r < RB0 + RG::PXB; ++r) park[(q * RG::PXB + r - RB0) * T + tt] = X[q][r];
            __builtin_amdgcn_sched_barrier(0);
#if GD_RL_HPF & 1
            float2 hA[RG::CPL][F2];  // slice A's OTF columns in flight during its forward FFTs
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) hload(hA[u], line + LINES * u);
            __builtin_amdgcn_sched_barrier(0);
#endif
#if GD_RL_HPF & 4
            static_assert(RG::CPL == 2, "two columns per line and slice");
            float2 hA0[F2];  // column 0's OTF, in flight during the FFTs
            hload(hA0, line);
            __builtin_amdgcn_sched_barrier(0);
#endif
            if constexpr ((GD_RL_PAIR & 1) != 0) {
                reg_fft2<L, false>(CA[0], CA[1], opaque(j), my, tw);
                __builtin_amdgcn_sched_barrier(0);
            } else {
#pragma unroll
                for (int u = 0; u < RG::CPL; ++u) {
                    reg_fft<L, false, GD_RL_DPP != 0>(CA[u], opaque(j), my, tw);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#if GD_RL_HPF & 4
            float2 hA1[F2];  // column 1's OTF, in flight during the split and column 0's products
            hload(hA1, line + LINES);
            __builtin_amdgcn_sched_barrier(0);
#endif
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
#if GD_RL_HPF & 4
            happly(CA[0], hA0);
            __builtin_amdgcn_sched_barrier(0);
            happly(CA[1], hA1);
            __builtin_amdgcn_sched_barrier(0);
#else
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) {
#if GD_RL_HPF & 1
                happly(CA[u], hA[u]);
#else
                hmul(CA[u], line + LINES * u);
#endif
                __builtin_amdgcn_sched_barrier(0);
            }
#endif
            __builtin_amdgcn_sched_barrier(0);
            if (l0) {  // the lane's own Nyquist bins (written by the split above), times the column's OTF
#pragma unroll
                for (int s = 0; s < F2; ++s) {
                    const int ky = j + F1 * s;
                    const float2 hn = hnyq[ky];
                    const float2 cn = CONJ ? cmulc(nyqc[ky], hn) : cmul(nyqc[ky], hn);
                    CA[0][s] = make_float2(CA[0][s].x - cn.y, CA[0][s].y + cn.x);
                    if (s % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // four bins' reads in flight at a time
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr ((GD_RL_PAIR & 1) != 0) {
                reg_fft2<L, true>(CA[0], CA[1], opaque(j), my, tw);
                pin(CA[0]);
                pin(CA[1]);
                __builtin_amdgcn_sched_barrier(0);
            } else {
#pragma unroll
                for (int u = 0; u < RG::CPL; ++u) {
                    reg_fft<L, true, GD_RL_DPP != 0>(CA[u], opaque(j), my, tw);
                    pin(CA[u]);  // the column results materialised here (spill-free register allocation)
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (l0) {
#pragma unroll
                for (int s = 0; s < F2; ++s) nyqo[j + F1 * s] = CA[0][s].y;
            }
#pragma unroll
            for (int q = 0; q < RG::PPL; ++q)
#pragma unroll
                for (int r = RB0; r < RB0 + RG::PXB; ++r) X[q][r] = park[(q * RG::PXB + r - RB0) * T + opaque(tt)];
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
            lds_barrier();  // slice B read -> exchange areas + parked column A results
#pragma unroll
            for (int s = 0; s < F2; ++s) park[s * T + tt] = CA[RG::CPL - 1][s];
            __builtin_amdgcn_sched_barrier(0);
#if GD_RL_HPF & 2
            float2 hB[RG::CPL][F2];  // slice B's OTF columns in flight during its forward FFTs
#pragma unroll
            for (int u = 0; u < RG::CPL; ++u) hload(hB[u], KS + line + LINES * u);
            __builtin_amdgcn_sched_barrier(0);
#endif
            if constexpr ((GD_RL_PAIR & 2) != 0) {
                reg_fft2<L, false>(CB[0], CB[1], opaque(j), my, tw);
#pragma unroll
                for (int u = 0; u < RG::CPL; ++u) hmul(CB[u], KS + line + LINES * u);
                reg_fft2<L, true>(CB[0], CB[1], opaque(j), my, tw);
                pin(CB[0]);
                pin(CB[1]);
                __builtin_amdgcn_sched_barrier(0);
            } else {
#pragma unroll
                for (int u = 0; u < RG::CPL; ++u) {
                    reg_fft<L, false, GD_RL_DPP != 0>(CB[u], opaque(j), my, tw);
#if GD_RL_HPF & 2
                    happly(CB[u], hB[u]);
#else
                    hmul(CB[u], KS + line + LINES * u);
#endif
                    reg_fft<L, true, GD_RL_DPP != 0>(CB[u], opaque(j), my, tw);
                    pin(CB[u]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int s = 0; s < F2; ++s) CA[RG::CPL - 1][s] = park[s * T + opaque(tt)];
        };
        // row pass: per half, the columns' results -> row half spectra -> row IFFT -> pointwise ->
        // (row FFT -> X); UPD: the x update and store, else the ratio
        auto rows = [&](auto updc) {
            constexpr bool UPD = decltype(updc)::value;
            static_for<0, 2>([&](auto hfc) {
                constexpr int hf = decltype(hfc)::value;
                lds_barrier();  // parked results / exchange areas -> row half spectra
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
                if (tt < L / 2) S[tt * SLD + L / 2] = make_float2(nyqo[hf * L / 2 + tt], 0.f);
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
                // the pointwise step of row pair w (V = X[2 hf + w], already inverse-transformed)
                auto pointwise = [&](float2 (&V)[F2], int w) {
                    const size_t ro0 = (size_t)(hf * L / 2 + 2 * (opaque(line) + LINES * w)) * L + opaque(j);
                    float2 src[F2];  // (row e, row o) pixels: y (ratio), x (update)
                    const float* sp = (UPD ? xg : yg) + ro0;
#pragma unroll
                    for (int r = 0; r < F2; ++r) src[r] = make_float2(sp[F1 * r], sp[L + F1 * r]);
#pragma unroll
                    for (int r = 0; r < F2; ++r) {
                        if constexpr (UPD) {
                            // x * numerator / divisor
                            V[r] = GD_RL_FASTDIV ? make_float2(src[r].x * V[r].x * idiv, src[r].y * V[r].y * idiv)
                                                 : make_float2(src[r].x * V[r].x / div, src[r].y * V[r].y / div);
                            xg[ro0 + F1 * r] = V[r].x;
                            xg[ro0 + L + F1 * r] = V[r].y;
                        } else {
                            V[r] = make_float2(rl_div(fmaxf(src[r].x, 0.f), V[r].x), rl_div(fmaxf(src[r].y, 0.f), V[r].y));  // y / Hx
                        }
                    }
                };
                if constexpr ((GD_RL_PAIR & 4) != 0) {
                    static_assert(RG::HPL == 2, "two row pairs per line and half");
                    reg_fft2<L, true>(X[2 * hf], X[2 * hf + 1], opaque(j), my, tw);
                    __builtin_amdgcn_sched_barrier(0);
                    pointwise(X[2 * hf], 0);
                    __builtin_amdgcn_sched_barrier(0);
                    pointwise(X[2 * hf + 1], 1);
                    __builtin_amdgcn_sched_barrier(0);
                    if (!(UPD && last)) reg_fft2<L, false>(X[2 * hf], X[2 * hf + 1], opaque(j), my, tw);
                    pin(X[2 * hf]);
                    pin(X[2 * hf + 1]);
                    __builtin_amdgcn_sched_barrier(0);
                } else {
#pragma unroll
                    for (int w = 0; w < RG::HPL; ++w) {
                        float2 (&V)[F2] = X[2 * hf + w];
                        reg_fft<L, true, GD_RL_DPP != 0>(V, opaque(j), my, tw);
                        pointwise(V, w);
                        if (!(UPD && last)) reg_fft<L, false, GD_RL_DPP != 0>(V, opaque(j), my, tw);
                        pin(V);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            });
        };
        cols(std::false_type{});
        if (it == 0) GD_TRACE(2);
        rows(std::false_type{});
        if (it == 0) GD_TRACE(3);
        cols(std::true_type{});
        if (it == 0) GD_TRACE(4);
        rows(std::true_type{});
        if (it == 0) GD_TRACE(5);
    }
    __syncthreads();
    GD_TRACE(6);
}
