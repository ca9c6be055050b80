/* gdeconv.h - C ABI of the MI355X spectral deconvolution engine (libgdeconv.so, gfx950).
 *
 * Conventions (every entry point):
 *   - plain C types only; images are fp32 [N][H][W] row-major (the NCHW C=1 tensors of the
 *     reference), per-galaxy scalars are (pointer, stride-in-elements) pairs, stride 0 = broadcast;
 *   - every pointer is a caller-allocated DEVICE pointer; the library never allocates, copies to
 *     the host or synchronises: work is enqueued on `stream` (a hipStream_t, e.g. torch's current
 *     stream) and the call returns immediately, so calls can be captured in a hipGraph;
 *   - return GD_OK (0) or a negative GD_ERR_* code; gd_last_error() gives a per-thread message.
 *     No C++ exception crosses the ABI.  Re-entrant across streams given distinct workspaces;
 *   - spectra are half spectra stored TRANSPOSED, complex64 [N][W/2+1][H] (kx-major, ky
 *     contiguous); `ws` is a workspace of gd_workspace_bytes(N, H, W) bytes;
 *   - sizes: any H x W with 2 <= H, W <= 4096 (utils/utils_torch.py's torch.fft path takes any size);
 *     square 32/48/64/96/128/256 run compile-time-planned kernels, every other size the runtime-
 *     planned ones (csrc/gd_generic.hpp) with the same operation chains.  The Gaussian ADMM init and
 *     iteration run one launch per call at 256^2 (k_gal_reg_init / k_gal_reg), 32/48/64 (k_gal_small*)
 *     and every multiple of 16 from 80 to 160, 96 and 128 included (k_gal_mid_init / k_gal_mid); PSFs
 *     square, even side <= min(H, W).
 *
 * Reference interfaces replaced (paths relative to mbertagna/Galaxy-Deconv @ 2025-03-07):
 *   gd_psf_to_otf       utils/utils_torch.py:79-92   psf_to_otf(ker, size)
 *   gd_conv_fft_batch   utils/utils_torch.py:46-50   conv_fft_batch(H, x)   (conj=1: conv_fft_batch(conj(H), x))
 *   gd_rfft2/gd_irfft2  utils/utils_torch.py:22-27   fftn / ifftn over dims [2,3] (real input, half spectrum)
 *   gd_admm_init        models/Unrolled_ADMM.py:181-196 + init_l2 :170-175 (+ first V step of :207)
 *   gd_admm_iter        models/Unrolled_ADMM.py:199-214 loop body around the denoiser call :208
 *   gd_admm_iter_v      the same, arguments packed (interpreted callers)
 *                       (X_Update :315-319, V_Update_{Poisson,Gaussian} :326-328/:335-336, duals
 *                       :212-213, next V step, output scaling :215)
 *   gd_wiener           models/Wiener.py:10-20       Wiener.forward(y, psf, alpha)
 *   gd_richardson_lucy  models/Richard_Lucy.py:10-24 Richard_Lucy(n_iters).forward(y, psf)
 *   gd_tikhonov         models/Tikhonet.py:15-31     Tikhonov(filter).forward(y, psf, alpha, lam)
 *   gd_filter_power     models/Tikhonet.py:26-27     LtL = |psf_to_otf(laplacian_kernel(), y.size())|^2
 *   gd_gx_init          models/unrolled_admm_gaussian.py:111-127  UnrolledADMMGaussian Y, H, init_l2
 *   gd_gx_xupdate       models/unrolled_admm_gaussian.py:85-93 (+ dual update :145, denoiser input :142)
 *   gd_gx_xupdate_backward  adjoint of XUpdateGaussian (autograd for train.py:41's model)
 *   gd_pack_*           utils/utils_data.py:87-103 Galaxy_Dataset.__getitem__ (per-file torch.load of
 *                       psf/obs/gt + alpha = obs.mean()) and :131-136 get_dataloader's batching: whole
 *                       batches read from one packed file (host side; no device pointers)
 */
#ifndef GDECONV_H
#define GDECONV_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GD_ABI_VERSION 5  /* 5: strict 0 / 1 fused-path setters, capture pipelining opt-in (mode 1 gone) */

#define GD_OK 0
#define GD_ERR_ARG (-1)
#define GD_ERR_UNSUPPORTED (-2)
#define GD_ERR_HIP (-3)

#define GD_LLH_GAUSSIAN 0
#define GD_LLH_POISSON 1

int gd_abi_version(void);
const char* gd_engine_rev(void);
/* sha256 prefix (16 hex digits) of the sources this library was compiled from (the csrc .hip and .hpp
   files and this header; __graft_entry__.build passes it in): smoke() compares it with the tree it runs in */
const char* gd_engine_src_hash(void);
/* hipRuntimeGetVersion of the HIP runtime this library runs on (in a PyTorch process: the runtime PyTorch bundles,
   e.g. 70051831 = ROCm 7.0 for torch 2.10+rocm7.0, whatever /opt/rocm holds), or a negative error code */
int gd_hip_runtime_version(void);
const char* gd_last_error(void);
int gd_supported_size(int H, int W);  /* 1 compile-time-planned, 2 runtime-planned, 0 unsupported */
size_t gd_workspace_bytes(int N, int H, int W);
size_t gd_otf_bytes(int N, int H, int W);

/* OTF of h x w PSFs placed in an H x W image with pixel (h/2, w/2) circularly shifted to (0,0). */
int gd_psf_to_otf(const float* psf, long long psf_gstride, int h, int w, int N, int H, int W,
                  void* otf_half, void* ws, void* stream);

/* out = Re IFFT2(FFT2(x) * H) (conj != 0: * conj(H)); one OTF per galaxy. */
int gd_conv_fft_batch(const void* otf_half, int conj, const float* x, float* out, int N, int H, int W,
                      void* ws, void* stream);
/* The same with otf_gstride complex elements between galaxies' OTFs: (W/2+1)*H (one per galaxy) or 0
 * (one OTF for the whole batch: the broadcast of the reference's fftn(x) * H with H [1,1,H,W],
 * utils/utils_torch.py:46-50).  Any other stride: GD_ERR_ARG. */
int gd_conv_fft_batch_strided(const void* otf_half, long long otf_gstride, int conj, const float* x, float* out,
                              int N, int H, int W, void* ws, void* stream);

/* Forward real 2D FFT into image slot 0 of a workspace-shaped buffer `spec`
 * (gd_workspace_bytes(N,H,W) bytes; spectrum = first N*(W/2+1)*H complex of each galaxy's slot 0,
 * i.e. element [g][0][kx][ky]).  gd_irfft2 inverts it in place (spec is clobbered). */
int gd_rfft2(const float* x, void* spec, int N, int H, int W, void* stream);
int gd_irfft2(void* spec, float* x, int N, int H, int W, void* stream);

/* Unrolled ADMM.  The per-forward state lives in an opaque device buffer of
 * gd_admm_state_bytes(N,H,W,llh) bytes whose first gd_otf_bytes(N,H,W) bytes are the half-spectrum
 * OTF (Poisson).  llh = GD_LLH_GAUSSIAN keeps the state in the SPECTRAL domain - |H|^2,
 * conj(H) F(max(y,0)/alpha), F(u1), conj(H) F(v - u2) - since every step of the Gaussian iteration is
 * linear: one forward and one inverse transform per iteration.  GD_LLH_POISSON (sqrt in the V step)
 * keeps the OTF and u1, v - u2 as images.  Everything a later call needs is in `state`; `ws`
 * (gd_workspace_bytes) is scratch for the duration of one call only.  The buffer's layout is private to
 * the engine (at 256^2 the Gaussian slots are 256 KiB apart: HBM channel spread).
 *
 * gd_admm_init: OTF, x0 = clamp(init_l2) -> zin (the first denoiser input, x0 + u1 with u1 = 0),
 *               u1 = u2 = 0 and the first V step with rho2 = rho2_iters[..., 0].  llh = Gaussian: the
 *               first V step is formed by iteration 0 (gd_admm_iter's rho2 is rho2_iters[..., 0]), so
 *               the init reads no rho (rho2 may be NULL) and may run while the SubNet computes the
 *               schedule (gd_admm_init_reads_rho); likewise Poisson in state layout 4.
 * gd_admm_iter: one loop body after the denoiser produced z from zin (iter = 0-based index):
 *               X update, duals, then (unless last) the next V step with rho2_next and the next
 *               denoiser input x + u1 -> zin_or_out; last != 0 -> zin_or_out = x (times alpha for
 *               Poisson).  z may alias zin_or_out (identity denoiser). */
size_t gd_admm_state_bytes(int N, int H, int W, int llh);
/* Which state layout gd_admm_init would write NOW for (H, W, llh): 1 = Gaussian spectral, 2 = Poisson
 * in two whole-galaxy passes (256^2 with a fused iteration: [|H|^2 | H | U1 | W~ | X] + w), 3 = Poisson
 * three-kernel ([otf | u1 | w]), 4 = Poisson at square L <= 112 with the fused init and iteration (the
 * buffers of 3; the init leaves H x0 in the w slot and reads no rho, iteration 0 forms w1 with its rho2);
 * negative = unsupported.  The Poisson layout follows gd_set_fused_iteration / gd_set_fused_init and, at 256^2,
 * the batch (gd_set_fused_min_batch), so a caller records it at init and checks it before each gd_admm_iter (a
 * toggle in between would bind a different layout than the init wrote). */
int gd_admm_state_layout(int N, int H, int W, int llh);
/* 1 if gd_admm_init reads its rho2 argument for (H, W, llh) (Poisson layouts 2 and 3: the first V step
 * is taken in the init), 0 if it does not (Gaussian, every size; Poisson layout 4), negative = unsupported. */
int gd_admm_init_reads_rho(int H, int W, int llh);
int gd_admm_init(const float* y, const float* psf, long long psf_gstride, int h, int w,
                 const float* alpha, long long alpha_stride, const float* rho2, long long rho2_stride,
                 int llh, int N, int H, int W, void* state, float* zin, void* ws, void* stream);
int gd_admm_iter(const float* y, const float* z, float* zin_or_out, const float* alpha, long long alpha_stride,
                 const float* rho1, long long rho1_stride, const float* rho2, long long rho2_stride,
                 const float* rho2_next, long long rho2_next_stride, int llh, int iter, int last, int N, int H,
                 int W, void* state, void* ws, void* stream);
/* gd_admm_iter with its 20 arguments packed in that order into one int64 array (pointers and strides as
 * integers, the int arguments widened): same semantics and return codes.  For interpreted callers whose
 * per-argument conversion costs more than the call (Python ctypes: 2.9 us for the 20-argument call, 0.6 us for a
 * short one) - at 256 x 48^2 the host sets the pace of an eager forward (gdeconv.engine.ADMMState.step). */
int gd_admm_iter_v(const long long* argv);

/* x = Re IFFT2(conj(H) FFT2(y) / (|H|^2 + 350/alpha)). */
int gd_wiener(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
              long long alpha_stride, float* x, int N, int H, int W, void* ws, void* stream);

/* Richardson-Lucy from x0 = max(y,0); otf_half receives the OTF (gd_otf_bytes). */
int gd_richardson_lucy(const float* y, const float* psf, long long psf_gstride, int h, int w, int n_iters,
                       float* x, int N, int H, int W, void* otf_half, void* ws, void* stream);

/* Tikhonov solve: x = Re IFFT2(conj(H) FFT2(y/alpha) / (|H|^2 + lam * LtL)); ltl = NULL is the
 * 'Identity' filter (divisor |H|^2 + lam).  ltl: real half spectra [*][W/2+1][H] (transposed, as the
 * OTF), ltl_gstride elements between galaxies (0 = one shared filter), e.g. from gd_filter_power.
 * lam: per-galaxy scalar (stride 0 = the reference's single learnable lambda). */
int gd_tikhonov(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
                long long alpha_stride, const float* lam, long long lam_stride, const float* ltl,
                long long ltl_gstride, float* x, int N, int H, int W, void* ws, void* stream);

/* power_half[g][kx][ky] = |FFT2(filt[g])|^2 over the half spectrum (filt: real images [N][H][W],
 * any placement, e.g. the circularly shifted Laplacian of the reference's psf_to_otf). */
int gd_filter_power(const float* filt, float* power_half, int N, int H, int W, void* ws, void* stream);

/* Same for ONE filter given as ntaps non-zero pixels (rc = [row, col] pairs in [0,H) x [0,W), vals),
 * by direct DFT in double rounded once - for the sparse Tikhonov Laplacian, whose |L|^2 sits in the
 * divisor where |H|^2 vanishes (fp32 FFT rounding would be amplified there). */
int gd_filter_power_taps(const int* rc, const float* vals, int ntaps, float* power_half, int H, int W,
                         void* stream);

/* UnrolledADMMGaussian (the variant train.py trains): images H x W (both even, <= 2048, square or not:
 * a non-square image runs on the runtime-planned kernels) and PSFs of the SAME size, zero-padded per
 * axis to the 2H x 2W grid (pad_double) with the reference's
 * ifftshift / fftshift / crop_half expressed as origin placement (the shift is a common phase that
 * cancels).  state: gd_gx_state_bytes - |H|^2 and G = F(max(y,0)) conj(H) on the 2H x 2W grid, written
 * by gd_gx_init, which also writes z0 = init_l2 (H x W).  ws: gd_workspace_bytes(N, 2H, 2W).
 *
 * gd_gx_xupdate: x = XUpdateGaussian(Y, Ht, HtH, z, u, rho) (H x W).  u may be NULL (zero).  If
 *   x_prev != NULL, first u = u + rho_prev (x_prev - z) in place (the dual update of the previous
 *   iteration, fused).  zin != NULL: also writes rho x + u (the next denoiser input).  xspec != NULL
 *   (gd_gx_spec_bytes): saves the X spectrum for the backward.
 * gd_gx_xupdate_backward: given dL/dx, writes dL/dz = rho M g, dL/du = -M g (M = the X update's
 *   linear part, self-adjoint) and per-(galaxy, kx) parts of dL/drho [N][W+1] (sum them per galaxy);
 *   z is the forward's z, xspec the forward's saved spectrum. */
size_t gd_gx_state_bytes(int N, int H, int W);
size_t gd_gx_spec_bytes(int N, int H, int W);
int gd_gx_init(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
               long long alpha_stride, int N, int H, int W, void* state, float* z0, void* ws, void* stream);
int gd_gx_xupdate(const float* z, float* u, const float* x_prev, const float* rho, long long rho_stride,
                  const float* rho_prev, long long rho_prev_stride, float* x, float* zin, void* xspec,
                  int N, int H, int W, void* state, void* ws, void* stream);
int gd_gx_xupdate_backward(const float* grad_x, const float* z, const float* rho, long long rho_stride,
                           const void* xspec, float* grad_z, float* grad_u, float* grad_rho_part, int N, int H,
                           int W, void* state, void* ws, void* stream);

/* SubNet feature extractor (models/Unrolled_ADMM.py:77-84): from the 128x128 half-spectrum OTF
 * of the PSFs (gd_psf_to_otf with H = W = 128; |OTF|^2 = |FFT2(pad128(psf))|^2), MaxPool2 and the
 * four Down blocks' 8 conv3x3 + ReLU layers (BatchNorm folded in) -> feat [N][1024] in the
 * reference's flatten order.  params: gd_subnet_param_count() floats, per conv layer l = 0..7
 * (cin,cout) = (1,4),(4,4),(4,8),(8,8),(8,16),(16,16),(16,16),(16,16): weights tap-major
 * [cin][3][3][cout] (nn.Conv2d's [cout][cin][3][3] permuted (1, 2, 3, 0)) then bias [cout]. */
int gd_subnet_param_count(void);
int gd_subnet_features(const void* otf128_half, const float* params, float* feat, int N, void* stream);

/* The whole SubNet forward (models/Unrolled_ADMM.py:77-86): the features above into feat (caller
 * scratch, [N][1024] floats), then one batched MLP launch [feat; alpha] -> 64 -> ReLU -> 64 -> ReLU ->
 * n_out -> Softplus, + 1e-6 -> rhos [N][n_out] (rho1 = rhos[:, :n], rho2 = rhos[:, n:] for n_out = 2n).
 * mlp_params: gd_subnet_mlp_param_count(n_out) floats, the nn.Linear weights TRANSPOSED: W1^T [1025][64] |
 * b1 [64] | W2^T [64][64] | b2 [64] | W3^T [64][n_out] | b3 [n_out]; alpha: per-galaxy scalars with
 * alpha_stride (0 = one alpha).  n_out in [1, 64]; gd_subnet_mlp_param_count returns 0 outside it. */
int gd_subnet_mlp_param_count(int n_out);
int gd_subnet_rhos(const void* otf128_half, const float* params, const float* mlp_params, const float* alpha,
                   long long alpha_stride, float* feat, float* rhos, int n_out, int N, void* stream);

/* gd_subnet_rhos from the PSFs themselves (psf [*][h][h], psf_gstride floats between galaxies, 0 = one
 * shared PSF; h even, <= 64): |FFT2(pad128(psf))|^2 is computed inside the feature kernel, so no
 * gd_psf_to_otf pre-pass and no 128^2 OTF buffer (models/Unrolled_ADMM.py:77-83). */
int gd_subnet_rhos_psf(const float* psf, long long psf_gstride, int h, const float* params, const float* mlp_params,
                       const float* alpha, long long alpha_stride, float* feat, float* rhos, int n_out, int N,
                       void* stream);

/* gd_admm_init (llh = Gaussian, or Poisson in state layout 4) and gd_subnet_rhos_psf of the same batch in
 * ONE launch: the SubNet's workgroups and the init's share the CUs (models/Unrolled_ADMM.py:177-196, the
 * rhos of :77-90 and init_l2 :170-175; those inits read no rho, so the two are independent).  For small square
 * images (32, 48, 64: the LSST stamps of configs[1]) and batches of at most the fused-SubNet limit;
 * gd_admm_init_subnet_supported says whether a call is fusable, otherwise the call returns
 * GD_ERR_UNSUPPORTED and the caller runs the two entry points.  Results are bit-identical to the pair. */
int gd_admm_init_subnet_supported(int N, int H, int W, int h, int w, int llh, int n_out);
int gd_admm_init_subnet(const float* y, const float* psf, long long psf_gstride, int h, int w, const float* alpha,
                        long long alpha_stride, int llh, int N, int H, int W, void* state, float* zin,
                        const float* params, const float* mlp_params, float* rhos, int n_out, void* ws, void* stream);

/* Infinity-Cache pipelining: multi-kernel operations (ADMM init/iteration, Wiener, Richardson-Lucy)
 * run over the batch in chunks of about `bytes` of workspace (default 96 MiB, i.e. 186 galaxies at
 * 256^2); consecutive chunks go to internal HIP streams (default 2) forked from and joined back into
 * the caller's stream, so each chunk's spectra stay resident in the 256 MiB Infinity Cache while the
 * chip stays full.  bytes = 0: one pass over the batch.  Both setters return the previous value;
 * process-wide, set them before enqueuing work. */
size_t gd_set_chunk_bytes(size_t bytes);
int gd_set_pipeline_streams(int streams);

/* Chunk pipelining under stream capture, for the CALLING HOST THREAD only: mode 0 (the default) runs a captured
 * operation's chunks in sequence on the capturing stream; mode 2 forks them onto streams of the calling thread (never
 * the internal streams eager calls of other threads use, since streams that join a capture stay in it until
 * hipStreamEndCapture), each operation with an event set of its own.  Opt in to 2 only when enqueuing from the
 * capturing stream itself (gdeconv.graphs.GraphedForward does) when the HIP runtime is older than 7.2
 * (gd_hip_runtime_version() < 70200000): there a fork from a stream that joined the capture through an event (onto
 * any other streams, no engine call needed) segfaults inside hipStreamEndCapture; ROCm 7.2's runtime captures the
 * same sequence (tools/capture_probe.hip mode 2).  -1 restores the default (the GD_CAPTURE_PIPELINE
 * environment variable, 0 or 2, else 0).  Returns the previous override (-1: none), or GD_ERR_UNSUPPORTED (setting
 * unchanged) for any other mode. */
int gd_set_capture_pipeline(int mode);

/* Fused iterations: at the sizes that have them (see "sizes" above; Poisson at 256^2 and square L <= 112)
 * gd_admm_iter runs one workgroup per galaxy holding the galaxy's spectra on-chip (no workspace traffic).
 * on = 1 (default) selects them; 0 selects the chained path (row pass / column pass / row pass through
 * the workspace).  Returns the previous setting (0 or 1), or GD_ERR_ARG (setting unchanged) for any other value;
 * process-wide. */
int gd_set_fused_iteration(int on);

/* Richardson-Lucy at 256^2 (gd_richardson_lucy, models/Richard_Lucy.py:10-24): on = 1 (default) runs the
 * OTF, then the whole n_iters loop of each galaxy inside one 512-thread workgroup (k_rl_reg: the
 * galaxy's spectra stay on-chip; x, y and the OTF are re-read from the cache hierarchy); 0 selects the
 * chunked chain (four launches per iteration through the workspace).  Returns the previous setting (0 or 1), or
 * GD_ERR_ARG (setting unchanged) for any other value; process-wide. */
int gd_set_fused_rl(int on);

/* SubNet from the PSFs (gd_subnet_rhos_psf): batches of at most n galaxies run features + MLP in ONE
 * launch, one workgroup per galaxy (each reads the MLP weights from L2; `feat` is not written); larger
 * batches run the feature kernel and the batched MLP kernel (8 galaxies per workgroup).  The rhos are
 * bit-identical either way (same summation order).  Default 256; n < 0 only queries.  Returns the
 * previous value. */
int gd_set_subnet_fused_max(int n);

/* 256^2: batches of at least n galaxies run the whole-galaxy kernels when those are on, smaller batches the chained
 * row / column kernels, whose many small workgroups fill the CUs that one workgroup per galaxy leaves idle below a
 * round of workgroups (results within rounding of each other).  op 0 = Gaussian ADMM (k_gal_reg and the one-launch
 * init; the same state layout either way, so chosen per call; default 96), 1 = Poisson ADMM (the two-pass path,
 * state layout 2, against the three-kernel chain, layout 3: see gd_admm_state_layout; default 192), 2 =
 * Richardson-Lucy (k_rl_reg against the chunked chain; default 96).  n < 0 only queries.  Returns the previous
 * value (GD_ERR_ARG for another op); process-wide. */
int gd_set_fused_min_batch(int op, int n);

/* Fused Gaussian init (replaces the chunked RF_YA -> psf_rows -> C_G_INIT -> RIF_CLAMP -> C_G_W1 chain
 * behind gd_admm_init, models/Unrolled_ADMM.py:170-175 + the first V step :335-336): at 256^2 (PSF side
 * <= 64) the PSF's row spectra go into the state's U1 slot, then one workgroup per galaxy runs y ->
 * |H|^2, G, x0 = clamp(X0) -> zin and F(x0) -> W~ with no workspace traffic (k_gal_reg_init).  on = 1
 * (default) selects it, 0 the chunked chain.  At the mid sizes (80 ... 160, multiples of 16) the one-launch
 * k_gal_mid_init (the placed PSF's row spectra parked in the U1 slot, the half spectrum in LDS) runs when
 * BOTH this and gd_set_fused_iteration are on, in place of the RF_PSF_Y -> C_G_INIT -> RIF_CLAMP -> C_G_W1
 * chain.  Returns the previous setting (0 or 1), or GD_ERR_ARG (setting unchanged) for any other value;
 * process-wide. */
int gd_set_fused_init(int on);

/* Opt-in timing with hipEvents: level 1 brackets every whole operation (op_admm_init/op_admm_iter,
 * the SubNet kernel) on the caller's stream; level 2 also brackets every kernel launch on its own
 * stream (adds two event records per launch - under pipelining that perturbs what it measures).
 * gd_profile_collect() waits for the events and returns the number of distinct entries;
 * gd_profile_get(i, ...) reads the i-th (name, total ms, launches); gd_profile_reset() clears. */
int gd_profile_enable(int level);
int gd_profile_collect(void);
int gd_profile_get(int i, char* name, int name_len, double* total_ms, long long* launches);
int gd_profile_reset(void);

/* Packed galaxy datasets (GDPACK01; writer: gdeconv/ingest.py).  HOST-side entry points: `dst` is
 * host memory (pinned by the caller for fast H2D), nothing touches the GPU.  Sections: */
#define GD_PACK_OBS 0   /* fp32 [n][H][W] observations                         */
#define GD_PACK_PSF 1   /* fp32 [n][h][w] PSFs                                 */
#define GD_PACK_GT 2    /* fp32 [n][H][W] ground truth (when dims[4] != 0)     */
#define GD_PACK_ALPHA 3 /* fp32 [n]       alpha = obs.ravel().mean() per galaxy */
#define GD_PACK_INFO 4  /* UTF-8 JSON     the dataset's info.json (n_train, n_test, sequence, ...) */

/* Open `path`; *n = galaxies, dims = {H, W, h, w, has_gt}.  *handle is freed by gd_pack_close. */
int gd_pack_open(const char* path, void** handle, long long* n, int* dims);
/* Bytes of a section (-1 on a bad handle / section). */
long long gd_pack_section_bytes(void* handle, int section);
/* Galaxies [g0, g0 + count) of a section -> dst (contiguous), read by up to nthreads pread threads.
 * GD_PACK_INFO ignores g0 / count and copies the whole JSON (gd_pack_section_bytes bytes). */
int gd_pack_read(void* handle, int section, long long g0, long long count, void* dst, int nthreads);
/* Galaxies idx[0..count) of a section (0..3) -> dst in that order (shuffled batches). */
int gd_pack_gather(void* handle, int section, const long long* idx, long long count, void* dst, int nthreads);
int gd_pack_close(void* handle);

#ifdef __cplusplus
}
#endif

#endif /* GDECONV_H */
