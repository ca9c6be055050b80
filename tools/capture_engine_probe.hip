// The capture crash's shape on the engine itself, without torch: Unrolled_ADMM's spectral forward (init + 8
// iterations, identity denoiser) at N x L^2 with the chunked runtime-planned Gaussian init (fused init off, chunk bytes
// forced down) captured on stream A, the init on a side stream B forked from A (ADMMState.init_concurrent), the
// chunks pipelined over the capture streams (gd_set_capture_pipeline(2)), B joined back to A, then the iterations
// on A; hipStreamEndCapture, instantiate, replay, and a bit-for-bit check against the eager forward.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o variants/capture_engine_probe tools/capture_engine_probe.hip
//   capture_engine_probe [side=1] [N=330] [L=160] [chunks=6]
//     side 0: the init on A (no side stream); 1: on B (created before the capture); 2: on B created inside the capture
//     with hipStreamCreateWithPriority (what torch.cuda.Stream() does there); 3: as 2, the init's chunks in sequence
//     (gd_set_capture_pipeline(0) around it: the shipped Python guard); 4: A and B created as torch creates its pool
//     streams (hipStreamCreateWithPriority, non-blocking, priority 0) before the capture, the fork and the join through
//     temporary events destroyed right after the wait (torch's Stream.wait_stream)
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"

#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define GK(x) do { int r_ = (x); if (r_ != GD_OK) { printf("engine error %d (%s) at %d\n", r_, gd_last_error(), __LINE__); exit(1); } } while (0)

__global__ void k_img(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u + seed;
        x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
        p[i] = 0.01f * ((x & 0xffffff) / float(0x1000000)) - 0.002f;
    }
}
__global__ void k_psf(float* p, int N, int h) {
    const int g = blockIdx.x;
    for (int i = threadIdx.x; i < h * h; i += blockDim.x) {
        const float dy = (i / h) - h / 2 + 0.5f, dx = (i % h) - h / 2 + 0.5f, s = 2.0f + (g % 7) * 0.3f;
        p[(size_t)g * h * h + i] = __expf(-(dx * dx + dy * dy) / (2 * s * s)) / (2 * 3.14159265f * s * s);
    }
}
__global__ void k_const(float* p, int n, float base, float step) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = base + step * (i % 13);
}

int main(int argc, char** argv) {
    const int side = argc > 1 ? atoi(argv[1]) : 1, N = argc > 2 ? atoi(argv[2]) : 330, L = argc > 3 ? atoi(argv[3]) : 160;
    const int chunks = argc > 4 ? atoi(argv[4]) : 6, h = 48, n_it = 8;
    float *y, *psf, *alpha, *rho1, *rho2, *zin, *out;
    void *state, *ws;
    CK(hipMalloc(&y, (size_t)N * L * L * 4));
    CK(hipMalloc(&zin, (size_t)N * L * L * 4));
    CK(hipMalloc(&out, (size_t)N * L * L * 4));
    CK(hipMalloc(&psf, (size_t)N * h * h * 4));
    CK(hipMalloc(&alpha, N * 4));
    CK(hipMalloc(&rho1, (size_t)N * n_it * 4));
    CK(hipMalloc(&rho2, (size_t)N * n_it * 4));
    CK(hipMalloc(&state, gd_admm_state_bytes(N, L, L, GD_LLH_GAUSSIAN)));
    CK(hipMalloc(&ws, gd_workspace_bytes(N, L, L) + 16));
    hipLaunchKernelGGL(k_img, dim3(1024), dim3(256), 0, 0, y, (size_t)N * L * L, 1u);
    hipLaunchKernelGGL(k_psf, dim3(N), dim3(256), 0, 0, psf, N, h);
    hipLaunchKernelGGL(k_const, dim3(4), dim3(256), 0, 0, alpha, N, 0.004f, 0.0003f);
    hipLaunchKernelGGL(k_const, dim3(8), dim3(256), 0, 0, rho1, N * n_it, 0.7f, 0.05f);
    hipLaunchKernelGGL(k_const, dim3(8), dim3(256), 0, 0, rho2, N * n_it, 0.9f, 0.04f);
    CK(hipDeviceSynchronize());
    const size_t tgal = (size_t)2 * (L / 2 + 1) * L * 8;
    gd_set_chunk_bytes((N / chunks + 1) * tgal);
    gd_set_fused_init(0);
    gd_set_capture_pipeline(2);
    hipStream_t A, B = nullptr;
    if (side == 4) {
        CK(hipStreamCreateWithPriority(&A, hipStreamNonBlocking, 0));
        CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, 0));
    } else {
        CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    }
    if (side == 1) CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    auto wait_tmp = [&](hipStream_t waiter, hipStream_t from) {  // torch's Stream.wait_stream
        hipEvent_t t;
        CK(hipEventCreateWithFlags(&t, hipEventDisableTiming));
        CK(hipEventRecord(t, from));
        CK(hipStreamWaitEvent(waiter, t, 0));
        CK(hipEventDestroy(t));
    };
    hipEvent_t eAB, eBA;
    CK(hipEventCreateWithFlags(&eAB, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eBA, hipEventDisableTiming));
    auto forward = [&](bool capturing) {
        hipStream_t is = A;
        if (side >= 1) {
            if ((side == 2 || side == 3) && capturing) CK(hipStreamCreateWithPriority(&B, hipStreamDefault, 0));
            if ((side == 2 || side == 3) && !capturing && !B) CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
            if (side == 4) {
                wait_tmp(B, A);
            } else {
                CK(hipEventRecord(eAB, A));
                CK(hipStreamWaitEvent(B, eAB, 0));
            }
            is = B;
        }
        const int old = side == 3 && capturing ? gd_set_capture_pipeline(0) : -2;
        GK(gd_admm_init(y, psf, (long long)h * h, h, h, alpha, 1, nullptr, 0, GD_LLH_GAUSSIAN, N, L, L, state, zin, ws, is));
        if (old != -2) gd_set_capture_pipeline(old);
        if (side == 4) {
            wait_tmp(A, B);
        } else if (side >= 1) {
            CK(hipEventRecord(eBA, B));
            CK(hipStreamWaitEvent(A, eBA, 0));
        }
        for (int it = 0; it < n_it; ++it) {
            const bool last = it == n_it - 1;
            GK(gd_admm_iter(y, zin, last ? out : zin, alpha, 1, rho1 + it, n_it, rho2 + it, n_it,
                            last ? nullptr : rho2 + it + 1, n_it, GD_LLH_GAUSSIAN, it, last, N, L, L, state, ws, A));
        }
    };
    forward(false);
    CK(hipStreamSynchronize(A));
    std::vector<float> ref((size_t)N * L * L), got(ref.size());
    CK(hipMemcpy(ref.data(), out, ref.size() * 4, hipMemcpyDeviceToHost));
    int rtv = 0;
    CK(hipRuntimeGetVersion(&rtv));
    printf("side %d, %d x %d^2, chunk bytes %zu, HIP runtime %d: eager forward done; capturing\n", side, N, L,
           (N / chunks + 1) * tgal, rtv);
    fflush(stdout);
    CK(hipStreamBeginCapture(A, hipStreamCaptureModeGlobal));
    forward(true);
    hipStreamCaptureStatus cs;
    unsigned long long id;
    hipGraph_t gg;
    const hipGraphNode_t* deps;
    size_t nd;
    CK(hipStreamGetCaptureInfo_v2(A, &cs, &id, &gg, &deps, &nd));
    size_t nodes = 0;
    CK(hipGraphGetNodes(gg, nullptr, &nodes));
    printf("  before end capture: A status %d deps %zu, %zu nodes\n", (int)cs, nd, nodes);
    fflush(stdout);
    hipGraph_t g;
    CK(hipStreamEndCapture(A, &g));
    printf("  end capture ok; instantiating\n");
    fflush(stdout);
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipMemset(out, 0, (size_t)N * L * L * 4));
    CK(hipGraphLaunch(ge, A));
    CK(hipStreamSynchronize(A));
    CK(hipMemcpy(got.data(), out, got.size() * 4, hipMemcpyDeviceToHost));
    const bool same = memcmp(got.data(), ref.data(), got.size() * 4) == 0;
    printf("  replay bit-identical to eager: %s\n", same ? "yes" : "NO");
    return same ? 0 : 2;
}
