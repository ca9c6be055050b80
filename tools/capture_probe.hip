// Minimal reproduction for the round-4 capture crash (profiles/r04dbg_160_graph_crash.txt): a stream capture that
// forks the capturing stream onto S internal streams and joins them back K times (once per pipelined engine
// operation), each fork/join carrying M chunks of kernels, as gd_engine.hip's for_chunks_hw does.
//   mode 0 ("shared"): ONE fork event and S join events, re-recorded at every fork / join (the engine's PipeRes)
//   mode 1 ("fresh"):  new events for every fork / join (created before the capture, one set per operation)
//   mode 2: mode 0's fork / join on a stream B that joined the capture through an event (ADMMState.init_concurrent's
//           side stream), B joined back at the end; mode 3: the same with kernels on the capturing stream meanwhile;
//   mode 6: mode 2 with the A -> B event destroyed right after B's wait (what torch's Stream.wait_stream does)
// Then hipStreamEndCapture, instantiate, launch twice, and check the result on the host.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/capture_probe tools/capture_probe.hip
//   tools/bin/capture_probe MODE K M [S=2] [KPC=3]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); fflush(stdout); exit(1); } } while (0)

__global__ void k_add(float* p, int n, float v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += v;
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0, K = argc > 2 ? atoi(argv[2]) : 8, M = argc > 3 ? atoi(argv[3]) : 9;
    const int S = argc > 4 ? atoi(argv[4]) : 2, KPC = argc > 5 ? atoi(argv[5]) : 3;
    const int n = 1 << 16;
    float* buf;
    CK(hipMalloc(&buf, (size_t)M * n * 4));
    CK(hipMemset(buf, 0, (size_t)M * n * 4));
    hipStream_t st, side[8];
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int i = 0; i < S; ++i) CK(hipStreamCreateWithFlags(&side[i], hipStreamNonBlocking));
    const int sets = mode == 1 ? K : 1;
    std::vector<hipEvent_t> fork(sets), join((size_t)sets * S);
    for (auto& e : fork) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : join) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // modes 2, 3: the fork / join happens on a stream B that joined the capture through an event (torch's side
    // stream of ADMMState.init_concurrent), B -> internal streams -> B, then A waits for B; mode 3 also launches
    // work on A while B's chunks run (the SubNet beside the init)
    // mode 4: as 2, but B is created after hipStreamBeginCapture (torch.cuda.Stream() inside the captured forward);
    // mode 5: as 2, with B and the internal streams used by eager work (a fork / join) before the capture
    hipStream_t B = nullptr;
    if (mode != 4) CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    hipEvent_t eAB, eBA;
    CK(hipEventCreateWithFlags(&eAB, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eBA, hipEventDisableTiming));
    if (mode == 5) {
        CK(hipEventRecord(eAB, st));
        CK(hipStreamWaitEvent(B, eAB, 0));
        CK(hipEventRecord(fork[0], B));
        for (int i = 0; i < S; ++i) {
            CK(hipStreamWaitEvent(side[i], fork[0], 0));
            hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, side[i], buf + (size_t)i * n, n, 0.0f);
            CK(hipEventRecord(join[i], side[i]));
            CK(hipStreamWaitEvent(B, join[i], 0));
        }
        CK(hipEventRecord(eBA, B));
        CK(hipStreamWaitEvent(st, eBA, 0));
        CK(hipDeviceSynchronize());
    }
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    if (mode == 4) CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    hipStream_t cap = st;
    if (mode >= 2) {
        CK(hipEventRecord(eAB, st));
        CK(hipStreamWaitEvent(B, eAB, 0));
        if (mode == 6) CK(hipEventDestroy(eAB));  // torch's Stream.wait_stream: a temporary event, destroyed at once
        cap = B;
    }
    for (int k = 0; k < K; ++k) {
        const int e = mode == 1 ? k : 0;
        hipStream_t st = cap;
        CK(hipEventRecord(fork[e], st));
        for (int i = 0; i < S; ++i) CK(hipStreamWaitEvent(side[i], fork[e], 0));
        for (int c = 0; c < M; ++c)
            for (int j = 0; j < KPC; ++j)
                hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, side[c % S], buf + (size_t)c * n, n, 1.0f);
        for (int i = 0; i < S; ++i) {
            CK(hipEventRecord(join[(size_t)e * S + i], side[i]));
            CK(hipStreamWaitEvent(st, join[(size_t)e * S + i], 0));
        }
    }
    if (mode >= 2) {
        if (mode == 3)
            for (int j = 0; j < KPC; ++j) hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, st, buf, n, 0.0f);
        CK(hipEventRecord(eBA, B));
        CK(hipStreamWaitEvent(st, eBA, 0));
    }
    printf("mode %d (%s) K=%d M=%d S=%d: captured, ending capture\n", mode,
           mode == 0 ? "shared events" : mode == 1 ? "fresh events" : mode == 2 ? "nested via stream B" :
           mode == 3 ? "nested + work on A" : mode == 4 ? "nested, B created during the capture" :
           mode == 5 ? "nested, streams used eagerly first" : "nested, the A->B event destroyed right after B's wait",
           K, M, S);
    fflush(stdout);
    hipGraph_t g;
    CK(hipStreamEndCapture(st, &g));
    size_t nodes = 0;
    CK(hipGraphGetNodes(g, nullptr, &nodes));
    printf("  end capture ok, %zu nodes; instantiating\n", nodes);
    fflush(stdout);
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    std::vector<float> h((size_t)M * n);
    CK(hipMemcpy(h.data(), buf, h.size() * 4, hipMemcpyDeviceToHost));
    const float want = 2.0f * K * KPC;
    long bad = 0;
    for (float v : h) bad += (v != want);
    printf("  replayed twice: %s (expected %.0f per element, %ld wrong)\n", bad ? "WRONG" : "ok", want, bad);
    return bad ? 2 : 0;
}
