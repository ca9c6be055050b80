// Minimal reproduction for the round-4 capture crash (profiles/r04dbg_160_graph_crash.txt): a stream capture that
// forks the capturing stream onto S internal streams and joins them back K times (once per pipelined engine
// operation), each fork/join carrying M chunks of kernels, as gd_engine.hip's for_chunks_hw does.
//   mode 0 ("shared"): ONE fork event and S join events, re-recorded at every fork / join (the engine's PipeRes)
//   mode 1 ("fresh"):  new events for every fork / join (created before the capture, one set per operation)
//   mode 2: mode 0's fork / join on a stream B that joined the capture through an event (ADMMState.init_concurrent's
//           side stream), B joined back at the end; mode 3: the same with kernels on the capturing stream meanwhile;
//   mode 6: mode 2 with the A -> B event destroyed right after B's wait (what torch's Stream.wait_stream does)
//   mode 7: mode 2's K fork / joins on B, B joined back to A, then K more on A itself onto the SAME internal streams
//           (the engine under capture: the init's chunks forked from the side stream, the iterations' from the
//           capturing stream, one set of capture streams); mode 8: the same in the opposite order (A first, then B)
//   mode 9: mode 7 with the internal streams CREATED after hipStreamBeginCapture (the engine's capture streams are
//           created at a thread's first pipelined operation under capture), so their first capture join is through
//           B; mode 10: the same creation with the first fork from A (mode 8's order)
//   mode 11: mode 2 with B joined back to A through a temporary event destroyed right after A's wait (torch's
//           Stream.wait_stream at ADMMState.join: the event was recorded on B, a stream that has forked streams)
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
    int rtv = 0;
    CK(hipRuntimeGetVersion(&rtv));
    printf("HIP runtime %d\n", rtv);
    float* buf;
    CK(hipMalloc(&buf, (size_t)M * n * 4));
    CK(hipMemset(buf, 0, (size_t)M * n * 4));
    hipStream_t st, side[8];
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const bool late = mode == 9 || mode == 10;
    if (!late)
        for (int i = 0; i < S; ++i) CK(hipStreamCreateWithFlags(&side[i], hipStreamNonBlocking));
    // PROBE_FRESH=1: modes >= 2 take a fresh event set per fork / join as well (the engine's ring of kCapSets sets)
    const bool fresh = mode == 1 || (std::getenv("PROBE_FRESH") && std::atoi(std::getenv("PROBE_FRESH")) == 1);
    const int sets = fresh ? 2 * K : 1;
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
    if (late)
        for (int i = 0; i < S; ++i) CK(hipStreamCreateWithFlags(&side[i], hipStreamNonBlocking));
    hipStream_t cap = st;
    if (mode >= 2) {
        CK(hipEventRecord(eAB, st));
        CK(hipStreamWaitEvent(B, eAB, 0));
        if (mode == 6) CK(hipEventDestroy(eAB));  // torch's Stream.wait_stream: a temporary event, destroyed at once
        cap = B;
    }
    const bool mixed = mode == 7 || mode == 8 || late;
    const bool a_first = mode == 8 || mode == 10;
    if (a_first) cap = st;
    for (int k = 0; k < (mixed ? 2 * K : K); ++k) {
        const int e = fresh ? k : 0;
        if (mixed && k == K) {  // switch the forking stream: B -> A (mode 7) or A -> B (mode 8)
            if (!a_first) {
                CK(hipEventRecord(eBA, B));
                CK(hipStreamWaitEvent(st, eBA, 0));
                cap = st;
            } else {
                cap = B;
            }
        }
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
    if (mode >= 2 && !(mixed && !a_first)) {
        if (mode == 3)
            for (int j = 0; j < KPC; ++j) hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, st, buf, n, 0.0f);
        if (mode == 11) {
            hipEvent_t tmp;
            CK(hipEventCreateWithFlags(&tmp, hipEventDisableTiming));
            CK(hipEventRecord(tmp, B));
            CK(hipStreamWaitEvent(st, tmp, 0));
            CK(hipEventDestroy(tmp));
        } else {
            CK(hipEventRecord(eBA, B));
            CK(hipStreamWaitEvent(st, eBA, 0));
        }
    }
    printf("mode %d%s (%s) K=%d M=%d S=%d: captured, ending capture\n", mode, fresh && mode != 1 ? " fresh" : "",
           mode == 0 ? "shared events" : mode == 1 ? "fresh events" : mode == 2 ? "nested via stream B" :
           mode == 3 ? "nested + work on A" : mode == 4 ? "nested, B created during the capture" :
           mode == 5 ? "nested, streams used eagerly first" : mode == 6 ? "nested, the A->B event destroyed right after B's wait" :
           mode == 7 ? "internal streams forked from B, then from A" : mode == 8 ? "internal streams forked from A, then from B" :
           mode == 9 ? "internal streams created in the capture, forked from B, then A" : mode == 10 ? "internal streams created in the capture, forked from A, then B" :
                        "nested, B joined to A by a temporary event destroyed after the wait",
           K, M, S);
    // every stream's capture state just before hipStreamEndCapture: status (0 none, 1 active, 2 invalidated), capture
    // id and the number of nodes its next captured operation would depend on (its unjoined tail)
    auto info = [&](const char* name, hipStream_t x) {
        hipStreamCaptureStatus cs;
        unsigned long long id = 0;
        hipGraph_t gg = nullptr;
        const hipGraphNode_t* deps = nullptr;
        size_t nd = 0;
        const hipError_t e = hipStreamGetCaptureInfo_v2(x, &cs, &id, &gg, &deps, &nd);
        printf("  %-8s err %d status %d id %llu graph %p deps %zu\n", name, (int)e, (int)cs, id, (void*)gg, nd);
    };
    info("A", st);
    if (B) info("B", B);
    for (int i = 0; i < S; ++i) {
        char nm[16];
        snprintf(nm, sizeof nm, "int%d", i);
        info(nm, side[i]);
    }
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
    const float want = 2.0f * K * KPC * (mixed ? 2 : 1);
    long bad = 0;
    for (float v : h) bad += (v != want);
    printf("  replayed twice: %s (expected %.0f per element, %ld wrong)\n", bad ? "WRONG" : "ok", want, bad);
    return bad ? 2 : 0;
}
