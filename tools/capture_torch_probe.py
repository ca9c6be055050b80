"""Bisect the capture crash between torch and the engine: the engine's chunked Gaussian init on a torch side stream
(chunks pipelined over the capture streams, gd_set_capture_pipeline(2)) and 8 iterations on the capturing stream,
captured with torch.cuda.graph, without the model around it.  tools/capture_engine_probe.hip runs the same stream
topology with plain HIP capture and does not crash.

    python tools/capture_torch_probe.py VARIANT [N=330] [L=160]
      prealloc : every buffer allocated before the capture (no allocator call inside it)
      sidealloc: zin allocated inside the capture on the side stream (the init's output, as ADMMState does)
      mainalloc: zin allocated inside the capture on the capturing stream
      main     : prealloc with the init on the capturing stream itself (its chunks forked from the origin)
      ext      : prealloc under torch.cuda.graph, the capturing and the side stream created with hipStreamCreateWithFlags
                 (non-blocking) through ctypes and wrapped as torch.cuda.ExternalStream
      pure     : prealloc; every stream, event and the capture itself through ctypes HIP calls (torch only allocates the
                 buffers): the C++ probe's call sequence from inside a torch process
      hipcap   : prealloc, captured with hipStreamBeginCapture / hipStreamEndCapture (ctypes) on a torch stream
                 instead of torch.cuda.graph (torch's streams, not torch's CUDAGraph)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))

import torch  # noqa: E402


def main():
    variant = sys.argv[1]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 330
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 160
    from gdeconv import _lib
    from gdeconv.synth import make_batch
    lib = _lib.load()
    dev = torch.device("cuda:0")
    n_it, h = 8, 48
    obs, psf, alpha, _ = make_batch(N, L, seed=13, device=dev)
    psf = psf.reshape(N, psf.shape[-2], psf.shape[-1]).contiguous()
    h = psf.shape[-1]
    alpha = alpha.reshape(-1).float().contiguous()
    rho1 = torch.full((N, n_it), 0.7, device=dev)
    rho2 = torch.full((N, n_it), 0.9, device=dev)
    tgal = 2 * (L // 2 + 1) * L * 8
    lib.gd_set_chunk_bytes((N // 6 + 1) * tgal)
    lib.gd_set_fused_init(0)
    lib.gd_set_capture_pipeline(2)
    state = torch.empty(lib.gd_admm_state_bytes(N, L, L, 0), dtype=torch.uint8, device=dev)
    ws = torch.empty(lib.gd_workspace_bytes(N, L, L) + 16, dtype=torch.uint8, device=dev)
    out = torch.empty(N, L, L, device=dev)
    zin_pre = torch.empty(N, L, L, device=dev)
    y = obs.reshape(N, L, L).float().contiguous()
    hip = ctypes.CDLL("libamdhip64.so")

    def ext_stream():
        h = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0
        return torch.cuda.ExternalStream(h.value)
    side = ext_stream() if variant == "ext" else torch.cuda.Stream()
    S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731

    def forward(capturing):
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(main if variant == "main" else side):
            zin = torch.empty(N, L, L, device=dev) if (capturing and variant == "sidealloc") else zin_pre
            rc = lib.gd_admm_init(y.data_ptr(), psf.data_ptr(), h * h, h, h, alpha.data_ptr(), 1, None, 0, 0, N, L, L,
                                  state.data_ptr(), zin.data_ptr(), ws.data_ptr(), S())
            assert rc == 0, lib.gd_last_error()
        main.wait_stream(side)
        if capturing and variant == "mainalloc":
            z2 = torch.empty(N, L, L, device=dev)
            z2.copy_(zin)
            zin = z2
        for it in range(n_it):
            last = it == n_it - 1
            dst = out if last else zin
            rc = lib.gd_admm_iter(y.data_ptr(), zin.data_ptr(), dst.data_ptr(), alpha.data_ptr(), 1,
                                  rho1[:, it:].data_ptr(), n_it, rho2[:, it:].data_ptr(), n_it,
                                  None if last else rho2[:, it + 1:].data_ptr(), n_it, 0, it, int(last), N, L, L,
                                  state.data_ptr(), ws.data_ptr(), S())
            assert rc == 0, lib.gd_last_error()
        return out

    if variant == "pure":
        return pure(lib, hip, N, L, n_it, h, y, psf, alpha, rho1, rho2, state, ws, out, zin_pre)
    with torch.no_grad():
        ref = forward(False).clone()
    torch.cuda.synchronize()
    print(f"[torch probe] {variant}: eager done ({N} x {L}^2); capturing", flush=True)
    if variant == "hipcap":
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        graph, ge = ctypes.c_void_p(), ctypes.c_void_p()
        with torch.no_grad(), torch.cuda.stream(cs):
            assert hip.hipStreamBeginCapture(ctypes.c_void_p(cs.cuda_stream), 0) == 0
            forward(True)
            rc = hip.hipStreamEndCapture(ctypes.c_void_p(cs.cuda_stream), ctypes.byref(graph))
        assert rc == 0, rc
        print("[torch probe] end capture ok", flush=True)
        assert hip.hipGraphInstantiate(ctypes.byref(ge), graph, None, None, ctypes.c_size_t(0)) == 0
        out.zero_()
        torch.cuda.synchronize()
        assert hip.hipGraphLaunch(ge, ctypes.c_void_p(cs.cuda_stream)) == 0
    else:
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(g, stream=ext_stream() if variant == "ext" else None):
            forward(True)
        print("[torch probe] end capture ok", flush=True)
        out.zero_()
        g.replay()
    torch.cuda.synchronize()
    print(f"[torch probe] replay bit-identical to eager: {bool(torch.equal(out, ref))}", flush=True)


def pure(lib, hip, N, L, n_it, h, y, psf, alpha, rho1, rho2, state, ws, out, zin):
    vp = ctypes.c_void_p
    A, B = vp(), vp()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(A), 1) == 0 and hip.hipStreamCreateWithFlags(ctypes.byref(B), 1) == 0
    eAB, eBA = vp(), vp()
    assert hip.hipEventCreateWithFlags(ctypes.byref(eAB), 2) == 0 and hip.hipEventCreateWithFlags(ctypes.byref(eBA), 2) == 0

    def forward():
        assert hip.hipEventRecord(eAB, A) == 0 and hip.hipStreamWaitEvent(B, eAB, 0) == 0
        rc = lib.gd_admm_init(y.data_ptr(), psf.data_ptr(), h * h, h, h, alpha.data_ptr(), 1, None, 0, 0, N, L, L,
                              state.data_ptr(), zin.data_ptr(), ws.data_ptr(), B)
        assert rc == 0, lib.gd_last_error()
        assert hip.hipEventRecord(eBA, B) == 0 and hip.hipStreamWaitEvent(A, eBA, 0) == 0
        for it in range(n_it):
            last = it == n_it - 1
            dst = out if last else zin
            rc = lib.gd_admm_iter(y.data_ptr(), zin.data_ptr(), dst.data_ptr(), alpha.data_ptr(), 1,
                                  rho1[:, it:].data_ptr(), n_it, rho2[:, it:].data_ptr(), n_it,
                                  None if last else rho2[:, it + 1:].data_ptr(), n_it, 0, it, int(last), N, L, L,
                                  state.data_ptr(), ws.data_ptr(), A)
            assert rc == 0, lib.gd_last_error()
    torch.cuda.synchronize()
    forward()
    assert hip.hipStreamSynchronize(A) == 0
    ref = out.clone()
    print("[torch probe] pure: eager done; capturing", flush=True)
    assert hip.hipStreamBeginCapture(A, 0) == 0
    forward()
    graph, ge = vp(), vp()
    rc = hip.hipStreamEndCapture(A, ctypes.byref(graph))
    assert rc == 0, rc
    print("[torch probe] end capture ok", flush=True)
    assert hip.hipGraphInstantiate(ctypes.byref(ge), graph, None, None, ctypes.c_size_t(0)) == 0
    out.zero_()
    torch.cuda.synchronize()
    assert hip.hipGraphLaunch(ge, A) == 0 and hip.hipStreamSynchronize(A) == 0
    print(f"[torch probe] replay bit-identical to eager: {bool(torch.equal(out, ref))}", flush=True)


if __name__ == "__main__":
    main()
