"""The round-4 capture crash's configuration on the current engine, with the side-stream guard lifted, and every
stream's capture state printed right before hipStreamEndCapture.

Unrolled_ADMM(n_iters=8, Gaussian, identity denoiser) at N x L^2 with the chunked runtime-planned init (fused init
off) on ADMMState.init_concurrent's side stream; GraphedForward captures with the chunks pipelined over the capturing
thread's capture streams (gd_set_capture_pipeline 2).  ``--guard 0`` keeps mode 2 for the side-stream init too (the
engine's Python guard sets 0 there); ``--guard 1`` is the shipped behaviour.  Before torch's capture_end the tool
prints, for the capturing stream and the side stream, hipStreamGetCaptureInfo_v2's status / id / dependency count,
and for the graph being captured its node count and its leaves (nodes with no successor).  Then it ends the capture,
replays, and checks the replay bit-for-bit against the eager forward.

usage: python tools/capture_info.py [--n 330] [--size 160] [--guard 0|1] [--chunks 6]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

_hip = None


def hip():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipStreamGetCaptureInfo_v2.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                                    ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_void_p),
                                                    ctypes.POINTER(ctypes.POINTER(ctypes.c_void_p)),
                                                    ctypes.POINTER(ctypes.c_size_t)]
        _hip.hipGraphGetNodes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
        _hip.hipGraphGetEdges.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(ctypes.c_size_t)]
        _hip.hipGraphNodeGetType.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    return _hip


def capture_info(name, handle):
    st, cid, g, n = ctypes.c_int(), ctypes.c_ulonglong(), ctypes.c_void_p(), ctypes.c_size_t()
    deps = ctypes.POINTER(ctypes.c_void_p)()
    err = hip().hipStreamGetCaptureInfo_v2(ctypes.c_void_p(handle), ctypes.byref(st), ctypes.byref(cid), ctypes.byref(g),
                                           ctypes.byref(deps), ctypes.byref(n))
    d = [deps[i] for i in range(n.value)] if err == 0 and n.value else []
    print(f"  {name:10s} err {err} status {st.value} id {cid.value} graph {(g.value or 0):#x} deps {n.value}", flush=True)
    return g.value or 0, set(d)


def graph_leaves(g):
    n = ctypes.c_size_t()
    hip().hipGraphGetNodes(ctypes.c_void_p(g), None, ctypes.byref(n))
    nodes = (ctypes.c_void_p * n.value)()
    hip().hipGraphGetNodes(ctypes.c_void_p(g), nodes, ctypes.byref(n))
    e = ctypes.c_size_t()
    hip().hipGraphGetEdges(ctypes.c_void_p(g), None, None, ctypes.byref(e))
    fr, to = (ctypes.c_void_p * e.value)(), (ctypes.c_void_p * e.value)()
    hip().hipGraphGetEdges(ctypes.c_void_p(g), fr, to, ctypes.byref(e))
    has_succ = {fr[i] for i in range(e.value)}
    leaves = [nodes[i] for i in range(n.value) if nodes[i] not in has_succ]
    types = {}
    for x in leaves:
        t = ctypes.c_int()
        hip().hipGraphNodeGetType(ctypes.c_void_p(x), ctypes.byref(t))
        types[t.value] = types.get(t.value, 0) + 1
    print(f"  graph: {n.value} nodes, {e.value} edges, {len(leaves)} leaves (by node type: {types})", flush=True)
    return set(leaves)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=330)
    ap.add_argument("--size", type=int, default=160)
    ap.add_argument("--guard", type=int, default=0)
    ap.add_argument("--chunks", type=int, default=6)
    args = ap.parse_args()
    from bench import build_model
    from gdeconv import _lib, engine
    from gdeconv.graphs import GraphedForward
    from gdeconv.synth import make_batch
    lib = _lib.load()
    N, L = args.n, args.size
    tgal = 2 * (L // 2 + 1) * L * 8
    lib.gd_set_chunk_bytes((N // args.chunks + 1) * tgal)
    lib.gd_set_fused_init(0)
    if not args.guard:  # the side-stream init keeps the caller's capture mode (2 under GraphedForward)
        orig = lib.gd_set_capture_pipeline

        def keep_mode(mode):
            if mode == 0 and torch.cuda.is_current_stream_capturing():
                return orig(2)
            return orig(mode)
        lib.gd_set_capture_pipeline = keep_mode
    dev = torch.device("cuda:0")
    obs, psf, alpha, _ = make_batch(N, L, seed=13, device=dev)
    m = build_model(8, "Gaussian", dev)
    m.Z = torch.nn.Identity()
    with torch.no_grad():
        eager = m(obs, psf, alpha)
    torch.cuda.synchronize()
    print(f"[info] eager forward done: {N} x {L}^2, chunked init in ~{args.chunks} chunks, guard {args.guard}", flush=True)
    orig_end = torch.cuda.CUDAGraph.capture_end

    def end_with_info(self):
        cur = torch.cuda.current_stream()
        g, d_cap = capture_info("capturing", cur.cuda_stream)
        for i, e in enumerate(engine.ADMMState._side_streams.values()):
            s = e[0] if isinstance(e, tuple) else e
            capture_info(f"side{i}", s.cuda_stream)
        if g:
            leaves = graph_leaves(g)
            print(f"  capturing stream's dependencies that are leaves: {len(d_cap & leaves)} of {len(d_cap)}; "
                  f"leaves outside them: {len(leaves - d_cap)}", flush=True)
        print("[info] ending the capture", flush=True)
        return orig_end(self)
    torch.cuda.CUDAGraph.capture_end = end_with_info
    gf = GraphedForward(m, obs, psf, alpha, clone=True)
    torch.cuda.synchronize()
    print("[info] captured and instantiated", flush=True)
    out = gf(obs, psf, alpha)
    torch.cuda.synchronize()
    print(f"[info] replay bit-identical to eager: {bool(torch.equal(out, eager))}", flush=True)


if __name__ == "__main__":
    main()
