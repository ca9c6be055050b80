"""HIP-graph capture of a whole forward (serving the unrolled model).

The reference runs every forward eagerly from Python (``test.py:237``).  At LSST stamp size (48^2,
a few hundred galaxies) one ``Unrolled_ADMM`` forward is a chain of ~60 short launches - SubNet,
OTF, init_l2, 8 x (denoiser, spectral iteration) - and the host, not the GPU, sets the pace.
``GraphedForward`` records the forward once into a ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm)
and replays it: the engine's C ABI enqueues on torch's current stream and allocates nothing of its
own.  Under capture the engine runs an operation's Infinity-Cache chunks in sequence unless the caller
opts in (``gd_set_capture_pipeline``, per host thread); ``GraphedForward`` opts in (``pipeline=True``), since
it enqueues from the capturing stream itself: the chunks then fork onto capture streams of this host thread
(never the internal streams other threads' eager calls use), a fork / join per operation with its own
captured event set.  An init that ``ADMMState.init_concurrent`` runs on a side stream keeps its chunks serial
there on HIP runtimes before 7.2: a fork from a stream that joined the capture through an event segfaults inside
hipStreamEndCapture on the ROCm 7.0 runtime PyTorch bundles, with or without the engine (``tools/capture_probe.hip``
mode 2; ROCm 7.2's runtime captures it; ``profiles/r06_capture_rootcause.txt``).
A mode the caller set with ``gd_set_capture_pipeline`` before constructing is kept.  A server whose other host
threads keep launching work while one thread captures passes ``capture_error_mode="thread_local"`` (torch's
default "global" mode invalidates the capture on another thread's potentially unsafe call).

    g = GraphedForward(model, obs, psf, alpha)     # shapes fixed at capture
    rec = g(obs2, psf2, alpha2)                    # copies inputs in, replays, returns the output

The returned tensor is the graph's static output buffer (overwritten by the next replay) unless
``clone=True``.
"""
import torch


class GraphedForward:
    def __init__(self, model, *example, warmup=2, clone=False, pipeline=True, capture_error_mode="global"):
        for t in example:
            if not (torch.is_tensor(t) and t.is_cuda):
                raise ValueError("GraphedForward captures device tensors only")
        self.model = model
        self.clone = clone
        self.static_in = [t.detach().clone() for t in example]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(warmup):  # first calls build caches (folded BN, workspaces, MIOpen plans)
                model(*self.static_in)
        torch.cuda.current_stream().wait_stream(side)
        from . import _lib
        lib = _lib.load()
        prev = lib.gd_set_capture_pipeline(2 if pipeline else 0)
        if prev != -1:                      # the caller chose a mode for this thread: keep it
            lib.gd_set_capture_pipeline(prev)
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.no_grad(), torch.cuda.graph(self.graph, capture_error_mode=capture_error_mode):
                self.static_out = model(*self.static_in)
        finally:
            lib.gd_set_capture_pipeline(prev)

    def __call__(self, *inputs):
        if len(inputs) != len(self.static_in):
            raise ValueError(f"expected {len(self.static_in)} inputs, got {len(inputs)}")
        for dst, src in zip(self.static_in, inputs):
            if src.shape != dst.shape:
                raise ValueError(f"input shape {tuple(src.shape)} differs from the captured {tuple(dst.shape)}")
            if src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out.clone() if self.clone else self.static_out

    def replay(self):
        """Re-run on whatever the static inputs (``self.static_in``) hold."""
        self.graph.replay()
        return self.static_out


__all__ = ["GraphedForward"]
