"""Runs tools/probes/stream_mix.hip: achieved TB/s of 1R/1W (copy), 2R/1W and 4R/3W float4 streams
at the masked Adam's size (2M x 59 floats per stream)."""
import ctypes as C
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "libstream_mix.so"))
n = 2_000_000 * 59 // 4 * 4
bufs = [torch.randn(n, device="cuda") for _ in range(7)]
stream = torch.cuda.current_stream().cuda_stream
for R, W in ((1, 1), (2, 1), (4, 3)):
    ins = (C.c_void_p * R)(*[b.data_ptr() for b in bufs[:R]])
    outs = (C.c_void_p * W)(*[b.data_ptr() for b in bufs[R:R + W]])
    dins = torch.tensor([b.data_ptr() for b in bufs[:R]], dtype=torch.int64, device="cuda")
    douts = torch.tensor([b.data_ptr() for b in bufs[R:R + W]], dtype=torch.int64, device="cuda")
    for grid in (2048, 8192, (n // 4 + 511) // 512):
        def go():
            assert lib.stream_mix(R, W, C.c_void_p(dins.data_ptr()), C.c_void_p(douts.data_ptr()), n, grid,
                                  C.c_void_p(stream)) == 0
        for _ in range(3):
            go()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            go()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"R{R}/W{W} grid {grid}: {ms * 1e3:.1f} us, {(R + W) * 4 * n / (ms * 1e-3) / 1e12:.2f} TB/s", flush=True)
