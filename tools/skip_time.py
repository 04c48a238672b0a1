"""Time the inner-skip 1x1 conv (msfno_conv1x1, C = 256) alone at config 2's size and
check it against a torch fp32 reference.  MSFNO_SKIP_P=0 selects the one-tile-per-
workgroup kernel.  Prints one line: kernel, ms per call (HIP events), algorithmic GB/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..",
                                "modulated-spherical-fourier-neural-operator_amd"))
from msfno_amd import _native as N  # noqa: E402


def main():
    B, C, P = 1, 256, 721 * 1440
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(B, C, P, generator=g, device=dev)
    w = torch.randn(C, C, generator=g, device=dev) / 16
    b = torch.randn(C, generator=g, device=dev)
    out = torch.empty_like(x)
    ws = torch.empty(N.lib().msfno_conv1x1_workspace_size(B, C, C), dtype=torch.uint8, device=dev)
    s = N.stream_of(x.device)

    def call():
        N.check(N.lib().msfno_conv1x1(w.data_ptr(), b.data_ptr(), x.data_ptr(), out.data_ptr(), B,
                                      C, C, P, ws.data_ptr(), ws.numel(), s), "conv1x1")
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    ref = torch.einsum("oi,bip->bop", w, x) + b[None, :, None]
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    n = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    gbs = 2 * B * C * P * 4 / ms / 1e6
    print(f"skip P={os.environ.get('MSFNO_SKIP_P', '1')} ms={ms:.4f} algGB/s={gbs:.0f} "
          f"rel_err={err:.2e}", flush=True)


if __name__ == "__main__":
    main()
