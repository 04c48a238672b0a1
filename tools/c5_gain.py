"""Config-5 trajectory scan: |y|max and per-step change over 112 steps for a few
decoder gains (picks a gain whose state keeps moving at O(1) without blowing up)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import conftest  # noqa: F401,E402
import torch  # noqa: E402

from msfno_amd.rollout import Rollout  # noqa: E402
from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed  # noqa: E402

DEV = "cuda"
for gain in [float(a) for a in sys.argv[1:]]:
    steps, ch = 112, 73
    torch.manual_seed(51)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=(721, 1440), in_chans=ch,
                                          out_chans=ch, embed_dim_sfno=256, num_layers=12,
                                          filter_type="non-linear", spectral_layers=3).eval()
    with torch.no_grad():
        for k, v in net.decoder.state_dict().items():
            if k.endswith("weight"):
                v.mul_(gain)
    net = net.to(DEV)
    g = torch.Generator(device=DEV).manual_seed(52)
    means = torch.randn(1, ch, 1, 1, generator=g, device=DEV)
    stds = torch.rand(1, ch, 1, 1, generator=g, device=DEV) + 0.5
    x0 = torch.randn(1, ch, 721, 1440, generator=g, device=DEV) * stds + means
    film = 0.1 * torch.randn(1, 2, 1, 256, generator=g, device=DEV)
    prev = None
    with torch.no_grad():
        for i, y in Rollout(net, means, stds, film=film, graph=True).run(x0, steps):
            if i % 16 == 0 or i == steps - 1:
                mv = (y - prev).abs().max().item() if prev is not None else float("nan")
                print(f"gain {gain}: step {i} |y|max {y.abs().max().item():.3e} change {mv:.3e}",
                      flush=True)
            prev = y.clone()
