"""Drive the config-2 SHT pair (721x1440, lmax 360, C=256) for kernel profiling."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "modulated-spherical-fourier-neural-operator_amd")]
import torch  # noqa: E402

from msfno_amd.harmonics import InverseRealSHT, RealSHT  # noqa: E402

f = RealSHT(721, 1440, lmax=360, mmax=361).float().cuda()
g = InverseRealSHT(721, 1440, lmax=360, mmax=361).float().cuda()
x = torch.randn(1, 256, 721, 1440, device="cuda")
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    a = f(x)
    y = g(a)
torch.cuda.synchronize()
print("ok", float(y.abs().max()))
