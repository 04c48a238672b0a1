"""Raw-buffer addressing of the fused MLP kernels (round 6): mlp_fused_h_kernel (the
block MLP: x1, residual, output) and mlp_gen_h_kernel (the encoder / decoder: x, x2,
addend, output) address their strided fp32 planes through buffer resources with 32-bit
lane offsets instead of 64-bit per-access address arithmetic.  The encoder's channels
past Cin and the decoder's output rows past Cout rely on the buffer range check (lane
offset past the plane -> read 0 / store dropped).  The arithmetic is unchanged, so the
outputs with buffer addressing (MSFNO_MH_BUF=1 MSFNO_MG_BUF=1; the block MLP's default is
64-bit addressing since it measured faster, the decoder's is buffer addressing) must equal
those of the 64-bit-address kernels (both 0) bit for bit.  Each side runs in a child process:
the switches are read once per process."""
import os
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu
DEV = "cuda"

# block cases (filter, nlat, nlon, lmax, B, wide): P % 64 != 0 (ragged last tile), two fields
BLOCKS = [("non-linear", 90, 180, 45, 2, False), ("linear", 45, 96, 23, 1, False)]
# MLP cases of tests/test_gpu_mlp_gen.py: the encoder at P % 4 != 0 (tile kernel, Cin 73:
# channels 73..95 read through the range check), the decoder (x2, rows 73..79 dropped)
MLPS = [(73, 0, 256, 256, 3001, 2, "broadcast", True), (256, 73, 256, 73, 2145, 2, None, False),
        (256, 73, 256, 73, 1000, 1, "batched", True)]


def _outputs():
    sys.path.insert(0, HERE)
    from test_gpu_mlp_gen import _run
    from test_gpu_x3h import _gpu
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    outs = [_gpu(c) for c in BLOCKS]
    outs += [_run(*c, seed=i)[0] for i, c in enumerate(MLPS)]
    return outs


def _child(tmp_path, buf):
    dump = tmp_path / f"buf{buf}.pt"
    env = dict(os.environ, MSFNO_MH_BUF=buf, MSFNO_MG_BUF=buf)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), str(dump)], env=env, cwd=HERE,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(dump, weights_only=True)


def test_buffer_addressing_equals_64bit_addressing(tmp_path):
    got = _child(tmp_path, "1")
    ref = _child(tmp_path, "0")
    for name, a, b in zip([str(c) for c in BLOCKS + MLPS], got, ref):
        nd = (a != b).sum().item()
        print(f"{name}: {nd} of {a.numel()} differ, max-abs {(a - b).abs().max().item():.3e}")
        assert torch.isfinite(a).all() and nd == 0, name


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(HERE))
    import conftest  # noqa: F401  (puts the package on sys.path)
    torch.save(_outputs(), sys.argv[1])
