"""The weight-stationary inner skip (mlp_fused_h.hip: skip_ws_kernel, MSFNO_SKIP_WS=1, for
C = 256 with per-channel scales and P % 4 == 0) against the per-tile skip_h kernel
(the default), each in a child process (the switch is read once per process).

Both run the same x3h arithmetic (skip_h's per-field weight image, the same three fp16
MFMAs per k-step in the same order, the same epilogue), so the block outputs must agree
bit for bit.  Cases: a field count that puts field boundaries inside a workgroup's chunk
range (weights reloaded mid-stream), a ragged last chunk (P = 16200 = 506 x 32 + 8),
and a batch of one with more chunks than workgroups.
Reference: sfnonet.py:366-371 (inner skip), oracle/sfno_ref.py."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if __name__ == "__main__":
    _repo = os.path.dirname(HERE)
    for _d in (HERE, _repo, os.path.join(_repo, "modulated-spherical-fourier-neural-operator_amd")):
        sys.path.insert(0, _d)

import numpy as np  # noqa: E402
import pytest  # noqa: E402
import torch  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [("non-linear", 90, 180, 45, 3), ("linear", 45, 96, 23, 5), ("non-linear", 33, 64, 32, 1)]


def _native(case):
    from test_gpu_mlp_fused import _block, _case
    cfg, p, x, gamma, beta = _case(*case, seed=17)
    blk = _block(cfg, p, *case[1:4])
    with torch.no_grad():
        return blk(x.to(DEV), gamma.to(DEV), beta.to(DEV), 0.7).cpu()


def _in_child(path, ws):
    r = subprocess.run([sys.executable, os.path.abspath(__file__), path],
                       env=dict(os.environ, MSFNO_SKIP_WS=ws), cwd=HERE,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(path)


def test_weight_stationary_skip_equals_per_tile(tmp_path):
    a = _in_child(str(tmp_path / "tile.npz"), "0")
    b = _in_child(str(tmp_path / "ws.npz"), "1")
    for i, case in enumerate(CASES):
        y0 = torch.from_numpy(a[f"c{i}"])
        y1 = torch.from_numpy(b[f"c{i}"])
        err = (y1 - y0).abs().max().item()
        print(f"{case}: max-abs {err:.3e}, {(y1 != y0).sum().item()} differ")
        assert torch.isfinite(y1).all()
        assert torch.equal(y1, y0), (case, err)


if __name__ == "__main__":
    np.savez(sys.argv[1], **{f"c{i}": _native(c).numpy() for i, c in enumerate(CASES)})
