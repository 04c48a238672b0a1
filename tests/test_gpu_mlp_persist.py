"""The persistent two-phase fused MLP (mlp_fused_h.hip: mlp_fused_hp_kernel,
MSFNO_MH_PERSIST=1) against the one-workgroup-per-tile kernel (the default), each in a
child process (the switch is read once per process) on batches that give every half-workgroup several
tiles (tile staging, the lag-1 slice stream across tile boundaries, the boundary
epilogue), a grid whose last workgroup has only one half busy, and a ragged last tile;
and the persistent path against the oracle at the many-tile size.

Reference arithmetic: sfnonet.py:376-382 and layers.py:161-168 (oracle/sfno_ref.py).
Bar: max-abs < 2e-5 * max(1, |y|) between the kernels (same x3h arithmetic, different
schedule), 1e-4 * max(1, |y|) against the oracle."""
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

from oracle import sfno_ref  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (filter, nlat, nlon, lmax, B): 12 x 254 tiles (about six per half on 256 CUs);
# 33 tiles (17 workgroups, the last with one half idle); 4 x 68 tiles, ragged (P = 4320)
CASES = [("non-linear", 90, 180, 45, 12), ("non-linear", 33, 64, 32, 1),
         ("linear", 45, 96, 23, 4)]


def _native(case):
    from test_gpu_mlp_fused import _block, _case
    cfg, p, x, gamma, beta = _case(*case, seed=11)
    blk = _block(cfg, p, *case[1:4])
    with torch.no_grad():
        return blk(x.to(DEV), gamma.to(DEV), beta.to(DEV), 0.7).cpu()


def _in_child(path, persist):
    r = subprocess.run([sys.executable, os.path.abspath(__file__), path],
                       env=dict(os.environ, MSFNO_MH_PERSIST=persist), cwd=HERE,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(path)


def test_persistent_equals_per_tile(tmp_path):
    other = _in_child(str(tmp_path / "per_tile.npz"), "0")
    mine = _in_child(str(tmp_path / "persistent.npz"), "1")
    for i, case in enumerate(CASES):
        y = torch.from_numpy(mine[f"c{i}"])
        y0 = torch.from_numpy(other[f"c{i}"])
        assert torch.isfinite(y).all()
        err = (y - y0).abs().max().item()
        print(f"{case}: max-abs {err:.3e} |y|max {y0.abs().max():.3f}")
        assert err < 2e-5 * max(1.0, y0.abs().max().item()), (case, err)


def test_persistent_many_tiles_matches_oracle(tmp_path):
    from test_gpu_mlp_fused import _case
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    case = CASES[0]
    cfg, p, x, gamma, beta = _case(*case, seed=11)
    y = torch.from_numpy(_in_child(str(tmp_path / "persistent.npz"), "1")["c0"])
    sht, isht = sfno_ref.make_transforms(case[1], case[2], case[3], case[3] + 1)
    with torch.no_grad():
        want = sfno_ref.block_forward(p, x, sht, isht, cfg, gamma, beta, 0.7)
    err = (y - want).abs().max().item()
    print(f"{case}: max-abs {err:.3e} |y|max {want.abs().max():.3f}")
    assert err < 1e-4 * max(1.0, want.abs().max().item())


if __name__ == "__main__":
    np.savez(sys.argv[1], **{f"c{i}": _native(c).numpy() for i, c in enumerate(CASES)})
