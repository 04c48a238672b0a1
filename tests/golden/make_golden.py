"""Generate the golden fixtures under tests/golden/ from the REFERENCE block code.

Runs only in the build container (where /root/reference exists); its outputs
(small .npz files: inputs, parameters, outputs) are committed and travel to the
GPU box — this script and the reference do not.

How the reference is loaded (SURVEY.md §8(c) recipe): the four reference files
``MSFNO/Models/sfno/{contractions,activations,layers,sfnonet}.py`` are imported
with ``importlib`` under a synthetic package, after ``sys.modules`` stubs for
modules that are absent here and off the hot path:

* ``numpy.lib.arraypad`` (dead import at layers.py:9, removed in numpy 2.x),
* ``xarray`` (unused by the block), the FiLM generators ``..mae.maenet``,
  ``..gcn.gcn``, ``..vit.vit`` (sfnonet.py:23-25; out of scope),
* ``torch_harmonics`` — un-vendored and not installable offline; replaced by the
  oracle's restatement ``oracle/sht_ref.py`` (so the SHT itself is pinned by the
  known-answer tests, not by these fixtures).

Every other line executed (SpectralFilterLayer, SpectralAttentionS2,
SpectralConvS2, contractions, ComplexReLU, MLP, InstanceNorm, FiLM, block
wiring, the ×1e5 rescale recipe) is the reference's own code.

Usage:  python tests/golden/make_golden.py [--net | --gconv | --large]   (only the
        network / global_conv / large-size fixtures)
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/MSFNO/Models"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import sht_ref  # noqa: E402


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def load_reference():
    class _Dummy(torch.nn.Module):
        def __init__(self, *a, **k):
            super().__init__()

    _stub("numpy.lib.arraypad", pad=np.pad)
    _stub("xarray")
    th = _stub("torch_harmonics", RealSHT=sht_ref.RealSHT, InverseRealSHT=sht_ref.InverseRealSHT)
    th.quadrature = _stub("torch_harmonics.quadrature",
                          legendre_gauss_weights=sht_ref.legendre_gauss_weights)
    pkg = "refmsfno"
    for sub in ("", ".sfno", ".mae", ".gcn", ".vit"):
        m = _stub(pkg + sub)
        m.__path__ = []
    _stub(pkg + ".mae.maenet", ContextCast=_Dummy)
    _stub(pkg + ".gcn.gcn", GCN=_Dummy, GCN_custom=_Dummy)
    _stub(pkg + ".vit.vit", ViT=_Dummy)
    mods = {}
    for name in ("contractions", "activations", "layers", "sfnonet"):
        full = f"{pkg}.sfno.{name}"
        spec = importlib.util.spec_from_file_location(full, os.path.join(REF, "sfno", name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[full] = mod
        spec.loader.exec_module(mod)
        mods[name] = mod
    return mods


def build_ref_block(sfnonet, nlat, nlon, lmax, mmax, C, filter_type, filmed, grid,
                    inner_skip="linear", outer_skip="identity", mlp_mode="distributed",
                    out_grid=None):
    """out_grid=(nlat_out, nlon_out, grid_out) builds a resampling block like the
    reference's block 0 / block 11 (sfnonet.py:578-579)."""
    from functools import partial
    sht = sht_ref.RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid).float()
    ng, wg, gg = out_grid if out_grid is not None else (nlat, nlon, grid)
    isht = sht_ref.InverseRealSHT(ng, wg, lmax=lmax, mmax=mmax, grid=gg).float()
    # the reference's ad-hoc rescale (sfnonet.py:551-555)
    sht.weights = sht.weights * 1e5
    isht.pct = isht.pct / 1e5
    norm = partial(torch.nn.InstanceNorm2d, num_features=C, eps=1e-6, affine=True,
                   track_running_stats=False)
    cls = sfnonet.FourierNeuralOperatorBlock_Filmed if filmed else sfnonet.FourierNeuralOperatorBlock
    blk = cls(sht, isht, C, filter_type=filter_type, mlp_ratio=2.0, norm_layer=(norm, norm),
              inner_skip=inner_skip, outer_skip=outer_skip, mlp_mode=mlp_mode,
              spectral_layers=3, complex_activation="real", use_complex_kernels=True)
    return blk, sht, isht


def randomize_(blk, gen):
    """Re-randomise norm affine and biases so outputs are O(1) and every term matters."""
    with torch.no_grad():
        for name, p in blk.named_parameters():
            if name.startswith("norm") and name.endswith("weight"):
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=gen))
            elif name.endswith("bias"):
                p.copy_(0.05 * torch.randn(p.shape, generator=gen))


def main():
    mods = load_reference()
    sfnonet = mods["sfnonet"]
    cases = [
        # name, nlat, nlon, lmax, mmax, C, grid, B, out_grid
        ("c1", 32, 64, 32, 33, 8, "equiangular", 1, None),
        ("c1b2", 32, 64, 32, 33, 8, "equiangular", 2, None),
        ("lg", 24, 48, 24, 25, 16, "legendre-gauss", 1, None),
        ("mid", 91, 180, 45, 46, 16, "equiangular", 1, None),
        # resampling blocks: block-0 style (equiangular -> Gauss) and block-11 style
        ("down", 33, 64, 16, 17, 8, "equiangular", 1, (16, 32, "legendre-gauss")),
        ("up", 16, 32, 16, 17, 8, "legendre-gauss", 1, (33, 64, "equiangular")),
    ]
    wirings = {
        "middle": dict(inner_skip="linear", outer_skip="identity", mlp_mode="distributed"),
        "first": dict(inner_skip=None, outer_skip=None, mlp_mode="distributed"),
        "last": dict(inner_skip=None, outer_skip=None, mlp_mode="none"),
    }
    for (name, nlat, nlon, lmax, mmax, C, grid, B, out_grid) in cases:
        for filter_type in ("non-linear", "linear"):
            for filmed in (False, True):
                for wname, wiring in wirings.items():
                    if name == "down" and wname != "first":
                        continue
                    if name == "up" and wname != "last":
                        continue
                    if name not in ("c1", "down", "up") and wname != "middle":
                        continue
                    if name == "mid" and not filmed:
                        continue
                    seed = 1234
                    torch.manual_seed(seed)
                    blk, sht, isht = build_ref_block(sfnonet, nlat, nlon, lmax, mmax, C,
                                                     filter_type, filmed, grid,
                                                     out_grid=out_grid, **wiring)
                    gen = torch.Generator().manual_seed(seed + 1)
                    randomize_(blk, gen)
                    blk.eval()
                    x = torch.randn(B, C, nlat, nlon, generator=gen)
                    gamma = 0.1 * torch.randn(B, C, generator=gen)
                    beta = 0.1 * torch.randn(B, C, generator=gen)
                    scale = 0.7
                    with torch.no_grad():
                        y = blk(x, gamma, beta, scale) if filmed else blk(x)
                        a = sht(x)
                        xr = isht(a) if out_grid is None else None
                    full_sd = blk.state_dict()
                    # transform tables are recomputed by every consumer; keep only names
                    sd = {k: v.numpy() for k, v in full_sd.items()
                          if not k.endswith((".weights", ".pct"))}
                    ft = "nl" if filter_type == "non-linear" else "lin"
                    tag = f"{name}_{ft}_{'film' if filmed else 'plain'}_{wname}"
                    out = {
                        "meta_nlat": nlat, "meta_nlon": nlon, "meta_lmax": lmax, "meta_mmax": mmax,
                        "meta_C": C, "meta_B": B, "meta_grid": grid, "meta_filter": filter_type,
                        "meta_filmed": int(filmed), "meta_scale": scale, "meta_wiring": wname,
                        "x": x.numpy(), "gamma": gamma.numpy(), "beta": beta.numpy(),
                        "y": y.numpy(), "sht_x": a.numpy(),
                        "state_dict_keys": np.array(sorted(full_sd.keys())),
                    }
                    if out_grid is None:
                        out["isht_sht_x"] = xr.numpy()
                    else:
                        out["meta_out_nlat"], out["meta_out_nlon"], out["meta_out_grid"] = out_grid
                    for k, v in sd.items():
                        out["p__" + k] = v
                    path = os.path.join(HERE, tag + ".npz")
                    np.savez_compressed(path, **out)
                    print("wrote", path, y.shape, float(y.abs().max()))


def main_net():
    """The network around the block (sfnonet.py:406-686): encoder, pos_embed, a
    4-block stack (block 0 equiangular 33x64 -> Gauss 8x16, block 3 back), big
    skip, decoder — the reference's own FourierNeuralOperatorNet."""
    mods = load_reference()
    sfnonet = mods["sfnonet"]
    for filter_type in ("non-linear", "linear"):
        seed = 4321
        torch.manual_seed(seed)
        kw = dict(spectral_transform="sht", filter_type=filter_type, img_size=(33, 64),
                  scale_factor=4, in_chans=5, out_chans=5, embed_dim_sfno=16, num_layers=4,
                  spectral_layers=3)
        net = sfnonet.FourierNeuralOperatorNet("cpu", None, **kw)
        gen = torch.Generator().manual_seed(seed + 1)
        randomize_(net, gen)
        with torch.no_grad():  # O(1) outputs: non-trivial pos_embed, unit-gain encoder/decoder
            net.pos_embed.copy_(0.1 * torch.randn(net.pos_embed.shape, generator=gen))
            for name, p in net.named_parameters():
                if name.startswith(("encoder", "decoder")) and name.endswith("weight"):
                    p.copy_(torch.randn(p.shape, generator=gen) / p.shape[1] ** 0.5)
        net.eval()
        x = torch.randn(2, 5, 33, 64, generator=gen)
        with torch.no_grad():
            y = net(x)
        full_sd = net.state_dict()
        ft = "nl" if filter_type == "non-linear" else "lin"
        out = {"meta_kind": "net", "meta_filter": filter_type, "meta_nlat": 33, "meta_nlon": 64,
               "meta_scale_factor": 4, "meta_in_chans": 5, "meta_out_chans": 5, "meta_C": 16,
               "meta_num_layers": 4, "x": x.numpy(), "y": y.numpy(),
               "state_dict_keys": np.array(sorted(full_sd.keys()))}
        for k, v in full_sd.items():
            if not k.endswith((".weights", ".pct")):
                out["p__" + k] = v.numpy()
        path = os.path.join(HERE, "net", f"net_{ft}.npz")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        np.savez_compressed(path, **out)
        print("wrote", path, tuple(y.shape), float(y.abs().max()))


def main_global_conv():
    """FourierNeuralOperatorBlock_Filmed.global_conv(x, residual) (sfnonet.py:341-356)
    with residual != x, both filters, config-1 shapes, middle-block wiring."""
    mods = load_reference()
    sfnonet = mods["sfnonet"]
    for filter_type in ("non-linear", "linear"):
        seed = 777
        torch.manual_seed(seed)
        blk, sht, isht = build_ref_block(sfnonet, 32, 64, 32, 33, 8, filter_type, True,
                                         "equiangular")
        gen = torch.Generator().manual_seed(seed + 1)
        randomize_(blk, gen)
        blk.eval()
        x = torch.randn(2, 8, 32, 64, generator=gen)
        residual = 3.0 * torch.randn(2, 8, 32, 64, generator=gen)
        with torch.no_grad():
            y = blk.global_conv(x, residual)
            y_self = blk.global_conv(x, x)
        full_sd = blk.state_dict()
        ft = "nl" if filter_type == "non-linear" else "lin"
        out = {"meta_kind": "global_conv", "meta_filter": filter_type, "meta_nlat": 32,
               "meta_nlon": 64, "meta_lmax": 32, "meta_mmax": 33, "meta_C": 8,
               "meta_grid": "equiangular", "x": x.numpy(), "residual": residual.numpy(),
               "y": y.numpy(), "y_self": y_self.numpy(),
               "state_dict_keys": np.array(sorted(full_sd.keys()))}
        for k, v in full_sd.items():
            if not k.endswith((".weights", ".pct")):
                out["p__" + k] = v.numpy()
        path = os.path.join(HERE, "gconv", f"gconv_{ft}.npz")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        np.savez_compressed(path, **out)
        print("wrote", path, tuple(y.shape), float(y.abs().max()))


LARGE_CASES = [
    # tag, nlat, nlon, lmax, mmax, C, grid, filter, filmed, rows kept, channels kept
    # (SURVEY §8(c) "What pins results": mid-size LG C=64, the default network's inner
    # block, config 2 full size)
    ("lg121_c64_nl", 121, 240, 60, 61, 64, "legendre-gauss", "non-linear", True,
     (0, 30, 60, 90, 120), tuple(range(64))),
    ("lg121_c64_lin", 121, 240, 60, 61, 64, "legendre-gauss", "linear", True,
     (0, 30, 60, 90, 120), tuple(range(64))),
    ("inner120_c256_nl", 120, 240, 120, 121, 256, "legendre-gauss", "non-linear", False,
     (0, 40, 80, 119), tuple(range(8))),
    ("c2_721_c256_nl", 721, 1440, 360, 361, 256, "equiangular", "non-linear", True,
     (0, 180, 360, 540, 720), tuple(range(8))),
]


def main_large(only=None):
    """Reference blocks at the sizes that matter, built from a committed recipe
    (golden_util.param_recipe / recipe_normal) and stored as output rows x channels
    plus per-channel moments: middle-block wiring, B=1, scale 1."""
    from golden_util import moments, param_recipe, recipe_normal
    mods = load_reference()
    sfnonet = mods["sfnonet"]
    for (tag, nlat, nlon, lmax, mmax, C, grid, ft, filmed, rows, chans) in LARGE_CASES:
        if only and only not in tag:
            continue
        torch.manual_seed(0)
        blk, sht, isht = build_ref_block(sfnonet, nlat, nlon, lmax, mmax, C, ft, filmed, grid)
        out = {"meta_kind": "large", "meta_nlat": nlat, "meta_nlon": nlon, "meta_lmax": lmax,
               "meta_mmax": mmax, "meta_C": C, "meta_B": 1, "meta_grid": grid,
               "meta_filter": ft, "meta_filmed": int(filmed), "meta_scale": 1.0,
               "meta_wiring": "middle", "meta_x_seed": 9000 + C + nlat}
        names = sorted(n for n, _ in blk.named_parameters())
        with torch.no_grad():
            for i, (n, p) in enumerate(sorted(blk.named_parameters())):
                sigma, offset = param_recipe(n, tuple(p.shape), ft)
                seed = 100 + i
                p.copy_(recipe_normal(seed, p.shape, sigma, offset))
                out["r__" + n] = np.array([seed, sigma, offset], dtype=np.float64)
                out["s__" + n] = np.array(p.shape, dtype=np.int64)
        blk.eval()
        x = recipe_normal(out["meta_x_seed"], (1, C, nlat, nlon))
        gen = torch.Generator().manual_seed(77)
        gamma = 0.1 * torch.randn(1, C, generator=gen)
        beta = 0.1 * torch.randn(1, C, generator=gen)
        with torch.no_grad():
            y = blk(x, gamma, beta, 1.0) if filmed else blk(x)
        mean, std, mx = moments(y)
        r = torch.tensor(rows)
        c = torch.tensor(chans)
        out.update({"x_probe": x.reshape(-1)[:4096].numpy(), "gamma": gamma.numpy(),
                    "beta": beta.numpy(), "rows": r.numpy(), "chans": c.numpy(),
                    "rows_y": y[0][c][:, r].numpy(), "mom_mean": mean.numpy(),
                    "mom_std": std.numpy(), "mom_maxabs": mx.numpy(),
                    "state_dict_keys": np.array(sorted(blk.state_dict().keys()))})
        assert set(names) == {k[3:] for k in out if k.startswith("r__")}
        path = os.path.join(HERE, "large", tag + ".npz")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        np.savez_compressed(path, **out)
        print("wrote", path, tuple(y.shape), "max|y|", float(y.abs().max()),
              "std", float(y.std()))


if __name__ == "__main__":
    if "--net" in sys.argv:
        main_net()
    elif "--gconv" in sys.argv:
        main_global_conv()
    elif "--large" in sys.argv:
        main_large(sys.argv[sys.argv.index("--large") + 1] if len(sys.argv) > 2 else None)
    else:
        main()
        main_net()
        main_global_conv()
        main_large()
