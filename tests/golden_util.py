"""Helpers to read the committed golden fixtures (tests/golden/*.npz)."""
import glob
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(path):
    d = np.load(path, allow_pickle=False)
    meta = {k[5:]: d[k].item() for k in d.files if k.startswith("meta_")}
    params = {k[3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("p__")}
    arrays = {k: torch.from_numpy(d[k]) for k in d.files
              if not k.startswith(("meta_", "p__")) and d[k].dtype != np.dtype("<U1") and k != "state_dict_keys"}
    keys = [str(k) for k in d["state_dict_keys"]] if "state_dict_keys" in d.files else []
    return meta, params, arrays, keys


def wiring_cfg(meta):
    """(inner_skip, outer_skip, has_mlp) of the reference wiring stored in the fixture."""
    w = meta["wiring"]
    if w == "middle":
        return "linear", "identity", True
    if w == "first":
        return None, None, True
    return None, None, False


# ---- large fixtures (tests/golden/large/*.npz) -----------------------------------------
# Inputs and parameters at the sizes that matter are too big to commit, so they are
# stored as a recipe: numpy PCG64 standard normals (platform-independent, unlike torch's
# vectorised CPU normal fill) scaled and offset per tensor.  make_golden.py --large builds
# the reference block from the same recipe; the GPU tests rebuild the inputs from it.

def recipe_normal(seed, shape, sigma=1.0, offset=0.0):
    a = np.random.default_rng(int(seed)).standard_normal(tuple(int(s) for s in shape),
                                                         dtype=np.float32)
    if sigma != 1.0:
        a *= np.float32(sigma)
    if offset != 0.0:
        a += np.float32(offset)
    return torch.from_numpy(a)


def param_recipe(name, shape, filter_type):
    """(sigma, offset) of one block parameter: unit-gain weights so that every branch
    (spectral filter, inner skip, MLP) contributes O(1) to the output; norm affines
    near 1, small biases."""
    if name.startswith("norm") and name.endswith("weight"):
        return 0.1, 1.0
    if name.endswith("bias"):
        return 0.05, 0.0
    if name.startswith("filter_layer.filter.w"):
        if filter_type == "linear":       # (Cout, Cin, T, 2): sum over Cin complex terms
            return (2.0 * shape[1]) ** -0.5, 0.0
        return (2.0 * shape[0]) ** -0.5, 0.0  # (Cin, Cout, 2)
    return float(shape[1]) ** -0.5, 0.0   # 1x1 convs (Cout, Cin, 1, 1)


def load_large(path):
    """(meta, params, x, gamma, beta, expected): a large fixture with its recipe
    tensors rebuilt.  x is checked against the stored probe values."""
    d = np.load(path, allow_pickle=False)
    meta = {k[5:]: d[k].item() for k in d.files if k.startswith("meta_")}
    params = {}
    for k in d.files:
        if k.startswith("r__"):
            seed, sigma, offset = d[k]
            params[k[3:]] = recipe_normal(seed, d["s__" + k[3:]], sigma, offset)
    if meta["filter"] == "linear":  # buffers of SpectralConvS2 (layers.py:368-370)
        ii, jj = torch.tril_indices(meta["lmax"], meta["mmax"])
        params["filter_layer.filter.ii"], params["filter_layer.filter.jj"] = ii, jj
    x = recipe_normal(meta["x_seed"], (meta["B"], meta["C"], meta["nlat"], meta["nlon"]))
    probe = torch.from_numpy(d["x_probe"])
    assert torch.equal(x.reshape(-1)[:probe.numel()], probe), "recipe x differs from the fixture"
    exp = {k: torch.from_numpy(d[k]) for k in d.files if k.startswith(("rows_", "mom_"))}
    exp["rows"] = torch.from_numpy(d["rows"])
    exp["chans"] = torch.from_numpy(d["chans"])
    return meta, params, x, torch.from_numpy(d["gamma"]), torch.from_numpy(d["beta"]), exp


def moments(y):
    """Per-(batch, channel) mean, std and max-abs over the grid, fp64."""
    y = y.double()
    return (y.mean(dim=(-2, -1)), y.std(dim=(-2, -1)), y.abs().amax(dim=(-2, -1)))
