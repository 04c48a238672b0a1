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
