"""Diagnostic: where the persistent fused MLP (MSFNO_MH_PERSIST=1) differs from the
per-tile kernel.  Runs the block in two child processes and reports the error by field,
tile ordinal within a half-workgroup, wave-local 16-pixel group and channel block."""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CASES = [("non-linear", 33, 64, 32, 1), ("non-linear", 90, 180, 45, 3), ("non-linear", 90, 180, 45, 12)]


def child(out):
    for d in (os.path.join(REPO, "tests"), REPO,
              os.path.join(REPO, "modulated-spherical-fourier-neural-operator_amd")):
        sys.path.insert(0, d)
    import torch
    from test_gpu_mlp_fused import _block, _case
    res = {}
    for i, case in enumerate(CASES):
        cfg, p, x, gamma, beta = _case(*case, seed=11)
        blk = _block(cfg, p, *case[1:4])
        with torch.no_grad():
            res[f"c{i}"] = blk(x.cuda(), gamma.cuda(), beta.cuda(), 0.7).cpu().numpy()
    np.savez(out, **res)


def main():
    tmp = os.environ.get("TMPDIR", "/tmp")
    outs = {}
    for mode in ("0", "1"):
        path = os.path.join(tmp, f"hp_diag_{mode}.npz")
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "child", path],
                           env=dict(os.environ, MSFNO_MH_PERSIST=mode), capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-3000:])
            sys.exit(1)
        outs[mode] = np.load(path)
    import torch  # noqa: F401  (device count for the grid below)
    cus = 256
    for i, case in enumerate(CASES):
        a = outs["0"][f"c{i}"]
        b = outs["1"][f"c{i}"]
        B, C = a.shape[:2]
        P = a.shape[2] * a.shape[3]
        d = np.abs(a - b).reshape(B, C, P)
        tpf = -(-P // 64)
        ntiles = B * tpf
        G = min(cus, -(-ntiles // 2))
        bad = d > 1e-4 * max(1.0, np.abs(a).max())
        print(f"case {case}: tiles {ntiles} grid {G} max-abs {d.max():.3e} bad {bad.mean():.4f}")
        # per tile
        tile_bad = np.zeros(ntiles)
        for z in range(B):
            for t in range(tpf):
                tile_bad[z * tpf + t] = bad[z, :, 64 * t:64 * t + 64].mean()
        tiles = np.arange(ntiles)
        half = tiles % 2
        k = tiles // (2 * G)
        for h in (0, 1):
            for kk in range(int(k.max()) + 1):
                sel = (half == h) & (k == kk)
                if sel.any():
                    print(f"  half {h} tile-ordinal {kk}: {sel.sum()} tiles, bad frac {tile_bad[sel].mean():.4f}")
        # by wave-local 16-pixel group and channel block (over all tiles)
        grp = np.zeros(4)
        for lw in range(4):
            cols = [64 * t + 16 * lw + j for t in range(tpf) for j in range(16) if 64 * t + 16 * lw + j < P]
            grp[lw] = bad[:, :, cols].mean()
        print("  by wave group:", np.round(grp, 4))
        print("  by channel block of 16:", np.round(bad.mean(axis=(0, 2)).reshape(16, 16).mean(axis=1), 3))
        print("  by pixel within 16:", np.round(np.array([bad[:, :, j::16].mean() for j in range(16)]), 3))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(sys.argv[2])
    else:
        main()
