"""bench.py's roofline objects from a stage profile (host logic only, no GPU): the
network line names its dominant kernel with the work of the fused x3h encoder /
decoder launches, and the PMC traffic of the block's dominant kernel is looked up
from the newest committed profile (profiles/*/pmc_traffic.json) under the current
kernel symbol."""
import os
import sys

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_net_roofline_names_the_fused_encoder_decoder():
    args = bench.parse_args(["--workload", "net"])
    stages = {"mlp_gen": (2.5, 2), "spectral_l1": (0.7, 12), "fft_inv": (0.98, 13)}
    r = bench.net_roofline(stages, args, 1)
    C, P = args.C, args.nlat * args.nlon
    work = 2 * P * C * ((73 + C) + (C + 73 + 73))
    assert r["kernel"] == "mlp_gen" and r["bound"] == "mfma"
    assert r["launches_per_step"] == 2
    assert abs(r["achieved"] - work / 2.5e-3 / 1e12) < 0.01
    assert r["engine"].startswith("x3h") and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3


def test_block_mlp_traffic_comes_from_a_committed_profile():
    traffic, src = bench.pmc_traffic("mlp_fused")
    assert traffic and src and os.path.exists(os.path.join(REPO, src))
    # the fused MLP's compulsory bytes (x1, residual, output: 3 x 1.06 GB) bound it below
    assert traffic > 3 * 256 * 721 * 1440 * 4
