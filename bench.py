"""SFNO-Block forward throughput on MI355X (BASELINE.json metric / config 2).

Workload (one "step"): one SFNO-Block forward — FourierNeuralOperatorBlock_Filmed
with the reference-default non-linear spectral filter, middle-block wiring
(inner skip 1x1 conv, outer identity skip, MLP ratio 2), InstanceNorm eps 1e-6,
FiLM on — over one synthetic 721x1440x256 field per GPU (x ~ N(0,1), seed 0),
lmax=360/mmax=361 equiangular SHT with the reference's ×1e5 rescale, random
init weights of that architecture (reference init recipe, seed 1).

Multi-GPU: one process per GPU.  ``python bench.py --gpus N`` (N > 1, no
WORLD_SIZE in the environment) starts the N rank processes itself before any
GPU call (children, never exec; the reference's own launch is mp.spawn,
MSFNO/main.py:1149-1156); under torchrun the ranks come from the environment and
--gpus must equal WORLD_SIZE.  "scaling": "weak" (batch fields per GPU):
  --parallel latband (the N>1 default): ONE batch of batch*N fields (N=8: the
      config-4 batch of 8) is latitude-band sharded over the N ranks
      (SURVEY.md §8e): two RCCL all-to-alls and two small all-gathers per block
      forward (msfno_amd.sfno.LatBandBlock), pipelined over --band-chunks
      sub-batches so one sub-batch's exchange overlaps another's compute.  The
      replica number (below) is printed beside it as the comm-free upper bound.
  --parallel replicas: each rank runs its own field batch through the
      whole-field block; no data-path collective.
The timed region is bracketed by barrier + synchronize and the max over ranks
is used.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (timed
with hipEvents on the block's stream over the timed region) and the oracle's
CPU timing on a bounded sample (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "modulated-spherical-fourier-neural-operator_amd")
for _p in (REPO, PKG_DIR):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 MFMA 157.3 TF (spec)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 MFMA ~2.5 PF dense (spec)
# fp32 GEMMs on the "x6" engine (csrc/gemm_x6.hip): six bf16 MFMAs per fp32 product
# block (exact three-term operand split), so their roof is the bf16 peak / 6
PEAK_X6_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6.0
# the "x3h" engine (default; csrc/mlp_fused_h.hip, gemm_x6c.hip gemm_x3c, gemm_x6.hip
# gemm_x3): fp32 as two fp16 terms, three fp16 MFMAs per product (fp16 dense MFMA
# peak = the bf16 one, MI355X_MICROARCH.md), so the roof is 2.5 PF / 3
PEAK_FP16_MFMA_TFLOPS = 2500.0
PEAK_X3H_TFLOPS = PEAK_FP16_MFMA_TFLOPS / 3.0
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


# stages that run on the block's side stream (concurrent with the SHT)
SIDE_STAGES = {"inner_skip"}
# stage -> kernel symbol in the rocprofv3 summaries (profiles/<tag>/kernel_stats.csv);
# fc1 (bias + GELU epilogue) and fc2 (bias + residual) are the only launches of their
# template instantiations in the block (x6 engine, 256x256 tiles; f32 engine kept
# for MSFNO_GEMM=f32)
STAGE_KERNEL_X6 = {
    # fc1: x1 planes (from the inverse FFT) by LDS-DMA, bias + GELU, h written as
    # bf16x3 planes (EPI 133; two-stage DMA ring)
    "mlp_fc1": "void msfno::gemm_x6p_kernel<133, 2, 8, 256>(msfno::GemmParams)",
    # fc2: h planes staged by LDS-DMA (x6p), bias + outer skip (EPI 3)
    "mlp_fc2": "void msfno::gemm_x6p_kernel<3, 2, 8, 256>(msfno::GemmParams)",
    # inner skip: fp32 x split in-kernel (gemm_x6, bias epilogue); the plane form
    # (MSFNO_SKIP_PLANES=1) is gemm_x6p_kernel<1, 2, 8, 256>
    "inner_skip": "void msfno::gemm_x6_kernel<256, 256, 4, 2, true, 1, false>(msfno::GemmParams)",
    # fc1 -> GELU -> fc2 in one kernel, hidden activation on-chip (csrc/mlp_fused.hip)
    "mlp_fused": "void msfno::(anonymous namespace)::mlp_fused_kernel<1, 0, 0, 2, 0>"
                 "(msfno::(anonymous namespace)::MlpFusedParams)",
}
STAGE_KERNEL_F32 = {
    "mlp_fc1": "void msfno::gemm_f32_kernel<128, 256, 16, true, 5>(msfno::GemmParams)",
    "mlp_fc2": "void msfno::gemm_f32_kernel<256, 128, 16, true, 3>(msfno::GemmParams)",
}
# x3h engine: the fused MLP, the inner skip (fp32 x, bias epilogue) and the spectral
# MLP chain; the unfused fc1 / fc2 pair stays on x6
STAGE_KERNEL_X3H = dict(STAGE_KERNEL_X6, **{
    # inner skip at C = 256: the persistent pipelined skip (skip_h for P % 4 != 0,
    # MSFNO_SKIP_H=0: gemm_x3)
    "inner_skip": "msfno::(anonymous namespace)::skip_hp_kernel("
                  "msfno::(anonymous namespace)::SkipHPParams)",
    # (paired MFMA triples since round 6; the profiles before it name the same tiling
    # and addressing <2, false>, same HBM traffic)
    "mlp_fused": ("void msfno::(anonymous namespace)::mlp_fused_h_kernel<2, false, false, true>"
                  "(msfno::(anonymous namespace)::MlpHParams)",
                  "void msfno::(anonymous namespace)::mlp_fused_h_kernel<2, false>"
                  "(msfno::(anonymous namespace)::MlpHParams)"),
    "legendre_fwd": "void msfno::(anonymous namespace)::legendre_x3f_kernel<3>("
                    "msfno::(anonymous namespace)::X3FParams)",
    "legendre_inv": "msfno::(anonymous namespace)::legendre_x3r_kernel("
                    "msfno::(anonymous namespace)::X3DParams)",
})
# the network line (config 3): one encoder and one decoder launch per step, default
# kernels of the x3h engine at 721 x 1440 (their PMC bytes are summed per step)
STAGE_KERNEL_X3H["mlp_gen"] = (
    "void msfno::(anonymous namespace)::mlp_gen_hp_kernel<3, 16, true, 4, 2>"
    "(msfno::(anonymous namespace)::MlpGParams)",
    "void msfno::(anonymous namespace)::mlp_gen_h_kernel<11, 5, false, true>"
    "(msfno::(anonymous namespace)::MlpGParams)")

# the linear filter's weight stream at batch 1 (any engine)
STAGE_KERNEL_LINEAR = {
    "linear_contract": "void msfno::compl_contract_dma_kernel<2>(float const*, float const*, "
                       "float*, int, int, long, int)",
}
X6_STAGES = {"mlp_fc1", "mlp_fc2", "inner_skip", "mlp_fused"}
X6_SPEC_STAGES = {"spectral_l0", "spectral_l1", "spectral_l2", "spectral_out"}
X3H_STAGES = {"inner_skip", "mlp_fused", "mlp_gen"} | X6_SPEC_STAGES


def leg_x3h():
    """The Legendre GEMMs run on the x3h engine (legendre_x3.hip) unless MSFNO_LEG_X3=0."""
    e = os.environ.get("MSFNO_LEG_X3")
    return e == "1" if e is not None else x3h_engine()


def x3h_engine():
    """The x3h engine is the library default (mlp_fused_h.hip mlp_fused_h_env:
    MSFNO_ENGINE=x6 selects the six-bf16-MFMA engine instead; MSFNO_GEMM=f32 the fp32
    MFMA kernels)."""
    return x6_engine()[0] and os.environ.get("MSFNO_ENGINE", "") != "x6"


def x6_engine():
    """Dense-GEMM engine the library uses (csrc/gemm_x6.hip gemm_use_x6 /
    api.cpp spec_use_x6 read the same switches)."""
    dense = os.environ.get("MSFNO_GEMM", "") != "f32"
    spec = dense and not os.environ.get("MSFNO_SPEC_X6", "").startswith("0")
    return dense, spec


def mlp_fused(C, hid):
    """The block MLP runs as one fused kernel (csrc/mlp_fused.hip: C 256, H 512, x6
    engine; MSFNO_MLP_FUSED=0 keeps the fc1 / fc2 GEMM pair): x1 then stays fp32."""
    return x6_engine()[0] and C == 256 and hid == 512 and \
        not os.environ.get("MSFNO_MLP_FUSED", "").startswith("0")


def mfma_peak(stage):
    dense, spec = x6_engine()
    if (x3h_engine() and stage in X3H_STAGES) or (stage.startswith("legendre") and leg_x3h()):
        return PEAK_X3H_TFLOPS, "x3h (fp32 via 2-term fp16 split, fp16 MFMA / 3)"
    if (dense and stage in X6_STAGES) or (spec and stage in X6_SPEC_STAGES):
        return PEAK_X6_TFLOPS, "x6 (fp32 via 3-term bf16 split, bf16 MFMA / 6)"
    return PEAK_FP32_MFMA_TFLOPS, "f32 MFMA"


def pmc_traffic(stage):
    """HBM bytes per launch of the stage's kernel from the newest committed PMC
    summary (profiles/*/pmc_traffic.json, written by tools/rocpd_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected), or None."""
    sym = STAGE_KERNEL_LINEAR.get(stage) or (
        STAGE_KERNEL_X3H if x3h_engine() else
        STAGE_KERNEL_X6 if x6_engine()[0] else STAGE_KERNEL_F32).get(stage)
    if sym is None:
        return None, None
    syms = (sym,) if isinstance(sym, str) else sym
    import glob
    import re

    def newest_first(path):  # r01_v10 after r01_v9: compare the numbers, not the text;
        # a round's closing profile (rNN_end) after every other profile of that round
        tag = os.path.basename(os.path.dirname(path))
        m = re.match(r"r(\d+)_(.*)", tag)
        rnd, rest = (int(m.group(1)), m.group(2)) if m else (-1, tag)
        return (rnd, rest.startswith("end"),
                [(0, int(t), "") if t.isdigit() else (1, 0, t) for t in re.split(r"(\d+)", rest)])

    files = []
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_traffic.json")),
                    key=newest_first, reverse=True):
        try:
            with open(f) as fh:
                files.append((f, json.load(fh)["kernels"]))
        except (OSError, ValueError, KeyError):
            continue
    if stage == "mlp_gen":  # the network's encoder + decoder launches: both from one profile
        for f, ks in files:
            b = [ks.get(sy, {}).get("hbm_bytes") for sy in syms]
            if all(b):
                return round(sum(b)), os.path.relpath(f, REPO)
        return None, None
    # the current kernel symbol in any profile first, then the older names of the same kernel
    for sy in syms:
        for f, ks in files:
            k = ks.get(sy)
            if k and k.get("hbm_bytes"):
                return round(k["hbm_bytes"]), os.path.relpath(f, REPO)
    return None, None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="GPUs = rank processes (one per GPU)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1, help="fields per GPU per step")
    ap.add_argument("--filter", default="non-linear", choices=["non-linear", "linear"])
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--nlat", type=int, default=721)
    ap.add_argument("--nlon", type=int, default=1440)
    ap.add_argument("--lmax", type=int, default=360)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on CPU (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads (0: the physical cores this job may use, see host_cores)")
    ap.add_argument("--cpu-reps", type=int, default=3, help="timed oracle reps after 1 warm-up (median)")
    ap.add_argument("--stages", action="store_true", help="print per-stage timings to stderr")
    ap.add_argument("--workload", default="block", choices=["block", "net"],
                    help="block: one SFNO-Block forward per field (config 2, the headline); "
                         "net: one 6 h step of the 12-block FourierNeuralOperatorNet_Filmed "
                         "(config 3: encoder, blocks on the 120x240 Gauss grid, decoder; 73 ch)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture one step in a HIP graph and replay it (default: on for "
                         "--workload net, off for block)")
    ap.add_argument("--parallel", default="auto", choices=["auto", "replicas", "latband"],
                    help="N>1: one batch of batch*N fields latitude-band sharded over the N GPUs "
                         "(RCCL all-to-all; the auto default) or independent replicas")
    ap.add_argument("--band-chunks", type=int, default=0,
                    help="latband: sub-batches pipelined so exchanges overlap compute "
                         "(0: one sub-batch per field, at most 4)")
    ap.add_argument("--band-inner", default="shard", choices=["shard", "replicate"],
                    help="--workload net, latband: shard every block, or replicate the inner "
                         "(h, w) blocks on every rank after one all-gather (SURVEY 8(e))")
    ap.add_argument("--replicas-check", type=int, default=1,
                    help="latband, N>1: also time the replica mode (comm-free upper bound)")
    ap.add_argument("--linear-check", type=int, default=1,
                    help="N=1, non-linear headline: also time config 2's linear filter (the "
                         "per-mode weight stream) and print it as the line's 'linear' object")
    ap.add_argument("--net-check", type=int, default=1,
                    help="N=1 block headline: also time config 3 (the 12-block filmed net, "
                         "one 6 h step) and print it as the line's 'net' object")
    ap.add_argument("--band-check", type=int, default=1,
                    help="latband, N>1: after the timed region compare field 0's sharded "
                         "output with the whole-field block on rank 0 (max-abs in the line)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / process-group check only (gloo, no GPU): ranks report in")
    return ap.parse_args(argv)


parse_args = parse


def stage_work(name, B, C, nlat, nlon, lmax, mmax, hid, shid, rows=None, mset=None):
    """Algorithmic work per launch: ('mfma', flops) or ('hbm', bytes).  Latitude-band
    shards: `rows` local latitude rows, `mset` the rank's zonal wavenumbers."""
    ms = range(mmax) if mset is None else mset
    T = sum(max(lmax - m, 0) for m in ms)
    rows = nlat if rows is None else rows
    P = rows * nlon
    BC = B * C
    tab = {
        "mlp_fc1": ("mfma", 2 * B * P * C * hid),
        "mlp_fc2": ("mfma", 2 * B * P * C * hid),
        "mlp_fused": ("mfma", 4 * B * P * C * hid),
        "inner_skip": ("mfma", 2 * B * P * C * C),
        "spectral_l0": ("mfma", 8 * B * T * C * shid),
        "spectral_l1": ("mfma", 8 * B * T * shid * shid),
        "spectral_l2": ("mfma", 8 * B * T * shid * shid),
        "spectral_out": ("mfma", 8 * B * T * shid * C),
        "legendre_fwd": ("mfma", 2 * (2 * BC) * nlat * T),
        "legendre_inv": ("mfma", 2 * (2 * BC) * nlat * T),
        # HBM-bound stages: compulsory bytes moved
        # rfft: x read + spectrum written (+ x as bf16x3 planes for the inner-skip GEMM
        # with MSFNO_SKIP_PLANES=1 on the x6 engine, whole-field block only)
        "fft_fwd": ("hbm", BC * rows * (nlon * 4 + mmax * 8 +
                                        (nlon * 6 if x6_engine()[0] and mset is None and
                                         os.environ.get("MSFNO_SKIP_PLANES") == "1" else 0))),
        # irfft: Yn read + skip-branch row read + x1 written (bf16x3 planes, 6 B per
        # value, on the x6 engine with the unfused MLP; fp32 for the fused one)
        "fft_inv": ("hbm", BC * rows * (mmax * 8 + nlon * 4 +
                                        nlon * (6 if x6_engine()[0] and not mlp_fused(C, hid)
                                                else 4))),
        "transpose_fwd": ("hbm", 2 * BC * rows * mmax * 8),
        "transpose_inv": ("hbm", 2 * BC * rows * mmax * 8),
        "linear_contract": ("hbm", 8 * C * C * T + 2 * 8 * BC * T),
        # latitude-band pack: the forward transpose into the send buffer (this rank's rows)
        "band_pack": ("hbm", 2 * BC * rows * mmax * 8),
    }
    return tab.get(name)


def build_block(args, dev):
    from functools import partial

    from oracle import sfno_ref  # parameter recipe only (same numbers as the parity tests)
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from msfno_amd.sfno import FourierNeuralOperatorBlock_Filmed

    C, nlat, nlon, lmax = args.C, args.nlat, args.nlon, args.lmax
    mmax = lmax + 1
    cfg = sfno_ref.BlockCfg(filter_type=args.filter)
    big_linear = args.filter == "linear" and C > 64
    if big_linear:
        # the per-mode weight (C, C, T, 2) is 34 GB at C=256: it is drawn on the GPU by
        # the module constructor (reference init 0.02*randn, layers.py:386-387) and only
        # the remaining parameters come from the host recipe
        p = sfno_ref.make_block_params(C, lmax, mmax, sfno_ref.BlockCfg(filter_type="non-linear"),
                                       seed=1)
        p = {k: v for k, v in p.items() if not k.startswith("filter_layer.")}
    else:
        p = sfno_ref.make_block_params(C, lmax, mmax, cfg, seed=1)
    sht = RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular").float()
    isht = InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular").float()
    sht.weights = sht.weights * 1e5
    isht.pct = isht.pct / 1e5
    norm = partial(torch.nn.InstanceNorm2d, num_features=C, eps=1e-6, affine=True,
                   track_running_stats=False)
    torch.manual_seed(1)
    with torch.device(dev if big_linear else "cpu"):
        blk = FourierNeuralOperatorBlock_Filmed(sht, isht, C, filter_type=args.filter,
                                                mlp_ratio=2.0, norm_layer=(norm, norm),
                                                inner_skip="linear", outer_skip="identity",
                                                mlp_mode="distributed", spectral_layers=3)
    blk.load_state_dict(p, strict=False)
    return blk.eval().to(dev), p, cfg


def host_cores():
    """(threads to use, description) for the CPU baseline: the physical cores this
    process may run on (affinity mask ÷ SMT, cgroup quota) — capped by the job's CPU
    share when the launcher sets one (OMP_NUM_THREADS; 16 per GPU on the GPU box)."""
    import subprocess
    info = {}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            info[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass

    def num(key, default):
        try:
            return int(info.get(key, default))
        except ValueError:
            return default
    logical = len(os.sched_getaffinity(0))
    tpc = max(1, num("Thread(s) per core", 1))
    physical = num("Core(s) per socket", 0) * num("Socket(s)", 1) or logical // tpc
    usable = max(1, min(physical, logical // tpc))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
            usable = min(usable, quota)
    except (OSError, ValueError):
        pass
    share = os.environ.get("OMP_NUM_THREADS")
    threads = usable
    if share and share.isdigit() and int(share) > 0:
        threads = min(usable, int(share))
    desc = (f"{info.get('Model name', 'unknown CPU')}; host {physical} physical cores "
            f"({logical} logical CPUs in the affinity mask, {tpc} threads/core"
            + (f", cgroup quota {quota} CPUs" if quota else "")
            + (f", job CPU share OMP_NUM_THREADS={share}" if share else "") + ")")
    return threads, desc


def cpu_baseline(args, p, cfg):
    """Oracle (torch-CPU restatement of the reference block) on a bounded sample:
    1 warm-up + --cpu-reps timed fields, median.  The linear filter
    at C > 64 is timed at C = 32 (its 34 GB weight at C = 256 does not fit the
    sample budget)."""
    from oracle import sfno_ref
    auto, desc = host_cores()
    threads = args.cpu_threads if args.cpu_threads > 0 else auto
    torch.set_num_threads(threads)
    C, nlat, nlon, lmax = args.C, args.nlat, args.nlon, args.lmax
    note = ""
    if args.filter == "linear" and C > 64:
        C = 32
        p = sfno_ref.make_block_params(C, lmax, lmax + 1, cfg, seed=1)
        note = " (linear filter timed at C=32)"
    if p is None:
        p = sfno_ref.make_block_params(C, lmax, lmax + 1, cfg, seed=1)
    sht, isht = sfno_ref.make_transforms(nlat, nlon, lmax, lmax + 1)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, C, nlat, nlon, generator=g)
    gamma = 0.1 * torch.randn(1, C, generator=g)
    beta = 0.1 * torch.randn(1, C, generator=g)
    times = []
    with torch.no_grad():
        sfno_ref.block_forward(p, x, sht, isht, cfg, gamma, beta, 1.0)   # warm-up
        for _ in range(max(1, args.cpu_reps)):
            t0 = time.perf_counter()
            sfno_ref.block_forward(p, x, sht, isht, cfg, gamma, beta, 1.0)
            times.append(time.perf_counter() - t0)
    times.sort()
    dt = times[len(times) // 2]
    return {"value": 1.0 / dt, "unit": "fields/s", "cores": threads, "kind": "port",
            "cpu": desc,
            "sample": f"median of {len(times)} fields ({nlat}x{nlon}x{C}, lmax={lmax}, "
                      f"{args.filter} filter) after 1 warm-up; oracle/sfno_ref.py torch-CPU "
                      f"restatement, {threads} threads; s/field "
                      f"{', '.join(f'{t:.2f}' for t in times)}{note}"}


def run_net(args, rank, world, dev, dist, backend):
    """Config 3: one autoregressive 6 h step of the reference-default network
    (FourierNeuralOperatorNet_Filmed, sfnonet.py:699-860): 73 -> 256 channels,
    12 blocks (block 0 721x1440 -> 120x240 Gauss, blocks 1-10 at 120x240 lmax 120,
    block 11 back to 721x1440), FiLM on the last block, big skip, decoder.
    Synthetic input and FiLM modulation (the FiLM generator is out of scope)."""
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed
    torch.manual_seed(1)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=(args.nlat, args.nlon),
                                          in_chans=73, out_chans=73, embed_dim_sfno=args.C,
                                          num_layers=12, filter_type=args.filter,
                                          spectral_layers=3).eval().to(dev)
    B = args.batch
    parallel = args.parallel
    if parallel == "auto":
        parallel = "latband" if dist else "replicas"
    band = parallel == "latband"
    if band:
        # config 5's multi-GPU form: ONE batch of `batch` fields stepped through the
        # network latitude-band sharded over the ranks (LatBandNet; strong scaling)
        from msfno_amd.sfno import LatBandNet, TorchComm
        shard = LatBandNet(net, rank, world, device=dev,
                           comm=TorchComm() if dist else None, inner=args.band_inner)
        g = torch.Generator(device=dev).manual_seed(0)
        x = shard.take(torch.randn(B, 73, args.nlat, args.nlon, generator=g, device=dev))
        film = 0.1 * torch.randn(B, 2, 1, args.C, generator=g, device=dev)
        run = shard
    else:
        g = torch.Generator(device=dev).manual_seed(1000 * rank)
        x = torch.randn(B, 73, args.nlat, args.nlon, generator=g, device=dev)
        film = 0.1 * torch.randn(B, 2, 1, args.C, generator=g, device=dev)
        run = net

    def barrier():
        if dist:
            torch.distributed.barrier()

    # the sharded step is captured too when its exchanges run on RCCL (recorded into
    # the graph); gloo collectives are host calls
    use_graph = args.graph != 0 and (not band or (dist and backend == "nccl"))
    with torch.no_grad():
        for _ in range(max(args.warmup, 1)):
            y = run(x, film, 1.0)
        torch.cuda.synchronize()
        if use_graph and band and dist:
            run.comm.quiesce()  # RCCL watchdog: nothing pending while the capture runs
        if use_graph:
            # one 6 h step as a HIP graph: removes the host cost of ~300 launches and
            # the per-call module bookkeeping (the 120x240 blocks are launch-bound)
            graph = torch.cuda.CUDAGraph()
            ok = True
            try:
                with torch.cuda.graph(graph):
                    y = run(x, film, 1.0)
            except RuntimeError as e:
                if not band:
                    raise
                print(f"bench: sharded step not capturable on rank {rank} ({e})", file=sys.stderr)
                ok = False
                torch.cuda.synchronize()
            if band and dist:
                # every rank replays, or every rank steps eagerly (no replayed collective
                # may meet an eager one)
                ok = run.comm.all_agree(ok)
            if ok:
                graph.replay()
                torch.cuda.synchronize()
            else:
                use_graph = False
                y = run(x, film, 1.0)

        if use_graph:
            def step():
                graph.replay()
        else:
            def step():
                return run(x, film, 1.0)
        from msfno_amd import _native as N
        if args.stages and not use_graph:
            N.profile_collect()
            N.profile_enable(True)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        if args.stages and not use_graph and rank == 0:
            N.profile_enable(False)
            for k, (ms, c) in sorted(N.profile_collect().items(), key=lambda kv: -kv[1][0]):
                print(f"  stage {k:18s} {ms / args.steps:8.3f} ms/step x{c // args.steps}",
                      file=sys.stderr)
    if dist:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu",
                         dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()
    assert torch.isfinite(y).all()
    roof = None
    if rank == 0 and not band:
        # roofline of the step's dominant kernel: one more (untimed, eager) step with
        # the stage profiler on (the graph replay above cannot be split into kernels)
        from msfno_amd import _native as N
        with torch.no_grad():
            N.profile_collect()
            N.profile_enable(True)
            run(x, film, 1.0)
            torch.cuda.synchronize()
            N.profile_enable(False)
            roof = net_roofline(N.profile_collect(), args, B)
    line = None
    if rank == 0:
        line = {
            "metric": "FourierNeuralOperatorNet_Filmed 6h steps/sec (12 blocks, 73 ch, 721x1440)",
            "value": round((1 if band else world) * B * args.steps / elapsed, 3),
            "unit": "steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "strong" if band else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (x~N(0,1), FiLM modulation ~0.1 N(0,1), random-init weights)",
            "roofline": roof,
            "config": {"workload": f"sfno_net12_filmed_{args.nlat}x{args.nlon}_C{args.C}_73ch",
                       "batch_per_gpu": B, "filter": args.filter, "hip_graph": use_graph,
                       "band_inner": args.band_inner if band else None,
                       "parallelism": (f"latband{world}" if band else
                                       (f"replicas{world}" if world > 1 else "single"))}}
    del run, x, y
    if not band:
        del net
    torch.cuda.empty_cache()
    return line


def net_cpu_baseline(args):
    """Config 3 on the host: oracle.sfno_ref.net_forward (the torch-CPU restatement of
    FourierNeuralOperatorNet_Filmed.forward, sfnonet.py:787-860) on ONE 6 h step after
    one warm-up step (a bounded sample: ~5 s per step on 16 cores), same shapes and
    default parameter recipe as the GPU line."""
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed
    from oracle import sfno_ref
    auto, desc = host_cores()
    threads = args.cpu_threads if args.cpu_threads > 0 else auto
    torch.set_num_threads(threads)
    torch.manual_seed(1)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=(args.nlat, args.nlon),
                                          in_chans=73, out_chans=73, embed_dim_sfno=args.C,
                                          num_layers=12, filter_type=args.filter,
                                          spectral_layers=3)
    params = {k: v.detach() for k, v in net.state_dict().items()
              if not k.endswith((".weights", ".pct"))}
    del net
    ncfg = sfno_ref.NetCfg(img_size=(args.nlat, args.nlon), scale_factor=6, num_layers=12,
                           filter_type=args.filter)
    tr = sfno_ref.make_net_transforms(ncfg)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, 73, args.nlat, args.nlon, generator=g)
    gamma = 0.1 * torch.randn(1, 1, args.C, generator=g)
    beta = 0.1 * torch.randn(1, 1, args.C, generator=g)
    times = []
    with torch.no_grad():
        for rep in range(2):
            t0 = time.perf_counter()
            sfno_ref.net_forward(params, x, ncfg, transforms=tr, film=(gamma, beta), scale=1.0)
            times.append(time.perf_counter() - t0)
    dt = times[-1]
    return {"value": 1.0 / dt, "unit": "steps/s", "cores": threads, "kind": "port", "cpu": desc,
            "sample": f"1 step of the 12-block filmed net ({args.nlat}x{args.nlon}, C={args.C}, "
                      f"73 ch) after 1 warm-up; oracle/sfno_ref.py net_forward, {threads} "
                      f"threads; s/step {times[0]:.2f} (warm-up), {times[1]:.2f}"}


def net_line(args, dev):
    """Config 3 beside the N = 1 block line (the driver runs bench.py --gpus 1 only):
    one 6 h step of the 12-block filmed network at 721 x 1440, HIP-graph replayed, its
    roofline and CPU baseline."""
    import copy
    na = copy.copy(args)
    na.workload = "net"
    na.graph = -1
    torch.cuda.empty_cache()
    line = run_net(na, 0, 1, dev, False, "nccl")
    if args.cpu_baseline:
        line["cpu_baseline"] = net_cpu_baseline(na)
    return {k: line[k] for k in ("metric", "value", "unit", "ms_per_step", "roofline", "config",
                                 "cpu_baseline") if k in line}


def net_roofline(stages, args, B):
    """Config 3's dominant kernel: of the profiled stages whose work is known for the
    network (the fused encoder + decoder MLPs or their fc1 / fc2 GEMMs, 73 -> 256 -> 256 and 329 -> 256 ->
    73 at the full grid; the block MLPs of blocks 0..10 on the 120x240 grid, the last
    block having none), the one with the most device time per step; work and time
    summed over the step's launches of it."""
    C, P = args.C, args.nlat * args.nlon
    P_in = 120 * 240
    work = {
        # encoder 73 -> C -> C and decoder (C + 73) -> C -> 73, each one fused x3h launch
        # (csrc/mlp_gen_h.hip; MSFNO_MLP_GEN_H=0: the fc1 / fc2 GEMM pairs below)
        "mlp_gen": 2 * B * P * C * ((73 + C) + (C + 73 + 73)),
        "mlp_fc1": 2 * B * P * C * (73 + (C + 73)),
        "mlp_fc2": 2 * B * P * C * (C + 73),
        # blocks 0..10 (block 0's MLP runs on its 120x240 output grid); the last block
        # has none (mlp_mode="none", sfnonet.py:583/729)
        "mlp_fused": 4 * B * C * (2 * C) * 11 * P_in,
    }
    known = {k: v for k, v in stages.items() if k in work}
    if not known:
        return None
    name, (ms, cnt) = max(known.items(), key=lambda kv: kv[1][0])
    ach = work[name] / (ms / 1000.0) / 1e12
    peak, engine = mfma_peak(name)
    # HBM bytes per step of the encoder + decoder launches (stored PMC profile; default
    # kernels at the full grid only)
    tr, tr_src = (pmc_traffic(name) if name == "mlp_gen" and B == 1 and C == 256 and
                  args.nlat == 721 and args.nlon == 1440 and cnt == 2 else (None, None))
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1),
            "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": tr,
            "traffic_source": (f"stored PMC profile {tr_src} (encoder + decoder per step; "
                               "not measured in this run)" if tr_src else None),
            "kernel": name, "engine": engine, "launches_per_step": cnt,
            "ms_per_step": round(ms, 4), "work_per_step": f"{work[name] / 1e9:.1f} GFLOP",
            "all_stages_ms": {k: round(v[0], 3) for k, v in
                              sorted(stages.items(), key=lambda kv: -kv[1][0])[:8]}}


def launch(args):
    """``--gpus N`` (N > 1) without WORLD_SIZE: start the N rank processes (one per
    GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their environment) as children of
    this process, which never touches the GPU.  Returns the first failing exit code
    (the other ranks are then terminated) or 0."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for pr in list(alive):
            r = pr.poll()
            if r is None:
                continue
            alive.remove(pr)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in alive:
                    q.terminate()
        time.sleep(0.1)
    return rc


def _max_over_ranks(v, dist, dev, backend):
    if not dist:
        return v
    t = torch.tensor([v], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return t.item()


def timed(step, args, dist, dev, backend):
    """W untimed warm-up steps, then exactly K steps between barrier + synchronize
    on both sides; returns (last output, max-over-ranks seconds, stage profile)."""
    from msfno_amd import _native as N

    def barrier():
        if dist:
            torch.distributed.barrier()
    y = None
    for _ in range(args.warmup):
        y = step()
    torch.cuda.synchronize()
    N.profile_collect()  # discard
    N.profile_enable(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        y = step()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    N.profile_enable(False)
    stages = N.profile_collect()
    return y, _max_over_ranks(t1 - t0, dist, dev, backend), stages


# stage spans that are not kernels: waits on a collective (latitude-band exchange)
NON_KERNEL_STAGES = {"band_exchange"}


def roofline(stages, args, B, C, rows, mset, name=None):
    """Roofline of the dominant kernel: the main-stream stage with the largest device
    time (the inner-skip GEMM overlaps the SHT on a side stream: its event span is not
    a kernel duration, so it is not eligible), or of stage ``name``."""
    mmax = args.lmax + 1
    hid = shid = 2 * C
    side = os.environ.get("MSFNO_SIDE_STREAM", "1") != "0"
    elig = {k: v for k, v in stages.items()
            if not (side and k in SIDE_STAGES) and k not in NON_KERNEL_STAGES
            and stage_work(k, B, C, args.nlat, args.nlon, args.lmax, mmax, hid, shid,
                           rows, mset) is not None}
    if name is not None:
        elig = {k: v for k, v in elig.items() if k == name}
    if not elig:
        return None
    name, (tot_ms, cnt) = max(elig.items(), key=lambda kv: kv[1][0])
    avg_s = tot_ms / cnt / 1000.0
    kind, amount = stage_work(name, B, C, args.nlat, args.nlon, args.lmax, mmax, hid, shid,
                              rows, mset)
    whole = rows is None and mset is None
    tr, tr_src = pmc_traffic(name) if (B == 1 and C == 256 and args.nlat == 721 and whole
                                        and (args.filter == "non-linear"
                                             or name == "linear_contract")) else (None, None)
    if kind == "mfma":
        ach = amount / avg_s / 1e12
        peak, engine = mfma_peak(name)
        return {"bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1),
                "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": tr,
                "traffic_source": (f"stored PMC profile {tr_src} (same kernel and shape; not "
                                   "measured in this run)") if tr_src else None,
                "kernel": name, "engine": engine, "avg_ms": round(avg_s * 1e3, 4),
                "work_per_launch": f"{amount / 1e9:.2f} GFLOP"}
    ach = amount / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": tr,
            "traffic_source": (f"stored PMC profile {tr_src}" if tr_src else None),
            "kernel": name, "avg_ms": round(avg_s * 1e3, 4),
            "work_per_launch": f"{amount / 1e9:.3f} GB"}


def print_stages(stages, args, B, C, rows, mset, tag=""):
    mmax = args.lmax + 1
    for k, (ms, c) in sorted(stages.items(), key=lambda kv: -kv[1][0]):
        w = stage_work(k, B, C, args.nlat, args.nlon, args.lmax, mmax, 2 * C, 2 * C, rows, mset)
        extra = ""
        if w:
            a = w[1] / (ms / c / 1e3)
            if w[0] == "mfma":
                pk = mfma_peak(k)[0]
                extra = f" {a / 1e12:.1f} TFLOP/s ({100 * a / 1e12 / pk:.0f}% of {pk:.0f})"
            else:
                extra = f" {a / 1e9:.0f} GB/s ({100 * a / 1e9 / PEAK_HBM_GBS:.0f}%)"
        print(f"  {tag}stage {k:18s} {ms / c:8.3f} ms x{c}{extra}", file=sys.stderr)


def linear_line(args, dev):
    """Config 2's second filter (SURVEY.md §8d "measure both filters"): the same
    block with the linear per-mode filter (SpectralConvS2, layers.py:398-427: the
    (C, C, T, 2) weight, 34.07 GB at C = 256, streamed once per field), same K / W.
    Its roofline is the weight-streaming contraction's (HBM); the CPU baseline is
    the oracle at C = 32 (the 34 GB weight does not fit the sample budget)."""
    import copy
    la = copy.copy(args)
    la.filter = "linear"
    torch.cuda.empty_cache()
    blk, p, cfg = build_block(la, dev)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(args.batch, args.C, args.nlat, args.nlon, generator=g).to(dev)
    gamma = (0.1 * torch.randn(args.batch, args.C, generator=g)).to(dev)
    beta = (0.1 * torch.randn(args.batch, args.C, generator=g)).to(dev)
    with torch.no_grad():
        y, elapsed, stages = timed(lambda: blk(x, gamma, beta, 1.0), la, False, dev, "nccl")
    assert torch.isfinite(y).all()
    roof = roofline(stages, la, args.batch, args.C, None, None, name="linear_contract")
    del blk, x, y
    torch.cuda.empty_cache()
    cpu = None
    if args.cpu_baseline:
        cpu = cpu_baseline(la, None, cfg)
    return {"filter": "linear", "value": round(args.batch * args.steps / elapsed, 3),
            "unit": "fields/s", "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "workload": f"sfno_block_fwd_{args.nlat}x{args.nlon}_C{args.C}_lmax{args.lmax}_"
                        "linear_filmed", "roofline": roof, "cpu_baseline": cpu}


def band_check(shard, blk, y, gamma, beta, args, rank, world, dev, backend):
    """Correctness of the sharded step (config 4): field 0's output rows from every
    rank, assembled on rank 0, against the whole-field block on rank 0 (the same
    module, unsharded) on the same input field.  Returns the check for the line."""
    C, nlon = args.C, args.nlon
    rows_all = [None] * world
    torch.distributed.all_gather_object(rows_all, list(shard.rows_out))
    maxr = max(len(r) for r in rows_all)
    mine = torch.zeros(1, C, maxr, nlon, device=dev)
    mine[:, :, :len(shard.rows_out)] = y[:1]
    if backend != "nccl":
        mine = mine.cpu()
    parts = [torch.empty_like(mine) for _ in range(world)]
    torch.distributed.all_gather(parts, mine)
    if rank != 0:
        return None
    full = torch.empty(1, C, args.nlat, nlon, device=dev)
    for r, t in enumerate(parts):
        idx = torch.tensor(rows_all[r], dtype=torch.long, device=dev)
        full.index_copy_(2, idx, t[:, :, :len(rows_all[r])].to(dev))
    gd = torch.Generator(device=dev).manual_seed(0)  # field 0 is the first draw (main)
    x0 = torch.randn(1, C, args.nlat, nlon, generator=gd, device=dev)
    with torch.no_grad():
        ref = blk(x0, gamma[:1].contiguous(), beta[:1].contiguous(), 1.0)
    err = (full - ref).abs().max().item()
    scale = ref.abs().max().item()
    del full, ref, x0
    torch.cuda.empty_cache()
    return {"field": 0, "max_abs": err, "max_ref": round(scale, 4),
            "ok": bool(err <= 2e-5 * max(1.0, scale)),
            "against": "the whole-field block (same module, unsharded) on rank 0"}


def dry_run(rank, world):
    """Process-group check without a GPU (tests/test_bench_launch.py): gloo."""
    import socket
    import torch.distributed as td
    td.init_process_group("gloo")
    seen = [None] * world
    td.all_gather_object(seen, (rank, socket.gethostname(), os.getpid()))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "world_size": td.get_world_size(),
                          "ranks_seen": len({r for r, _, _ in seen}),
                          "pids": sorted({p for _, _, p in seen})}), flush=True)
    td.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # one process per GPU, started here before anything touches the GPU
        sys.exit(launch(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(env_world or "1")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist = world > 1
    if args.dry_run:
        return dry_run(rank, world) if dist else print(json.dumps(
            {"dry_run": True, "n_gpus": 1, "world_size": 1, "ranks_seen": 1}))
    # rehearsal knobs for a one-GPU box (never used by the driver's runs):
    # MSFNO_BENCH_BACKEND=gloo and MSFNO_BENCH_SHARE_GPU=1 put every rank on cuda:0
    backend = os.environ.get("MSFNO_BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("MSFNO_BENCH_SHARE_GPU") == "1" else local
    if dist:
        import torch.distributed as td
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            td.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            td.init_process_group(backend)
        assert td.get_world_size() == world == args.gpus
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    ranks_seen, gpus_seen = 1, 1
    if dist:
        import socket
        props = torch.cuda.get_device_properties(dev)
        ident = (rank, socket.gethostname(), str(getattr(props, "uuid", gpu)))
        seen = [None] * world
        torch.distributed.all_gather_object(seen, ident)
        ranks_seen = len({r for r, _, _ in seen})
        gpus_seen = len({(h, u) for _, h, u in seen})

    if args.workload == "net":
        line = run_net(args, rank, world, dev, dist, backend)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist:
            torch.distributed.destroy_process_group()
        return
    blk, p, cfg = build_block(args, dev)
    C = args.C
    parallel = args.parallel
    if parallel == "auto":
        parallel = "latband" if dist else "replicas"
    band = parallel == "latband"
    rows = mset = None
    chunks = 1
    if band:
        # one batch of batch*N fields, each rank holding its latitude band of every field
        from msfno_amd.sfno import LatBandBlock, TorchComm
        B = args.batch * world
        shard = LatBandBlock(blk, rank, world, device=dev)
        rows, mset = len(shard.rows), [m for m, o in enumerate(shard.m_owner) if o == rank]
        gd = torch.Generator(device=dev).manual_seed(0)
        x = torch.empty(B, C, rows, args.nlon, device=dev)
        for b in range(B):  # field b is identical on every rank; keep this rank's rows
            x[b] = shard.take(torch.randn(1, C, args.nlat, args.nlon, generator=gd, device=dev))[0]
        gamma = 0.1 * torch.randn(B, C, generator=gd, device=dev)
        beta = 0.1 * torch.randn(B, C, generator=gd, device=dev)
        comm = TorchComm() if dist else None
        # at least two sub-batches whenever the batch allows (N = 2 exchanges over a
        # single xGMI link: one sub-batch's all-to-all hides behind the other's compute)
        chunks = args.band_chunks if args.band_chunks > 0 else max(1, min(4, B))

        def step():
            return shard(x, gamma, beta, 1.0, comm=comm, chunks=chunks)
    else:
        B = args.batch
        g = torch.Generator().manual_seed(1000 * rank)
        x = torch.randn(B, C, args.nlat, args.nlon, generator=g).to(dev)
        gamma = (0.1 * torch.randn(B, C, generator=g)).to(dev)
        beta = (0.1 * torch.randn(B, C, generator=g)).to(dev)

        def step():
            return blk(x, gamma, beta, 1.0)

    with torch.no_grad():
        y, elapsed, stages = timed(step, args, dist, dev, backend)
    fields = (B if band else world * B) * args.steps
    value = fields / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    # work per launch: a latitude-band step launches every kernel once per sub-batch
    B_launch = B / chunks if band else B
    roof = roofline(stages, args, B_launch, C, rows, mset)
    if args.stages:
        print_stages(stages, args, B_launch, C, rows, mset, tag=f"rank{rank} ")
    assert torch.isfinite(y).all()

    check = None
    if band and dist and args.band_check:
        check = band_check(shard, blk, y, gamma, beta, args, rank, world, dev, backend)

    replicas = None
    if band and dist and args.replicas_check:
        # the comm-free upper bound: every rank runs its own batch fields whole
        del x, shard
        torch.cuda.empty_cache()
        Br = args.batch
        gr = torch.Generator(device=dev).manual_seed(1000 * rank)
        xr = torch.randn(Br, C, args.nlat, args.nlon, generator=gr, device=dev)
        gr_, br_ = gamma[:Br].contiguous(), beta[:Br].contiguous()

        def rstep():
            return blk(xr, gr_, br_, 1.0)
        with torch.no_grad():
            _, rel, rstages = timed(rstep, args, dist, dev, backend)
        replicas = {"value": round(world * Br * args.steps / rel, 3), "unit": "fields/s",
                    "ms_per_step": round(1000.0 * rel / args.steps, 3),
                    "parallelism": f"replicas{world}", "global_batch": world * Br}
        del xr

    per_rank = None
    band_info = None
    if dist:
        ex = stages.get("band_exchange")
        mine = {"rank": rank, "kernel": roof and roof["kernel"], "avg_ms": roof and roof["avg_ms"],
                "frac": roof and roof["frac"],
                "exchange_wait_ms_per_step": round(ex[0] / args.steps, 3) if ex else None,
                "rows": rows, "m_count": len(mset) if mset is not None else None}
        per_rank = [None] * world
        torch.distributed.all_gather_object(per_rank, mine)
        if band:
            band_info = {"chunks": chunks, "rows_per_rank": [q["rows"] for q in per_rank],
                         "m_per_rank": [q["m_count"] for q in per_rank]}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        del blk
        torch.cuda.empty_cache()
        cpu = cpu_baseline(args, p, cfg)

    linear = None
    if world == 1 and args.linear_check and args.filter == "non-linear" and not band:
        linear = linear_line(args, dev)
    net = None
    if world == 1 and args.net_check and not band and (args.nlat, args.nlon) == (721, 1440):
        net = net_line(args, dev)

    if rank == 0:
        out = {
            "metric": "SFNO-Block forward fields/sec on 721x1440x256; rocprof HBM GB/s vs peak",
            "value": round(value, 3),
            "unit": "fields/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (x~N(0,1), random-init weights of the reference block)",
            "config": {"workload": f"sfno_block_fwd_{args.nlat}x{args.nlon}_C{C}_lmax{args.lmax}_"
                                   f"{args.filter}_filmed",
                       "batch_per_gpu": args.batch, "global_batch": B if band else B * world,
                       "filter": args.filter,
                       "band_inner": args.band_inner if band else None,
                       "parallelism": (f"latband{world}" if band else
                                       (f"replicas{world}" if world > 1 else "single"))},
            "ranks_seen": ranks_seen,
            "gpus_seen": gpus_seen,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if band_info:
            out["latband"] = band_info
        if per_rank:
            out["per_rank"] = per_rank
        if replicas:
            out["replicas_upper_bound"] = replicas
        if linear:
            out["linear"] = linear
        if net:
            out["net"] = net
        if check:
            out["latband_check"] = check
        print(json.dumps(out), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
