"""Host-side checks of the latitude-band sharded path, no GPU:
the partition and exchange counts exported by libmsfno, and the full data
movement of one sharded block forward — pack by owner of m, all-to-all,
re-assembly of full-latitude slabs, the return trip and the fp64 statistics
merge — run over a real world-size-2/3 ``gloo`` process group through
``msfno_amd.sfno.latband.TorchComm``.  The device kernels' index maps
(transpose_fwd/inv with the slab permutation, band_copy) are restated here in
numpy; the GPU tests (test_gpu_latband.py) check the kernels themselves."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from msfno_amd.sfno import latband


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,nlat,lmax,mmax", [(1, 32, 32, 33), (2, 33, 16, 17), (3, 721, 360, 361),
                                                  (8, 721, 360, 361), (5, 17, 9, 12)])
def test_partition_properties(world, nlat, lmax, mmax):
    rows, own = latband.band_partition(world, nlat, lmax, mmax)
    h = np.diff(rows)
    assert rows[0] == 0 and rows[-1] == nlat and h.min() >= 1 and h.max() - h.min() <= 1
    own = np.array(own)
    mact = min(lmax, mmax)
    assert (own[:mact] >= 0).all() and (own[mact:] == -1).all()
    cnt = np.bincount(own[:mact], minlength=world)
    assert cnt.max() - cnt.min() <= 1
    work = np.bincount(own[:mact], weights=lmax - np.arange(mact), minlength=world)
    if mact >= 2 * world:
        assert work.max() / work.mean() < 1.0 + 2.0 * world / mact + 0.05


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_exchange_counts_are_symmetric(world):
    nlat, lmax, mmax, R = 721, 360, 361, 2 * 2 * 8
    rows, own = latband.band_partition(world, nlat, lmax, mmax)
    for ph in (0, 1):
        c = [latband.exchange_counts(world, r, nlat, mmax, rows, own, R, ph) for r in range(world)]
        for r in range(world):
            for q in range(world):
                assert c[r][0][q] == c[q][1][r]
        tot = sum(sum(s) for s, _ in c)
        assert tot == R * nlat * min(lmax, mmax)   # every (row, m) of every field moves once


def test_partition_rejects_bad_input():
    with pytest.raises(NotImplementedError):
        latband.band_partition(65, 721, 360, 361)
    with pytest.raises(ValueError):
        latband.band_partition(8, 4, 4, 5)          # fewer rows than ranks
    rows, own = latband.band_partition(2, 16, 8, 9)
    own[0] = -1                                      # m = 0 unowned
    with pytest.raises(ValueError):
        latband.exchange_counts(2, 0, 16, 9, rows, own, 4, 0)


# ---- numpy restatement of the device index maps --------------------------------
def _perm(own, world):
    own = np.asarray(own)
    perm = -np.ones(len(own), dtype=np.int64)
    nm = np.bincount(own[own >= 0], minlength=world)
    start = np.concatenate([[0], np.cumsum(nm)[:-1]])
    for m in range(len(own)):
        if own[m] >= 0:
            perm[m] = start[own[m]]
            start[own[m]] += 1
    return perm


def _rows_of(B, C):   # spectral row r = (b*2 + ri)*C + c
    return [(b, ri, c) for b in range(B) for ri in range(2) for c in range(C)]


def _pack_fwd(Xn, perm, B, C):
    """transpose_fwd with slab map: Xn (BC, H, mmax) complex -> slabs (perm, R, H)."""
    H, mmax = Xn.shape[1], Xn.shape[2]
    R = 2 * B * C
    out = np.zeros(((perm >= 0).sum(), R, H), dtype=np.float32)
    for m in range(mmax):
        if perm[m] < 0:
            continue
        for r, (b, ri, c) in enumerate(_rows_of(B, C)):
            v = Xn[b * C + c, :, m]
            out[perm[m], r] = v.real if ri == 0 else v.imag
    return out.reshape(-1)


def _band_unpack(buf, nm, R, rows, nlat):
    """band_copy(to_bands=False): per-band blocks (nm*R, H_p) -> (nm*R, nlat)."""
    n = nm * R
    F = np.zeros((n, nlat), dtype=np.float32)
    for p in range(len(rows) - 1):
        hp = rows[p + 1] - rows[p]
        F[:, rows[p]:rows[p + 1]] = buf[n * rows[p]:n * rows[p] + n * hp].reshape(n, hp)
    return F


def _band_pack(F, rows):
    n = F.shape[0]
    out = np.zeros(n * rows[-1], dtype=np.float32)
    for p in range(len(rows) - 1):
        hp = rows[p + 1] - rows[p]
        out[n * rows[p]:n * rows[p] + n * hp] = F[:, rows[p]:rows[p + 1]].reshape(-1)
    return out


def _unpack_inv(buf, perm, mact, B, C, H, mmax):
    """transpose_inv with slab map: slabs (perm, R, H) -> Yn (BC, H, mmax) complex."""
    R = 2 * B * C
    Y = np.zeros((B * C, H, mmax), dtype=np.complex64)
    sl = buf.reshape(-1, R, H)
    for m in range(min(mact, mmax)):
        if perm[m] < 0:
            continue
        for r, (b, ri, c) in enumerate(_rows_of(B, C)):
            if ri == 0:
                Y[b * C + c, :, m] += sl[perm[m], r]
            else:
                Y[b * C + c, :, m] += 1j * sl[perm[m], r]
    return Y


def _welford(x):
    return np.array([x.size, x.mean(), ((x - x.mean()) ** 2).sum()])


def _merge(parts):
    n, mean, m2 = parts[0]
    for q in parts[1:]:
        nb, mb, m2b = q
        d = mb - mean
        tot = n + nb
        mean = mean + d * nb / tot
        m2 = m2 + m2b + d * d * n * nb / tot
        n = tot
    return n, mean, m2


def _rank_main(rank, world, port, B, C, nlat, lmax, mmax, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = latband.TorchComm()
        rows, own = latband.band_partition(world, nlat, lmax, mmax)
        R, mact = 2 * B * C, min(lmax, mmax)
        rng = np.random.default_rng(0)
        X = (rng.standard_normal((B * C, nlat, mmax))
             + 1j * rng.standard_normal((B * C, nlat, mmax))).astype(np.complex64)
        field = rng.standard_normal((B * C, nlat, 12))
        r0, r1 = rows[rank], rows[rank + 1]
        perm = _perm(own, world)
        mine = [m for m in range(mmax) if own[m] == rank]
        nm = len(mine)
        # statistics partials -> all_gather -> fp64 merge
        st = torch.tensor(np.stack([_welford(field[i, r0:r1]) for i in range(B * C)]))
        allst = comm.all_gather(st).numpy()
        for i in range(B * C):
            n, mean, m2 = _merge([allst[p, i] for p in range(world)])
            assert n == field[i].size
            np.testing.assert_allclose(mean, field[i].mean(), rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(m2 / n, field[i].var(), rtol=1e-10)
        # phase 0: rows -> m
        sc, rc = latband.exchange_counts(world, rank, nlat, mmax, rows, own, R, 0)
        send = torch.from_numpy(_pack_fwd(X[:, r0:r1], perm, B, C))
        assert send.numel() == sum(sc)
        recv = torch.zeros(sum(rc))
        comm.all_to_all(send, sc, recv, rc)
        F = _band_unpack(recv.numpy(), nm, R, rows, nlat).reshape(nm, R, nlat)
        for i, m in enumerate(mine):
            for r, (b, ri, c) in enumerate(_rows_of(B, C)):
                want = X[b * C + c, :, m]
                np.testing.assert_array_equal(F[i, r], want.real if ri == 0 else want.imag)
        # phase 1: m -> rows (send the assembled slabs back)
        sc1, rc1 = latband.exchange_counts(world, rank, nlat, mmax, rows, own, R, 1)
        send1 = torch.from_numpy(_band_pack(F.reshape(nm * R, nlat), rows))
        assert send1.numel() == sum(sc1)
        recv1 = torch.zeros(sum(rc1))
        comm.all_to_all(send1, sc1, recv1, rc1)
        Y = _unpack_inv(recv1.numpy(), perm, mact, B, C, r1 - r0, mmax)
        want = X[:, r0:r1].copy()
        want[:, :, mact:] = 0
        np.testing.assert_array_equal(Y, want)
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,B,C,nlat,lmax,mmax", [(2, 1, 3, 11, 6, 7), (3, 2, 2, 13, 8, 10)])
def test_sharded_exchange_over_gloo(world, B, C, nlat, lmax, mmax):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, B, C, nlat, lmax, mmax, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(world)}, res
