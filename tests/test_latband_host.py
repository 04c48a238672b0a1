"""Host-side checks of the latitude-band sharded path, no GPU:
the partition (bands of the northern half + their mirror rows) and exchange
counts exported by libmsfno, and the full data movement of one sharded block
forward — the folding pack by owner of m, all-to-all, the receive buffer read as
the forward Legendre GEMM's segmented operand, the return trip into the inverse
GEMM's segmented output, the unfolding unpack and the fp64 statistics merge — run
over a real world-size-2/3 ``gloo`` process group through
``msfno_amd.sfno.latband.TorchComm``.  The device kernels' index maps (band_pack /
band_unpack with the slab permutation, the GEMM's exchange-column addressing) are
restated here in numpy; the GPU tests (test_gpu_latband.py) check the kernels."""
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
    assert rows[0] == 0 and rows[-1] == nlat - nlat // 2 and h.min() >= 1
    assert h.max() - h.min() <= 1
    # the ranks' local rows (band + mirrors) cover every latitude exactly once
    loc = [latband.local_rows(world, r, nlat, rows) for r in range(world)]
    assert sorted(sum(loc, [])) == list(range(nlat))
    for r, lr in enumerate(loc):   # local row H-1-i is the mirror of local row i
        npair = max(0, min(rows[r + 1], nlat // 2) - rows[r])
        assert all(lr[len(lr) - 1 - i] == nlat - 1 - lr[i] for i in range(npair))
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
        # every (m, spectral row) moves once per source band: 2W floats (>= its rows)
        W = -(-max(np.diff(rows)) // 16) * 16
        assert tot == R * world * 2 * W * min(lmax, mmax)
        assert world * 2 * W <= nlat + world * 2 * 16


def test_partition_rejects_bad_input():
    with pytest.raises(NotImplementedError):
        latband.band_partition(65, 721, 360, 361)
    with pytest.raises(ValueError):
        latband.band_partition(8, 14, 4, 5)         # fewer northern rows than ranks
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


def _width(rows):     # exchange slab rows hold 2W floats
    return int(-(-max(np.diff(rows)) // 16) * 16)


def _band(rows, rank, nlat):  # (a, bw, np): band [a, a+bw), np rows with a mirror
    a, b = rows[rank], rows[rank + 1]
    return a, b - a, max(0, min(b, nlat // 2) - a)


def _pack_fwd(Xl, perm, B, C, bw, npair, W):
    """band_pack (symmetric): local spectra (BC, H, mmax) -> slabs (perm, R, 2W) of
    [Xs = X_i + X_{H-1-i} | Xa = X_i - X_{H-1-i}], zero pads."""
    H, mmax = Xl.shape[1], Xl.shape[2]
    R = 2 * B * C
    out = np.zeros(((perm >= 0).sum(), R, 2 * W), dtype=np.float32)
    for m in range(mmax):
        if perm[m] < 0:
            continue
        for r, (b, ri, c) in enumerate(_rows_of(B, C)):
            v = Xl[b * C + c, :, m]
            v = v.real if ri == 0 else v.imag
            for i in range(bw):
                out[perm[m], r, i] = v[i] + (v[H - 1 - i] if i < npair else 0)
                if i < npair:
                    out[perm[m], r, W + i] = v[i] - v[H - 1 - i]
    return out.reshape(-1)


def _unpack_inv(buf, perm, mact, B, C, bw, npair, W, mmax):
    """band_unpack (symmetric): slabs (perm, R, 2W) of [E | O] -> local Yn
    (BC, H, mmax): Y_i = E_i + O_i, Y_{H-1-i} = E_i - O_i."""
    R, H = 2 * B * C, bw + npair
    Y = np.zeros((B * C, H, mmax), dtype=np.complex64)
    sl = buf.reshape(-1, R, 2 * W)
    for m in range(min(mact, mmax)):
        if perm[m] < 0:
            continue
        for r, (b, ri, c) in enumerate(_rows_of(B, C)):
            E, O = sl[perm[m], r, :bw], sl[perm[m], r, W:W + npair]
            y = np.zeros(H, dtype=np.float32)
            y[:bw] = E
            y[:npair] += O
            y[bw:] = (E[:npair] - O)[::-1]
            Y[b * C + c, :, m] += y if ri == 0 else 1j * y
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
        R, mact, W = 2 * B * C, min(lmax, mmax), _width(rows)
        rng = np.random.default_rng(0)
        X = (rng.standard_normal((B * C, nlat, mmax))
             + 1j * rng.standard_normal((B * C, nlat, mmax))).astype(np.complex64)
        field = rng.standard_normal((B * C, nlat, 12))
        loc = latband.local_rows(world, rank, nlat, rows)
        a, bw, npair = _band(rows, rank, nlat)
        assert loc == list(range(a, a + bw)) + list(range(nlat - a - npair, nlat - a))
        perm = _perm(own, world)
        mine = [m for m in range(mmax) if own[m] == rank]
        nm = len(mine)
        # statistics partials -> all_gather -> fp64 merge
        st = torch.tensor(np.stack([_welford(field[i, loc]) for i in range(B * C)]))
        allst = comm.all_gather(st).numpy()
        for i in range(B * C):
            n, mean, m2 = _merge([allst[p, i] for p in range(world)])
            assert n == field[i].size
            np.testing.assert_allclose(mean, field[i].mean(), rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(m2 / n, field[i].var(), rtol=1e-10)
        # phase 0: rows -> m; the receive buffer is the forward Legendre GEMM's A:
        # exchange column k' = p*W + j of slab i, row r at p*(nm*R*2W) + (i*R + r)*2W + j
        sc, rc = latband.exchange_counts(world, rank, nlat, mmax, rows, own, R, 0)
        send = torch.from_numpy(_pack_fwd(X[:, loc], perm, B, C, bw, npair, W))
        assert send.numel() == sum(sc)
        recv = torch.zeros(sum(rc))
        comm.all_to_all(send, sc, recv, rc)
        buf = recv.numpy()
        blk = nm * R * 2 * W
        E = np.zeros((nm, R, world * W), dtype=np.float32)   # what the inverse GEMM writes
        O = np.zeros((nm, R, world * W), dtype=np.float32)
        for p in range(world):
            ap, bwp, npp = _band(rows, p, nlat)
            for i, m in enumerate(mine):
                for r, (b, ri, c) in enumerate(_rows_of(B, C)):
                    v = X[b * C + c, :, m]
                    v = v.real if ri == 0 else v.imag
                    base = p * blk + (i * R + r) * 2 * W
                    ks = np.arange(ap, ap + bwp)
                    kp = ks[:npp]
                    xs = v[ks].copy()
                    xs[:npp] += v[nlat - 1 - kp]
                    np.testing.assert_allclose(buf[base:base + bwp], xs, rtol=1e-6, atol=1e-6)
                    np.testing.assert_allclose(buf[base + W:base + W + npp],
                                               v[kp] - v[nlat - 1 - kp], rtol=1e-6, atol=1e-6)
                    assert not buf[base + bwp:base + W].any()
                    assert not buf[base + W + npp:base + 2 * W].any()
                    # identity "transform": E = Xs / 2 on pairs (Xs on the equator), O = Xa / 2
                    e = buf[base:base + bwp].copy()
                    e[:npp] *= 0.5
                    E[i, r, p * W:p * W + bwp] = e
                    O[i, r, p * W:p * W + npp] = 0.5 * buf[base + W:base + W + npp]
        # phase 1: m -> rows; the send buffer [dst p][slab][R][E_p | O_p]
        sc1, rc1 = latband.exchange_counts(world, rank, nlat, mmax, rows, own, R, 1)
        send1 = np.zeros((world, nm, R, 2 * W), dtype=np.float32)
        for p in range(world):
            send1[p, :, :, :W] = E[:, :, p * W:(p + 1) * W]
            send1[p, :, :, W:] = O[:, :, p * W:(p + 1) * W]
        send1 = torch.from_numpy(send1.reshape(-1))
        assert send1.numel() == sum(sc1)
        recv1 = torch.zeros(sum(rc1))
        comm.all_to_all(send1, sc1, recv1, rc1)
        Y = _unpack_inv(recv1.numpy(), perm, mact, B, C, bw, npair, W, mmax)
        want = X[:, loc].copy()
        want[:, :, mact:] = 0
        np.testing.assert_allclose(Y, want, rtol=1e-5, atol=1e-5)
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


class _FakeWork:
    def __init__(self, log, tag):
        self.log, self.tag = log, tag

    def wait(self):
        self.log.append(("wait",) + self.tag)


class _FakeComm:
    """Deferred collectives (the RCCL path's shape): issue returns a _Pending whose
    wait() is logged; nothing completes until then."""

    def __init__(self, log):
        self.log = log

    def all_gather_async(self, t):
        tag = ("all_gather", t["k"], t["stage"])
        self.log.append(("issue",) + tag)
        return latband._Pending(_FakeWork(self.log, tag), value=("gathered", t["k"], t["stage"]))

    def all_to_all_async(self, send, sc, recv, rc):
        tag = ("all_to_all", send["k"], send["stage"])
        self.log.append(("issue",) + tag)
        return latband._Pending(_FakeWork(self.log, tag))


def _fake_sub_batch(k, log, nstages=5):
    """A stage generator shaped like LatBandBlock.stages: stage s runs (logged), then
    posts a collective on its slot's buffers; the next stage may only run (and so
    reuse the slot's buffers) after that collective's wait."""
    for s in range(nstages - 1):
        log.append(("stage", k, s))
        buf = {"k": k, "stage": s}
        if s % 3 == 0:
            res = yield ("all_gather", buf)
            assert res == ("gathered", k, s)
        else:
            res = yield ("all_to_all", buf, [1], buf, [1])
            assert res is None
    log.append(("stage", k, nstages - 1))
    return f"out{k}"


@pytest.mark.parametrize("K", [1, 2, 4])
def test_drive_pipelined_issue_wait_order_with_deferred_handles(K):
    """_drive_pipelined against deferred (RCCL-style) handles: every collective is
    waited for exactly once, before its sub-batch's next stage runs (so a slot's
    send/recv buffers are reused only after the wait), each wait comes after the
    other started sub-batches' stages were enqueued behind the issue (the overlap),
    and the generators' return values come back in sub-batch order."""
    log = []
    gens = [_fake_sub_batch(k, log) for k in range(K)]
    outs = latband._drive_pipelined(gens, _FakeComm(log), stream=0)
    assert outs == [f"out{k}" for k in range(K)]
    issues = [e for e in log if e[0] == "issue"]
    waits = [e for e in log if e[0] == "wait"]
    assert sorted(i[1:] for i in issues) == sorted(w[1:] for w in waits)
    assert len(issues) == 4 * K
    pos = {e: i for i, e in enumerate(log)}
    for (_, kind, k, s) in issues:
        i_issue, i_wait = pos[("issue", kind, k, s)], pos[("wait", kind, k, s)]
        i_next = pos[("stage", k, s + 1)]
        assert i_issue < i_wait < i_next
        # between the issue and its wait, every other live sub-batch enqueued a stage
        if K > 1:
            between = {e[1] for e in log[i_issue:i_wait] if e[0] == "stage"}
            live = {j for j in range(K)
                    if ("stage", j, 0) in pos and pos[("stage", j, 0)] < i_wait
                    and pos[("stage", j, 4)] > i_issue and j != k}
            assert live <= between, (kind, k, s, live, between)
