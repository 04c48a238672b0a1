"""Latitude-band sharded SFNO-Block forward.

The reference scales only by data-parallel replicas (one whole field per
process, MSFNO/main.py:1153).  Here ONE batch of fields is split over the ranks
of a process group: rank r keeps a band of the northern half, rows
[row_start[r], row_start[r+1]) of [0, nlat - nlat//2), plus the mirror rows
nlat-1-k of that band (``local_rows``), of every field for the pointwise / FFT /
1x1-conv / MLP work, and the zonal wavenumbers {m : m_owner[m] == r} for the
Legendre transforms and the spectral filter, which couple all latitudes of one m
but are independent across m.  Owning mirror pairs keeps the hemisphere fold of
the symmetric Legendre transform local, so the exchange buffers are the Legendre
GEMMs' operands as they are (include/msfno.h).
Per block forward (include/msfno.h, "Latitude-band sharded SFNO-Block"):

    stage 0  skip GEMM (side stream) + FFT of local rows      -> norm0 partials
    all_gather(norm0 partials)                                  2*B*C*3 doubles
    stage 1  norm0 affine, pack spectra by owner of m
    all_to_all                                    B*C*nlat*mact*8 bytes in total
    stage 2  Legendre fwd -> spectral filter -> Legendre inv on the local m-set
    all_to_all                                                     same volume
    stage 3  inverse FFT of local rows + skip                   -> norm1 partials
    all_gather(norm1 partials)
    stage 4  norm1 (+FiLM) -> MLP (+outer skip)

Resampling blocks (the network's first block, 721x1440 -> 120x240, and its
last one back, sfnonet.py:573-614) take rows of the input grid and return rows
of the output grid: the two grids have their own band partitions.  The linear
filter's per-mode weight (C, C, T, 2) is sharded with the m-set: each rank keeps
and streams only its modes' slice (layers.py:398-427, contractions.py:37-41).

``forward(..., chunks=K)`` splits the batch into K sub-batches whose stages are
software-pipelined: while one sub-batch's all-to-all is in flight (RCCL runs it
on its own stream, ``async_op=True``), the others' FFTs, Legendre GEMMs and MLPs
run on the compute stream — the comm/compute overlap of SURVEY.md §8e.

The result equals ``block(x, gamma, beta, scale)`` on the gathered field up to
fp32 rounding (Welford statistics are merged in fp64).  Collectives go through
``torch.distributed`` (backend "nccl" = RCCL over xGMI on MI355X; "gloo" is
supported by staging through host memory).  ``LocalGroup`` runs several
virtual ranks of one process in lock step, for tests and single-GPU use.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _native as N


def band_partition(world: int, nlat: int, lmax: int, mmax: int):
    """Default partition: balanced bands of the northern half (world + 1 row
    boundaries over [0, nlat - nlat//2)) + zig-zag m ownership."""
    rows = (ctypes.c_int * (world + 1))()
    own = (ctypes.c_int * mmax)()
    N.check(N.lib().msfno_band_partition(world, nlat, lmax, mmax, rows, own), "band_partition")
    return list(rows), list(own)


def local_rows(world: int, rank: int, nlat: int, row_start):
    """Global latitude rows of `rank`'s local rows, in local order: its band
    ascending, then the band's mirror rows ascending."""
    rs = (ctypes.c_int * (world + 1))(*row_start)
    cnt = ctypes.c_int()
    N.check(N.lib().msfno_band_local_rows(world, rank, nlat, rs, None, ctypes.byref(cnt)),
            "band_local_rows")
    rows = (ctypes.c_int * max(cnt.value, 1))()
    N.check(N.lib().msfno_band_local_rows(world, rank, nlat, rs, rows, ctypes.byref(cnt)),
            "band_local_rows")
    return list(rows)[:cnt.value]


def exchange_counts(world, rank, nlat, mmax, row_start, m_owner, R, phase):
    """(send_counts, recv_counts) in floats per peer for all-to-all `phase`."""
    rs = (ctypes.c_int * (world + 1))(*row_start)
    mo = (ctypes.c_int * mmax)(*m_owner)
    sc = (ctypes.c_longlong * world)()
    rc = (ctypes.c_longlong * world)()
    N.check(N.lib().msfno_band_exchange_counts(world, rank, nlat, mmax, rs, mo, R, phase, sc, rc),
            "band_exchange_counts")
    return list(sc), list(rc)


class _Done:
    def __init__(self, value=None):
        self.value = value

    def wait(self):
        return self.value


class _Pending:
    """An in-flight collective: ``wait()`` makes the current stream wait for it
    (no host block with RCCL) and returns its result tensor (or None)."""

    def __init__(self, work, value=None):
        self.work, self.value = work, value

    def wait(self):
        self.work.wait()
        return self.value


class TorchComm:
    """Collectives of one torch.distributed process group."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.host = dist.get_backend(group) == "gloo"

    def all_agree(self, ok: bool) -> bool:
        """True on every rank iff `ok` on every rank (a MIN all-reduce): collective
        decisions such as capture-or-eager, so no rank replays recorded collectives
        while a peer steps eagerly."""
        dev = "cpu" if self.host else torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
        return bool(t.item())

    def quiesce(self):
        """Before a HIP-graph capture of this group's collectives: drain the device and
        let torch's ProcessGroupNCCL watchdog reap its completed work.  The watchdog
        polls each pending work's end event; on HIP a query of an event whose stream
        (RCCL's internal stream, which joins the capture) is capturing fails with
        hipErrorCapturedEvent and the watchdog aborts the process.  Works issued during
        capture are not handed to the watchdog, so an empty list before capture_begin
        avoids the race."""
        if self.host:
            return
        import time
        torch.cuda.synchronize()
        time.sleep(0.35)  # > 3 watchdog polling periods (100 ms)

    def all_gather(self, t):
        src = t.cpu() if self.host else t
        parts = [torch.empty_like(src) for _ in range(self.world)]
        self.dist.all_gather(parts, src, group=self.group)
        return torch.stack(parts).to(t.device)

    def all_to_all(self, send, send_counts, recv, recv_counts):
        ns, nr = sum(send_counts), sum(recv_counts)
        if self.host:
            r = torch.empty(nr, dtype=recv.dtype)
            self.dist.all_to_all_single(r, send[:ns].cpu(), recv_counts, send_counts,
                                        group=self.group)
            recv[:nr].copy_(r)
        else:
            self.dist.all_to_all_single(recv[:nr], send[:ns], recv_counts, send_counts,
                                        group=self.group)

    def all_gather_async(self, t):
        if self.host:
            return _Done(self.all_gather(t))
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        w = self.dist.all_gather_into_tensor(out, t, group=self.group, async_op=True)
        return _Pending(w, out)

    def all_to_all_async(self, send, send_counts, recv, recv_counts):
        if self.host:
            self.all_to_all(send, send_counts, recv, recv_counts)
            return _Done()
        ns, nr = sum(send_counts), sum(recv_counts)
        w = self.dist.all_to_all_single(recv[:nr], send[:ns], recv_counts, send_counts,
                                        group=self.group, async_op=True)
        return _Pending(w)


def _drive(gen, comm):
    """Run one rank's stage generator against `comm`."""
    req = next(gen)
    while True:
        if req[0] == "all_gather":
            res = comm.all_gather(req[1])
        else:
            _, send, sc, recv, rc = req
            comm.all_to_all(send, sc, recv, rc)
            res = None
        try:
            req = gen.send(res)
        except StopIteration as stop:
            return stop.value


def _issue(req, comm):
    if req[0] == "all_gather":
        return comm.all_gather_async(req[1])
    _, send, sc, recv, rc = req
    return comm.all_to_all_async(send, sc, recv, rc)


def _drive_pipelined(gens, comm, stream):
    """Software pipeline over sub-batch generators (one per sub-batch, stages
    0..4 with a collective between consecutive stages).  At tick t every started
    generator advances one stage, the one furthest along first, and sub-batch t
    starts: the collective a stage issues (async) is waited for only one tick
    later, after the other sub-batches' stages have been enqueued behind it.  A
    profiler mark ("band_exchange") brackets each wait on the compute stream, so
    the stage profile shows the exchange time that was NOT hidden."""
    K = len(gens)
    pending = [None] * K
    alive = [True] * K
    outs = [None] * K
    t = 0
    while any(alive):
        for k in range(min(t + 1, K)):
            if not alive[k]:
                continue
            if t == k:
                req = next(gens[k])
            else:
                h = pending[k]
                if isinstance(h, _Pending):
                    N.profile_mark("band_exchange", stream)
                res = h.wait()
                try:
                    req = gens[k].send(res)
                except StopIteration as stop:
                    alive[k] = False
                    pending[k] = None
                    outs[k] = stop.value
                    continue
            pending[k] = _issue(req, comm)
        t += 1
    return outs


class LocalGroup:
    """Lock-step execution of several virtual ranks in one process (the
    exchanges become device copies).  Used by the parity tests to run the
    sharded path on one GPU, and by world-size-1 runs."""

    @staticmethod
    def all_agree(ok: bool) -> bool:
        """Every virtual rank lives in this process and decides with it."""
        return bool(ok)

    @staticmethod
    def quiesce():
        torch.cuda.synchronize()

    @staticmethod
    def _exchange(reqs):
        """Serve one collective posted by every virtual rank (``reqs[r]``); returns
        each rank's result."""
        W = len(reqs)
        kind = reqs[0][0]
        assert all(r[0] == kind for r in reqs), "ranks out of step"
        if kind == "all_gather":
            stacked = torch.stack([r[1] for r in reqs])
            return [stacked] * W
        offs = []
        for p in range(W):
            o, acc = [], 0
            for c in reqs[p][2]:
                o.append(acc)
                acc += c
            offs.append(o)
        for q in range(W):
            recv, rc = reqs[q][3], reqs[q][4]
            acc = 0
            for p in range(W):
                n = rc[p]
                assert reqs[p][2][q] == n, "send/recv counts disagree"
                src = reqs[p][1][offs[p][q]:offs[p][q] + n]
                if src.data_ptr() != recv[acc:acc + n].data_ptr():
                    recv[acc:acc + n].copy_(src)
                acc += n
        return [None] * W

    @staticmethod
    def run(gens):
        reqs = [next(g) for g in gens]
        outs = [None] * len(gens)
        live = list(range(len(gens)))
        while live:
            res = LocalGroup._exchange([reqs[i] for i in live])
            nxt = []
            for j, i in enumerate(live):
                try:
                    reqs[i] = gens[i].send(res[j])
                    nxt.append(i)
                except StopIteration as stop:
                    outs[i] = stop.value
            live = nxt
        return outs

    @staticmethod
    def run_pipelined(gens):
        """Lock-step virtual ranks with the sub-batch pipeline of ``_drive_pipelined``:
        ``gens[r][k]`` is rank r's generator of sub-batch k.  The stages are enqueued
        in the same interleaved order as on a real rank (at tick t every started
        sub-batch advances one stage, the one furthest along first, then sub-batch t
        starts); each exchange is served once every rank has posted it."""
        W, K = len(gens), len(gens[0])
        reqs = [[None] * K for _ in range(W)]
        outs = [[None] * K for _ in range(W)]
        alive = [True] * K
        t = 0
        while any(alive):
            for k in range(min(t + 1, K)):
                if not alive[k]:
                    continue
                if t == k:
                    for r in range(W):
                        reqs[r][k] = next(gens[r][k])
                    continue
                res = LocalGroup._exchange([reqs[r][k] for r in range(W)])
                done = 0
                for r in range(W):
                    try:
                        reqs[r][k] = gens[r][k].send(res[r])
                    except StopIteration as stop:
                        outs[r][k] = stop.value
                        done += 1
                assert done in (0, W), "ranks out of step"
                if done:
                    alive[k] = False
            t += 1
        return outs


class _BandPlan:
    def __init__(self, grid_in, grid_out, lmax, mmax, world, rank, row_in, row_out, m_owner,
                 device):
        self.device = device
        h = ctypes.c_void_p()
        ri = (ctypes.c_int * (world + 1))(*row_in)
        ro = (ctypes.c_int * (world + 1))(*row_out)
        mo = (ctypes.c_int * mmax)(*m_owner)
        with torch.cuda.device(device):
            N.check(N.lib().msfno_band_plan_create2(grid_in[0], grid_in[1], grid_out[0],
                                                    grid_out[1], lmax, mmax, world, rank, ri, ro,
                                                    mo, ctypes.byref(h)),
                    "msfno_band_plan_create2")
        self.handle = h
        self.key = None

    def load(self, fwd_table, inv_table, key):
        if key == self.key:
            return
        with torch.cuda.device(self.device):
            N.check(N.lib().msfno_band_plan_load_tables(self.handle, fwd_table.data_ptr(),
                                                        inv_table.data_ptr(),
                                                        N.stream_of(self.device)),
                    "msfno_band_plan_load_tables")
        self._tables = (fwd_table, inv_table)
        self.key = key

    def counts(self, R, phase):
        sc = (ctypes.c_longlong * 64)()
        rc = (ctypes.c_longlong * 64)()
        N.check(N.lib().msfno_band_plan_exchange_counts(self.handle, R, phase, sc, rc),
                "msfno_band_plan_exchange_counts")
        return sc, rc

    def linear_modes(self):
        """Global tril indices of this rank's modes (ascending)."""
        n = ctypes.c_longlong()
        N.check(N.lib().msfno_band_linear_modes(self.handle, None, ctypes.byref(n)),
                "msfno_band_linear_modes")
        buf = (ctypes.c_longlong * max(n.value, 1))()
        N.check(N.lib().msfno_band_linear_modes(self.handle, buf, ctypes.byref(n)),
                "msfno_band_linear_modes")
        return list(buf)[:n.value]

    def __del__(self):
        try:
            if self.handle:
                N.lib().msfno_band_plan_destroy(self.handle)
        except Exception:
            pass


class LatBandBlock:
    """One rank's share of a latitude-band sharded FourierNeuralOperatorBlock[_Filmed].

    ``block`` is the (replicated) block module; ``forward(x_local, gamma, beta,
    scale)`` takes this rank's rows of the input grid, ``take(x)`` =
    ``x[:, :, rows]``, and returns its rows of the output grid, ``rows_out`` (the
    same rows unless the block resamples); ``assemble`` puts the ranks' outputs
    back together.  ``row_start`` partitions the northern half of the input grid,
    ``row_start_out`` that of the output grid (default: balanced bands)."""

    def __init__(self, block, rank: int, world: int, row_start=None, m_owner=None,
                 device=None, row_start_out=None):
        fwd, inv = block._transforms()
        self.block = block
        self.rank, self.world = rank, world
        self.nlat, self.nlon, self.lmax, self.mmax = fwd.nlat, fwd.nlon, fwd.lmax, fwd.mmax
        self.nlat_out, self.nlon_out = inv.nlat, inv.nlon
        if row_start is None or m_owner is None:
            rs, own = band_partition(world, self.nlat, self.lmax, self.mmax)
            row_start = rs if row_start is None else row_start
            m_owner = own if m_owner is None else m_owner
        if row_start_out is None:
            if (self.nlat_out, self.nlon_out) == (self.nlat, self.nlon):
                row_start_out = row_start
            else:
                row_start_out = band_partition(world, self.nlat_out, self.lmax, self.mmax)[0]
        self.row_start, self.m_owner = list(row_start), list(m_owner)
        self.row_start_out = list(row_start_out)
        self.device = device if device is not None else torch.device("cuda",
                                                                    torch.cuda.current_device())
        self.plan = _BandPlan((self.nlat, self.nlon), (self.nlat_out, self.nlon_out), self.lmax,
                              self.mmax, world, rank, self.row_start, self.row_start_out,
                              self.m_owner, self.device)
        self._bufs = {}
        self._lin = None   # (key, local weight slice)

        self.rows = local_rows(world, rank, self.nlat, self.row_start)
        self.rows_out = local_rows(world, rank, self.nlat_out, self.row_start_out)
        self._idx = {}

    def _index(self, rows, device):
        key = (id(rows), str(device))
        if key not in self._idx:
            self._idx[key] = torch.tensor(rows, dtype=torch.long, device=device)
        return self._idx[key]

    def take(self, x):
        """This rank's input rows x[:, :, rows] (contiguous)."""
        return x.index_select(2, self._index(self.rows, x.device)).contiguous()

    @staticmethod
    def assemble(shards, outs):
        """The full output field from every rank's output rows (``shards[r]``'s
        ``forward`` result in ``outs[r]``)."""
        o = outs[0]
        nlat = shards[0].nlat_out
        y = torch.empty(o.shape[0], o.shape[1], nlat, o.shape[3], dtype=o.dtype, device=o.device)
        for s, t in zip(shards, outs):
            y.index_copy_(2, s._index(s.rows_out, t.device), t)
        return y

    def _tables(self):
        fwd, inv = self.block._transforms()
        key = tuple((t.data_ptr(), t._version, t.dtype, str(t.device))
                    for t in (fwd.weights, inv.pct))
        if key == self.plan.key:  # (re)load only when a table tensor changed
            return
        tabs = []
        for t in (fwd.weights, inv.pct):
            if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
                t = t.to(device=self.device, dtype=torch.float32).contiguous()
            tabs.append(t)
        self.plan.load(tabs[0], tabs[1], key)

    def _linear_weight(self, w):
        """This rank's slice w[:, :, modes, :] of the per-mode weight (cached until
        the parameter changes); the whole weight when the rank owns every mode."""
        key = (w.data_ptr(), w._version, w.dtype, str(w.device))
        if self._lin is not None and self._lin[0] == key:
            return self._lin[1]
        modes = self.plan.linear_modes()
        # the contraction reads fp32 (C, C, T, 2) contiguous, as _fill_desc passes it
        wf = w.detach().float().contiguous()
        if len(modes) == w.shape[2]:
            local = wf
        else:
            idx = torch.tensor(modes, dtype=torch.long, device=w.device)
            local = wf.index_select(2, idx).contiguous()
        self._lin = (key, local)
        return local

    def _buffers(self, B, C, slot):
        key = (B, C, slot)
        if key not in self._bufs:
            R = 2 * B * C
            cnt = []
            for ph in (0, 1):
                sc, rc = self.plan.counts(R, ph)
                cnt.append((list(sc)[:self.world], list(rc)[:self.world]))
            n = max(max(sum(s), sum(r)) for s, r in cnt)
            dev = self.device
            send = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
            # one rank: the exchange is the identity, so the receive buffer IS the send
            # buffer (stage 2's inverse GEMM overwrites the forward GEMM's input only
            # after that GEMM has run: stream order)
            recv = send if self.world == 1 else torch.empty_like(send)
            self._bufs[key] = dict(
                counts=cnt, send=send, recv=recv,
                stats=torch.empty(B * C, 3, dtype=torch.float64, device=dev))
        return self._bufs[key]

    def stages(self, x, gamma=None, beta=None, scale=1.0, slot=0, out=None):
        """Generator over the five native stages; yields the collective requests
        ("all_gather", tensor) / ("all_to_all", send, send_counts, recv, recv_counts)
        and returns this rank's output rows.  ``slot`` (0..63) must differ between
        sub-batches in flight at the same time."""
        x = N.require_device_f32(x, "band block input")
        B, C, H, W = x.shape
        if H != len(self.rows) or W != self.nlon or C != self.block.embed_dim_sfno:
            raise ValueError(f"x_local must be (B, {self.block.embed_dim_sfno}, {len(self.rows)}, "
                             f"{self.nlon}), got {tuple(x.shape)}")
        self._tables()
        d, keep = self.block.native_desc()
        if d.filter_type == N.FILTER_LINEAR:
            wl = self._linear_weight(self.block.filter_layer.filter.w)
            d.lin_w = wl.data_ptr()
            keep.append(wl)
        if gamma is not None:
            gamma = gamma.detach().float().reshape(B, C).contiguous()
            beta = beta.detach().float().reshape(B, C).contiguous()
        L = N.lib()
        wkey = self.block.wcache_attach(d, keep, x.device)  # prepared-weight images
        bufs = self._buffers(B, C, slot)
        nbytes = L.msfno_band_workspace_size(d, self.plan.handle, B)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        if out is None:
            out = torch.empty(B, C, len(self.rows_out), self.nlon_out, dtype=torch.float32,
                              device=x.device)
        io = N.BandIO(x=x.data_ptr(), gamma=N.ptr(gamma), beta=N.ptr(beta),
                      film_scale=float(scale), out=out.data_ptr(), send=bufs["send"].data_ptr(),
                      recv=bufs["recv"].data_ptr(), stats_local=bufs["stats"].data_ptr(),
                      stats_all=None, slot=int(slot))
        stream = N.stream_of(x.device)

        def stage(i):
            with torch.cuda.device(x.device):
                N.check(L.msfno_band_block_stage(d, self.plan.handle, i, ctypes.byref(io), B,
                                                 ws.data_ptr(), nbytes, stream),
                        f"band stage {i}")

        (sc0, rc0), (sc1, rc1) = bufs["counts"]
        stage(0)
        st = yield ("all_gather", bufs["stats"])
        io.stats_all = st.data_ptr()
        stage(1)
        yield ("all_to_all", bufs["send"], sc0, bufs["recv"], rc0)
        stage(2)
        yield ("all_to_all", bufs["send"], sc1, bufs["recv"], rc1)
        stage(3)
        st2 = yield ("all_gather", bufs["stats"])
        io.stats_all = st2.data_ptr()
        stage(4)
        self.block.wcache_commit(wkey)
        del keep, st, st2
        return out

    def chunk_stages(self, x, gamma=None, beta=None, scale=1.0, chunks=1):
        """(out, generators): the batch split into ``chunks`` sub-batches, each with
        its own slot, writing its rows of ``out`` (the pipeline of ``forward``)."""
        x = N.require_device_f32(x, "band block input")
        B = x.shape[0]
        K = max(1, min(int(chunks), B, 64))
        out = torch.empty(B, x.shape[1], len(self.rows_out), self.nlon_out, dtype=torch.float32,
                          device=x.device)
        bounds = [B * k // K for k in range(K + 1)]
        gens = []
        for k in range(K):
            b0, b1 = bounds[k], bounds[k + 1]
            g = gamma[b0:b1] if gamma is not None else None
            be = beta[b0:b1] if beta is not None else None
            gens.append(self.stages(x[b0:b1], g, be, scale, slot=k, out=out[b0:b1]))
        return out, gens

    def forward(self, x, gamma=None, beta=None, scale=1.0, comm=None, chunks=1):
        """This rank's output rows.  ``chunks`` > 1 pipelines that many sub-batches
        (exchanges overlapped with the other sub-batches' compute)."""
        B = x.shape[0]
        K = max(1, min(int(chunks), B, 64))
        if K == 1:
            gen = self.stages(x, gamma, beta, scale)
            if self.world == 1 and comm is None:
                return LocalGroup.run([gen])[0]
            return _drive(gen, comm if comm is not None else TorchComm())
        out, gens = self.chunk_stages(x, gamma, beta, scale, K)
        if self.world == 1 and comm is None:
            for gen in gens:
                LocalGroup.run([gen])
            return out
        _drive_pipelined(gens, comm if comm is not None else TorchComm(), N.stream_of(x.device))
        return out

    __call__ = forward


class LatBandNet:
    """One rank's share of a latitude-band sharded FourierNeuralOperatorNet[_Filmed]
    forward (sfnonet.py:406-860): the multi-GPU form of configs 3 / 5 (one 6 h step
    of ONE field spread over the ranks).  The encoder and decoder are pointwise, so
    each rank runs them on its own rows (pos_embed sliced to them); the 12 blocks are
    LatBandBlocks whose band partitions chain (block 0 takes rows of the full grid
    and returns rows of the (h, w) Gauss grid, the last block maps back).  ``rows``
    are this rank's rows of the full grid (``take`` / ``LatBandBlock.assemble``
    conventions); ``forward(x_local, sst, scale)`` returns its rows of the output."""

    def __init__(self, net, rank: int, world: int, device=None, comm=None, chunks=1,
                 inner="shard"):
        """``inner``: "shard" (every block latitude-band sharded: four collectives per
        block) or "replicate" (the first and last blocks, which carry the
        full grid, stay sharded; the inner blocks run unsharded on every rank on the
        whole (h, w) state, gathered once after block 0: one all-gather instead of four
        collectives per inner block, at the price of computing the small inner blocks
        on every rank)."""
        if inner not in ("shard", "replicate"):
            raise ValueError(f"inner must be 'shard' or 'replicate', not {inner!r}")
        self.net = net
        self.rank, self.world = rank, world
        self.comm = comm
        self.chunks = chunks
        self.inner = inner
        nb = len(net.blocks)
        replicate = inner == "replicate" and nb > 2
        self._replicate = replicate
        sharded = [0, nb - 1] if replicate else list(range(nb))
        self._shard_of = {i: LatBandBlock(net.blocks[i], rank, world, device=device)
                          for i in sharded}
        self.shards = [self._shard_of[i] for i in sharded]
        if replicate:
            first, last = self._shard_of[0], self._shard_of[nb - 1]
            # every rank's rows of block 0's output grid (the gather's layout)
            self._gather_rows = [local_rows(world, r, first.nlat_out, first.row_start_out)
                                 for r in range(world)]
            self._gather_nlat = first.nlat_out
            self._gather_idx = {}
            assert last.nlat == first.nlat_out, "inner blocks must keep block 0's output grid"
        else:
            for a, b in zip(self.shards, self.shards[1:]):
                assert a.rows_out == b.rows, "block band partitions do not chain"
        self.rows = self.shards[0].rows
        self.rows_out = self.shards[-1].rows_out
        self.nlat_out = self.shards[-1].nlat_out
        self._pos = None

    def take(self, x):
        return self.shards[0].take(x)

    def _pos_local(self, device):
        pe = self.net.pos_embed
        key = (pe.data_ptr(), pe._version, str(device))
        if self._pos is None or self._pos[0] != key:
            idx = torch.tensor(self.rows, dtype=torch.long, device=pe.device)
            self._pos = (key, pe.detach().index_select(2, idx).to(device).contiguous())
        return self._pos[1]

    def stages(self, x, sst=None, scale=1.0, slot=0):
        """Generator over the whole network's exchanges (see LatBandBlock.stages);
        returns this rank's output rows.  ``slot`` as in LatBandBlock.stages (one per
        sub-batch in flight)."""
        net = self.net
        filmed = getattr(net, "_filmed", None)
        gamma = beta = None
        if filmed is not None:
            film_mod = net.film_gen(sst) if net.film_gen is not None else sst
            gamma, beta = film_mod[:, 0], film_mod[:, 1]
        residual = x
        h = net.encoder.native_forward(x, addend=self._pos_local(x.device))
        h = net.pos_drop(h)  # sfnonet.py:674 / 827 (identity in eval)

        def film_args(i):
            if filmed is not None and filmed(i):
                k = i - (net.num_layers - net.film_layers)
                return (gamma[:, k], beta[:, k], scale)
            return ()

        if not self._replicate:
            for i, s in enumerate(self.shards):
                h = yield from s.stages(h, *film_args(i), slot=slot)
            return net.decode(h, residual)
        nb = len(net.blocks)
        h = yield from self._shard_of[0].stages(h, *film_args(0), slot=slot)
        h = yield from self._gather(h)
        for i in range(1, nb - 1):  # sfnonet.py:838-844, unsharded on every rank
            h = net.blocks[i](h, *film_args(i))
        last = self._shard_of[nb - 1]
        h = yield from last.stages(last.take(h), *film_args(nb - 1), slot=slot)
        return net.decode(h, residual)

    def _gather(self, h):
        """The whole (h, w) state from every rank's rows of it: the rows padded to the
        largest band, one all-gather, placed by each rank's row list."""
        B, C, n, W = h.shape
        pad = max(len(r) for r in self._gather_rows)
        buf = h.new_zeros(B, C, pad, W)
        buf[:, :, :n].copy_(h)
        parts = yield ("all_gather", buf)
        full = h.new_empty(B, C, self._gather_nlat, W)
        for r, rows in enumerate(self._gather_rows):
            key = (r, str(h.device))
            if key not in self._gather_idx:
                self._gather_idx[key] = torch.tensor(rows, dtype=torch.long, device=h.device)
            full.index_copy_(2, self._gather_idx[key], parts[r][:, :, :len(rows)])
        return full

    def chunk_stages(self, x, sst=None, scale=1.0, chunks=1):
        """Generators of ``chunks`` sub-batches (fields are independent), each with its
        own exchange slot; the ``sst`` / modulation batch is split the same way."""
        B = x.shape[0]
        K = max(1, min(int(chunks), B, 64))
        bounds = [B * k // K for k in range(K + 1)]
        return [self.stages(x[bounds[k]:bounds[k + 1]],
                            sst[bounds[k]:bounds[k + 1]] if sst is not None else None,
                            scale, slot=k) for k in range(K)]

    def forward(self, x, sst=None, scale=1.0, comm=None, chunks=None):
        """This rank's output rows.  ``chunks`` > 1 pipelines that many sub-batches
        through the whole network: while one sub-batch's exchange is in flight the
        others' blocks run (the LatBandBlock pipeline, across all 12 blocks)."""
        comm = comm if comm is not None else self.comm
        gens = self.chunk_stages(x, sst, scale, self.chunks if chunks is None else chunks)
        if len(gens) == 1:
            if self.world == 1 and comm is None:
                return LocalGroup.run(gens)[0]
            return _drive(gens[0], comm if comm is not None else TorchComm())
        if self.world == 1 and comm is None:
            outs = [LocalGroup.run([g])[0] for g in gens]
        else:
            outs = _drive_pipelined(gens, comm if comm is not None else TorchComm(),
                                    N.stream_of(x.device))
        return torch.cat(outs, dim=0)

    __call__ = forward
