"""Row-block distributed objective on CPU: the partition map the
library exports, the RCCL-id hand-off over gloo, and a NumPy model of the exact
per-step schedule of gpemu_dist.hip (cyclic tile rows + augmented [f H] row, column
groups with pending updates inside the group, broadcast of the diagonal inverse,
all-gather of the panel column, own-row trailing update per group) run on 2 and 3
gloo ranks against a dense factorisation, extended by the gradient schedule (rows of
L^-1 finished by their owner after its group's earlier rows, broadcast, own-row
updates per group, per-rank partials X_r^T X_r whose sum is A^-1).  NumPy is only the test's
stand-in for the HIP tile kernels."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gp_emu_uqsa_amd import distributed, native


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("n,P,q", [(1, 1, 0), (128, 2, 3), (1000, 4, 11), (16384, 8, 11), (65536, 8, 21),
                                   (700, 3, 0), (700, 3, 150), (1000, 4, 400)])
def test_partition_map(n, P, q):
    """Tile rows per rank including the ceil((q+1)/128) augmented rows (q = 150: two, as
    set_data stores them for the linear mean of d = 150 inputs)."""
    nb = (n + 127) // 128
    na = (q + 1 + 127) // 128
    rows = distributed.partition(n, P, q)
    assert sorted(t for r in rows.values() for t in r) == list(range(nb + na))
    for r in range(P):
        assert rows[r] == list(range(r, nb + na, P))
        assert native.dist_local_rows(n, P, r, q) == len(rows[r])
    assert native.dist_owner(P, nb) == nb % P


def _uid_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        def make():
            calls.append(1)
            return bytes(range(128))
        out[rank] = (distributed.share_unique_id(make_id=make), len(calls))
    finally:
        dist.destroy_process_group()


def test_unique_id_shared_from_rank0():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_uid_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    assert res[0][0] == res[1][0] == bytes(range(128))
    assert res[0][1] == 1 and res[1][1] == 0          # only rank 0 creates the id


B = 8   # model tile size (the library uses 128; the schedule does not depend on it)


def _problem(n, q, seed=3):
    rng = np.random.RandomState(seed)
    X = rng.uniform(size=(n, 2))
    d2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    A = np.exp(-d2 / 0.3) + 0.05 * np.eye(n)
    F = rng.normal(size=(n, q + 1))
    return A, F


def _sched_worker(rank, world, port, n, q, W, CW, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        A, F = _problem(n, q)
        nb = n // B
        Pc = q + 1
        NA = -(-Pc // B)                                              # augmented tile rows
        gstart = [k - k % W for k in range(nb)]                      # column groups of width W
        gend = [min(gstart[k] + W, nb) for k in range(nb)]
        # augmented matrix: tile rows nb .. nb+NA-1 hold F^T (zero padded), their block 0
        full = np.zeros(((nb + NA) * B, (nb + NA) * B))
        full[:n, :n] = A
        full[n:n + Pc, :n] = F.T
        mine = [t for t in range(nb + NA) if t % world == rank]
        loc = {t: full[t * B:(t + 1) * B, :].copy() for t in mine}     # own tile rows
        logdet = np.zeros(nb + 1)
        gpanel = {}   # the group's gathered panel columns below it: gpanel[c][t] = L(t, c), t >= ge
        for k in range(nb):
            owner = k % world
            gb, ge = gstart[k], gend[k]
            kp = (k - gb) * B                                         # pending columns [gb, k)
            rows = [t for t in mine if t > k]
            # the owner: its diagonal tile less the pending update from its own row, factored;
            # broadcast block [-M | Dinv], M = Dinv L(k, gb:k) (one broadcast per step)
            bc = torch.zeros(B, kp + B, dtype=torch.float64)
            if owner == rank:
                for c in range(gb, k):
                    loc[k][:, k * B:(k + 1) * B] -= loc[k][:, c * B:(c + 1) * B] @ loc[k][:, c * B:(c + 1) * B].T
                L = np.linalg.cholesky(loc[k][:, k * B:(k + 1) * B])
                loc[k][:, k * B:(k + 1) * B] = L
                logdet[k] = np.log(np.diag(L)).sum()
                Dinv = np.linalg.inv(L)
                bc = torch.from_numpy(np.hstack([-(Dinv @ loc[k][:, gb * B:k * B]), Dinv]))
            dist.broadcast(bc, src=owner)
            BC = bc.numpy()
            for t in rows:                                            # panel: [L(t, gb:k) A(t,k)] [-M Dinv]^T
                loc[t][:, k * B:(k + 1) * B] = loc[t][:, gb * B:(k + 1) * B] @ BC.T
            if k + 1 == ge:                                           # group closes
                # ONE all-gather of the group's columns on the rows below it, then the
                # trailing update of the own rows
                below = [[t for t in range(nb + NA) if t % world == r and t >= ge] for r in range(world)]
                maxT = max(len(b) for b in below)
                send = torch.zeros(max(maxT, 1), ge - gb, B, B, dtype=torch.float64)
                for i, t in enumerate(below[rank]):
                    for w in range(ge - gb):
                        send[i, w] = torch.from_numpy(loc[t][:, (gb + w) * B:(gb + w + 1) * B])
                recv = [torch.zeros_like(send) for _ in range(world)]
                dist.all_gather(recv, send)
                gpanel = {c: {} for c in range(gb, ge)}
                for r in range(world):                               # unpermute
                    for i, t in enumerate(below[r]):
                        for w in range(ge - gb):
                            gpanel[gb + w][t] = recv[r][i, w].numpy()
                for t in [t for t in mine if t >= ge]:
                    for j in range(ge, t + 1):
                        for c in range(gb, ge):
                            loc[t][:, j * B:(j + 1) * B] -= loc[t][:, c * B:(c + 1) * B] @ gpanel[c][j].T
        ld = torch.from_numpy(logdet)
        dist.all_reduce(ld)
        # -Gram: each owner of an augmented row places its rows (lower tiles), all-reduced
        g = torch.zeros(Pc, Pc, dtype=torch.float64)
        for u in range(NA):
            if (nb + u) in loc:
                p0, pc = u * B, min(Pc - u * B, B)
                g[p0:p0 + pc, :p0 + pc] = torch.from_numpy(-loc[nb + u][:pc, nb * B:nb * B + p0 + pc].copy())
        dist.all_reduce(g)
        G = g.numpy()
        G = np.tril(G) + np.tril(G, -1).T
        # gradient: X = L^-1 by the recursive TRTRI (gpemu_dist.hip ensure_grad): pairs
        # [t0,h), [h,t1) of s tile columns, in column chunks of width <= CW: the own rows
        # c0:h of X11's chunk columns packed by pair, all-gathered, unpermuted by owner;
        # each rank's columns of M^T = X11^T L21^T, all-gathered, unpermuted; then
        # X21 = -X22 M on its own rows
        def unpermute_index(g, g0):
            r = g % world
            first = g0 + (r - g0 % world) % world
            return r, (g - first) // world

        Xl = {t: np.zeros((B, nb * B)) for t in mine if t < nb}
        for t in Xl:
            Xl[t][:, t * B:(t + 1) * B] = np.linalg.inv(loc[t][:, t * B:(t + 1) * B])
        s = 2
        while s // 2 < nb:
            a = s // 2
            pairs = [(t0, t0 + a, min(t0 + s, nb)) for t0 in range(0, nb - a, s)]
            for j0 in range(0, a, CW):
                cw, rows1 = min(CW, a - j0), a - j0
                mx1 = -(-rows1 // world)
                send = torch.zeros(len(pairs), mx1, B, cw * B, dtype=torch.float64)
                for p, (t0, h, t1) in enumerate(pairs):
                    c0 = t0 + j0
                    for j, t in enumerate([t for t in range(c0, h) if t % world == rank]):
                        send[p, j] = torch.from_numpy(Xl[t][:, c0 * B:(c0 + cw) * B])
                recv = [torch.zeros_like(send) for _ in range(world)]
                dist.all_gather(recv, send)
                mx2 = max(-(-(t1 - h) // world) for (_, h, t1) in pairs)
                send2 = torch.zeros(len(pairs), mx2, cw * B, B, dtype=torch.float64)
                for p, (t0, h, t1) in enumerate(pairs):
                    c0 = t0 + j0
                    G1 = np.zeros((rows1 * B, cw * B))
                    for gr in range(c0, h):
                        r, j = unpermute_index(gr, c0)
                        G1[(gr - c0) * B:(gr - c0 + 1) * B] = recv[r][p, j].numpy()
                    for j, i in enumerate([t for t in range(h, t1) if t % world == rank]):
                        send2[p, j] = torch.from_numpy(G1.T @ loc[i][:, c0 * B:h * B].T)
                recv2 = [torch.zeros_like(send2) for _ in range(world)]
                dist.all_gather(recv2, send2)
                for p, (t0, h, t1) in enumerate(pairs):
                    c0 = t0 + j0
                    G2 = np.zeros((cw * B, (t1 - h) * B))
                    for gc in range(h, t1):
                        r, j = unpermute_index(gc, h)
                        G2[:, (gc - h) * B:(gc - h + 1) * B] = recv2[r][p, j].numpy()
                    for i in [t for t in range(h, t1) if t % world == rank]:
                        Xl[i][:, c0 * B:(c0 + cw) * B] = -(Xl[i][:, h * B:(i + 1) * B] @ G2[:, :(i - h + 1) * B].T)
            s *= 2
        part = np.zeros((nb * B, nb * B))
        for xr in Xl.values():
            part += xr.T @ xr
        ainv = torch.from_numpy(part)
        dist.all_reduce(ainv)     # the library contracts each partial instead; the sum is A^-1
        out[rank] = (2.0 * float(ld.sum()), G.tolist(), ainv.numpy().tolist())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,q,CW", [(2, 1, 3, 8), (3, 1, 11, 2), (2, 3, 19, 1), (3, 4, 3, 3)])
def test_schedule_model_matches_dense(world, W, q, CW):
    """The row-block schedule of gpemu_dist.hip in NumPy over gloo ranks: per column step
    ONE broadcast from the diagonal owner of [-M | Dinv] (M = Dinv L(k, gb:k): the group's
    pending columns of row k ride with the inverse, so no rank needs a gathered panel row
    inside the group), and ONE all-gather per column group of its columns on the rows below
    it, before the group's trailing update.  W: column-group width (1 = a trailing update per
    column; 3 and 4 leave a ragged last group of the 7 tile columns); q + 1 > 8 spreads
    [f H]^T over 2-3 augmented tile rows; CW: the TRTRI's column-chunk width (1 and 2 split
    its upper levels)."""
    n = 7 * B
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_sched_worker, args=(world, port, n, q, W, CW, out), nprocs=world, join=True)
        res = dict(out)
    A, F = _problem(n, q)
    L = np.linalg.cholesky(A)
    Z = np.linalg.solve(L, F)
    Ainv = np.linalg.inv(A)
    for r in range(world):
        logdet, G, ainv = res[r]
        assert abs(logdet - np.linalg.slogdet(A)[1]) < 1e-10 * abs(logdet)
        assert np.max(np.abs(np.array(G) - Z.T @ Z)) < 1e-10 * np.max(np.abs(Z.T @ Z))
        assert np.max(np.abs(np.array(ainv) - Ainv)) < 1e-9 * np.max(np.abs(Ainv))


def _lockstep_worker(rank, world, port, out):
    from gp_emu_uqsa_amd import replicas
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sharded = replicas.my_items(5)
        distributed._OBJECTIVE = object()      # stand-in for an enabled collective objective
        try:
            lockstep = replicas.my_items(5)
            merged = replicas.gather_results({i: (float(i), np.zeros(1), None) for i in lockstep}, 5)
        finally:
            distributed._OBJECTIVE = None
        out[rank] = (sharded, lockstep, sorted(merged))
    finally:
        dist.destroy_process_group()


def test_collective_objective_runs_every_try_on_every_rank():
    """With distributed.enable_objective() each evaluation is collective, so every
    rank must step every multistart chain (no replica sharding)."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_lockstep_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    assert res[0][0] == [0, 2, 4] and res[1][0] == [1, 3]
    for r in range(2):
        assert res[r][1] == [0, 1, 2, 3, 4] and res[r][2] == [0, 1, 2, 3, 4]
