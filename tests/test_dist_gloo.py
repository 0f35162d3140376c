"""World-size-2 gloo test of the N>1 path on CPU (no GPU): each process takes its subdomain from
the product's host planner (mcx_plan / mcx_plan_halo — the same plan the RCCL transport sends),
bootstraps a communicator id the way bench.py does (broadcast_object_list), exchanges halo
values with gloo send/recv in the plan's message order, and runs a distributed PETSc-CG
(Jacobi) on its owned rows of the oracle's matrix.  The gathered solution must match the
single-process oracle solve."""
import json
import os
import subprocess
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, grid, procs, q):
    sys.path.insert(0, ROOT)
    import torch

    import macroc_amd as M
    from oracle import oracle as O

    O.set_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        NX, NY, NZ = grid
        argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", procs[0],
                "-da_processors_y", procs[1], "-da_processors_z", procs[2]]
        obj = [b"x" * M.COMM_ID_BYTES if rank == 0 else None]  # bench.py's id bootstrap pattern
        dist.broadcast_object_list(obj, src=0)
        assert len(obj[0]) == M.COMM_ID_BYTES
        pl = M.plan(argv, rank, world)
        halo = M.plan_halo(argv, rank, world)
        ref = O.Problem(NX, NY, NZ, rtol=1e-12)  # global matrix, one rank = natural order
        ref.newton_step1()
        rp, ci = ref.csr()
        A = ref.A_values()
        b_all = ref.b()
        # owned nodes (natural ids), local order x fastest
        i, j, k = np.meshgrid(np.arange(pl["nx"]), np.arange(pl["ny"]), np.arange(pl["nz"]), indexing="ij")
        own = ((pl["xs"] + i) + (pl["ys"] + j) * NX + (pl["zs"] + k) * NX * NY).transpose(2, 1, 0).ravel()
        ghosts = np.concatenate([rv for _, _, rv in halo]) if halo else np.zeros(0, dtype=np.int64)
        known = np.concatenate([own, ghosts])
        pos = {int(n): t for t, n in enumerate(known)}
        assert len(set(known.tolist())) == len(known), "ghost received twice"
        rows = (3 * own[:, None] + np.arange(3)).ravel()

        def exchange(xloc):  # xloc: values of `own` nodes (n_own, 3) -> values of `known` nodes
            full = np.zeros((len(known), 3))
            full[: len(own)] = xloc
            ownpos = {int(n): t for t, n in enumerate(own)}
            reqs, bufs = [], []
            for nbr, send_nat, recv_nat in halo:
                sbuf = torch.from_numpy(np.ascontiguousarray(xloc[[ownpos[int(n)] for n in send_nat]]))
                rbuf = torch.zeros((len(recv_nat), 3), dtype=torch.float64)
                reqs.append(dist.isend(sbuf, nbr))
                reqs.append(dist.irecv(rbuf, nbr))
                bufs.append((recv_nat, rbuf, sbuf))
            for r_ in reqs:
                r_.wait()
            for recv_nat, rbuf, _ in bufs:
                for t, n in enumerate(recv_nat):
                    full[pos[int(n)]] = rbuf[t].numpy()
            return full

        import scipy.sparse as sp

        lut = np.full(NX * NY * NZ, -1, dtype=np.int64)
        lut[known] = np.arange(len(known))
        sel = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in rows])
        lrows = np.repeat(np.arange(len(rows)), [rp[r + 1] - rp[r] for r in rows])
        lcols = 3 * lut[ci[sel] // 3] + ci[sel] % 3
        assert (lut[ci[sel] // 3] >= 0).all(), "halo plan misses a stencil neighbour"
        Aloc = sp.csr_matrix((A[sel], (lrows, lcols)), shape=(len(rows), 3 * len(known)))

        def spmv(xloc):
            return Aloc @ exchange(xloc.reshape(-1, 3)).ravel()

        def allsum(v):
            t = torch.tensor([float(v)], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t[0])

        b = b_all[rows]
        diag = np.array([A[rp[r] + np.searchsorted(ci[rp[r]:rp[r + 1]], r)] for r in rows])
        dinv = np.where(diag != 0, 1.0 / np.where(diag != 0, diag, 1.0), 1.0)
        x = np.zeros_like(b)
        r_ = b.copy()
        z = r_ * dinv
        dp = np.sqrt(allsum(z @ z))
        ttol = max(1e-12 * dp, 1e-50)
        beta = allsum(z @ r_)
        its = 0
        p = None
        for it in range(10000):
            its = it + 1
            p = z.copy() if it == 0 else z + (beta / betaold) * p
            w = spmv(p)
            dpi = allsum(p @ w)
            betaold = beta
            a = beta / dpi
            x = x + a * p
            r_ = r_ - a * w
            z = r_ * dinv
            dp = np.sqrt(allsum(z @ z))
            if dp <= ttol:
                break
            beta = allsum(z @ r_)
        q.put((rank, rows, x, its, ref.du()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("grid,procs", [((10, 8, 8), (2, 1, 1)), ((8, 9, 6), (1, 2, 1))])
def test_gloo_world2_distributed_cg(grid, procs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, grid, procs, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    n = 3 * grid[0] * grid[1] * grid[2]
    x = np.zeros(n)
    for _, rows, xr, its, duref in res:
        x[rows] = xr
    duref = res[0][4]
    assert np.linalg.norm(x - duref) <= 1e-10 * np.linalg.norm(duref)


def _warmup_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import types

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 0's budget decides for every rank (rank 1's own budget would allow the warmup)
        tight = types.SimpleNamespace(wall=1e-3 if rank == 0 else 1e9, tail=0.0)
        loose = types.SimpleNamespace(wall=1e9, tail=0.0)
        q.put((rank, bench.room_for_warmup(10.0, 20, tight, rank, world),
               bench.room_for_warmup(10.0, 20, loose, rank, world)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_warmup_guard_is_collective():
    """bench.py's --wall guard: whether another warmup step runs is rank 0's decision, broadcast,
    so every rank runs the same number of warmup steps (the timed steps are never cut)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_warmup_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(2))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert res == [(0, False, True), (1, False, True)]


def _bench(args, env=None, timeout=300):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def test_bench_gpus_flag_starts_the_ranks():
    """`python bench.py --gpus 2` without a launcher starts two ranks itself
    (torch.distributed.run, 127.0.0.1); in --dry-run they bootstrap over gloo and rank 0 reports
    the ranks that joined -- never a one-rank line."""
    out = _bench(["--gpus", "2", "--dry-run"])
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line == {"dry_run": True, "n_gpus": 2, "world_size": 2}, line
    assert "starting 2 ranks" in out.stderr and "[rank 1] dry run" in out.stderr


def test_bench_gpus_flag_fails_loudly():
    """Without enough GPUs, or under a launcher whose WORLD_SIZE differs, --gpus N exits non-zero with
    the reason instead of measuring one GPU and printing n_gpus 1."""
    if not os.path.exists("/dev/kfd"):
        out = _bench(["--gpus", "2"])
        assert out.returncode != 0 and "--gpus 2 but 0 GPU(s) are visible" in out.stderr, out.stderr[-2000:]
        assert not out.stdout.strip()
    out = _bench(["--gpus", "1"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "--gpus 1 but the launcher started WORLD_SIZE=2" in out.stderr, out.stderr[-2000:]
    assert not out.stdout.strip()
