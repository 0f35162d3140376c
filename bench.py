"""bench.py — Newton-iteration throughput of the MI355X MacroC hot path (BASELINE.json metric).

One "step" = the Newton iteration of time step 1 that performs the solve (src/main.c:61-79 of
the reference): VecZeroEntries(u) + apply_bc_on_u(U = -0.001), then set_strains, homogenize
(isotropic-elastic Gauss-point callback), assembly_res + VecNorm, assembly_jac (+ Dirichlet
rows/columns), KSPSolve(CG, Jacobi, rtol 1e-8) and u += du — every step redoes all of it from
the same state, nothing is cached across steps.  Workload: 256^3 nodes per GPU
(BASELINE configs[2]; weak scaling: N GPUs own a global grid of 256*(px,py,pz)).

    python bench.py [--gpus N] [--steps K] [--warmup W]      (N > 1: starts the N ranks itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

The headline storage is the default AIJ one: value-indexed (one index byte per 3x3 block into
a dictionary of the matrix's distinct blocks, rebuilt by every assembly inside the step; exact
values), its SpMV rows summed with fused multiply-adds (-mat_vi_fma 1, the default).  On one GPU
the same storage with the bit-exact CPU-order rows (-mat_vi_fma 0) and the AIJ-split storage
of the same matrix are measured after it (1 warmup + 1 step each, `variants` in the line;
`--variants aij-vi-exact,aij-split,aij-blocks,sbaij` for more) while the `--budget` wall time
lasts.  Also on one GPU, BASELINE config 5's path (128^3, the J2 Gauss-point law, three time
steps of non-linear Newton, default AIJ storage with exception nodes) is run and reported as
`config5` (`--config5 0` skips it).  Rank 0 prints ONE JSON line (the contract in the task
statement / DESIGN.md §6) once the headline, the variants and the CPU baseline are measured.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

T_START = time.perf_counter()  # wall-clock budget of the whole invocation (variants are guarded by it)


def launch_ranks():
    """`--gpus N` with N > 1 and no WORLD_SIZE in the environment (a plain `python bench.py --gpus 8`):
    start the N ranks here, one process per GPU through torch.distributed.run on 127.0.0.1, and
    exit with its status.  Runs before torch or the library is imported, so this parent never
    touches a GPU and never execs: the ranks are children.  Under a launcher (WORLD_SIZE set) a
    --gpus that differs from WORLD_SIZE is an error, never a silent one-rank run."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=None)
    pre.add_argument("--dry-run", action="store_true")
    a, _ = pre.parse_known_args()
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if a.gpus is not None and a.gpus != int(ws):
            sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={ws} ranks")
        return
    if a.gpus is None or a.gpus == 1:
        return
    if a.gpus < 1:
        sys.exit(f"bench.py: --gpus {a.gpus}")
    import socket

    ndev = a.gpus if a.dry_run else device_count()
    if ndev < a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but {ndev} GPU(s) are visible; one rank per GPU needs {a.gpus}")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: --gpus {a.gpus}: starting {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    sys.exit(subprocess.run(cmd).returncode)


def device_count():
    """GPUs visible to this process, counted without creating a device context (the parent of
    launch_ranks must not initialise the GPU): /dev/kfd absent -> 0, else torch's count, which
    on this image does not initialise the runtime; HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES
    respected by torch."""
    if not os.path.exists("/dev/kfd"):
        return 0
    out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                         capture_output=True, text=True, timeout=300)
    try:
        return int(out.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


if __name__ == "__main__":
    launch_ranks()

# torch first: the library then binds to the HIP runtime torch already loaded (one runtime per
# process); torch is only plumbing here (process group for barriers / max-over-ranks).
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import numpy as np  # noqa: E402

import macroc_amd as M  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# matrix storages: the reference's -dm_mat_type aij (DMSetMatType(da, MATAIJ), src/init.c:92) held
# value-indexed (one index byte per value into the matrix's <= 256 distinct values; the default,
# with fallback), as upper blocks + exact bf16 lower corrections (aij-split) or as plain AIJ blocks
# summed in the reference's MatMult order (inode column pairs); -dm_mat_type sbaij through DMSetFromOptions (src/init.c:93)
STORAGE_ARGS = {"aij": ["-dm_mat_type", "aij"], "aij-vi-exact": ["-dm_mat_type", "aij", "-mat_vi_fma", 0],
                "aij-split": ["-dm_mat_type", "aij", "-mat_aij_vi", 0],
                "aij-blocks": ["-dm_mat_type", "aij", "-mat_aij_vi", 0, "-mat_aij_split", 0],
                "sbaij": ["-dm_mat_type", "sbaij"]}
STORAGE_NAME = {0: "aij-blocks", 1: "sbaij", 2: "aij-split", 3: "aij-vi"}
KERNEL_NAME = {0: "k_spmv (AIJ stencil blocks, CPU AIJ row order)",
               1: "k_spmv_symp (SBAIJ phased z-marching tiles)",
               2: "k_spmv_symp<AIJS> (AIJ-split: upper blocks + bf16 lower corrections, z-marching)",
               3: "k_spmv_vi (value-indexed AIJ: index bytes + dictionary in LDS, CPU AIJ row order)",
               # value-indexed, one byte per 3x3 block (vi_blocks > 0): z-marching x ring in LDS
               # where a tile marches >= 4 planes (k_spmv_vibm), else x gathered (k_spmv_vib)
               "3b": "k_spmv_vibm (block-indexed AIJ: one byte per 3x3 block; x ring in LDS; wave-uniform blocks "
                     "from scalar loads, others from the dictionary in LDS; 16x4-node waves; rows summed with fused "
                     "multiply-adds)",
               "3be": "k_spmv_vibm (block-indexed AIJ as above, -mat_vi_fma 0: multiply then add in the CPU AIJ "
                      "row order, bit-exact)",
               "3bs": "k_spmv_st + k_spmv_face, one SpMV = the two launches (block-indexed AIJ, default-stencil "
                      "path: k_spmv_st marches the interior with the interior stencil's blocks from scalar loads, two "
                      "z-planes per step, x ring in LDS, no index bytes; k_spmv_face computes the 6 domain faces with "
                      "their class stencils from LDS-staged 64x4 patches and the listed rows from their index bytes; "
                      "rows summed with fused multiply-adds)"}


def kernel_name(r):
    if r["storage_id"] == 3 and r["vi_blocks"]:
        if r.get("st_listed", -1) >= 0:
            return KERNEL_NAME["3bs"]
        return KERNEL_NAME["3be" if r.get("exact") else "3b"]
    return KERNEL_NAME[r["storage_id"]]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def rank_grid(n):
    return {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2), 16: (4, 2, 2)}.get(n) or (n, 1, 1)


def pmc_commit(mat_type, NX, NY, NZ):
    """The commit the committed PMC traffic passes of this kernel were measured at (or None)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_spmv.json")
    try:
        with open(path) as f:
            return (json.load(f).get(f"{mat_type}:{NX}x{NY}x{NZ}") or {}).get("commit")
    except (OSError, ValueError):
        return None


def pmc_traffic(mat_type, NX, NY, NZ):
    """HBM bytes per SpMV launch from the committed rocprofv3 PMC passes (profiles/pmc_spmv.json:
    (FETCH_SIZE*2 [gfx950 wide-read correction] + WRITE_SIZE) * 1024 per launch, same kernel and
    grid), or None when no matching measurement exists."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_spmv.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(f"{mat_type}:{NX}x{NY}x{NZ}")
        return e["hbm_bytes_per_launch"] if e else None
    except (OSError, ValueError, KeyError):
        return None


def lds_limiter(mat_type, NX, NY, NZ):
    """LDS-array and VALU busy fractions of the headline SpMV kernel from the committed rocprofv3
    SQ counter passes (profiles/pmc_vibm.json, tools/pmc_vibm.sh: SQ_LDS_IDX_ACTIVE per CU and
    SQ_ACTIVE_INST_VALU per SIMD over SQ_BUSY_CYCLES per shader engine), or None.  The
    value-indexed kernel streams only ~80 B per node from HBM; what bounds it is reported beside
    the HBM roofline."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_vibm.json")
    try:
        with open(path) as f:
            e = json.load(f).get(f"{mat_type}:{NX}x{NY}x{NZ}")
        if not e:
            return None
        busy = {"LDS": e["lds_busy_frac"], "VALU": e.get("valu_busy_frac")}
        out = {"resource": "latency (no unit saturated)" if max(v or 0 for v in busy.values()) < 0.7 else
               max(busy, key=lambda k: busy[k] or 0),
               "lds_busy_frac": e["lds_busy_frac"], "valu_busy_frac": e.get("valu_busy_frac"),
               "wait_any_frac": e.get("wait_any_frac"), "kernel": e["kernel"],
               "valu_insts_per_wave_plane": e["valu_insts_per_wave_plane"],
               "lds_insts_per_wave_plane": e["lds_insts_per_wave_plane"],
               "source": "profiles/pmc_vibm.json (committed SQ counter passes, not measured by this run)",
               "measured": e.get("measured"), "measured_at_commit": e.get("commit")}
        return out
    except (OSError, ValueError, KeyError):
        return None


def host_cores():
    """CPUs this process may really use: the affinity mask, capped by a cgroup v2 CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


MPI_DIR = "/opt/conda"  # MPICH (its mpicc wrapper names a compiler that is not installed: gcc + its flags)


def cpu_mpi_build():
    """-O3 -march=native build of oracle/cpu_mpi.c for this host (timing only; -ffp-contract=off
    kept: the arithmetic of the reference's x86-64 build).  Falls back to the in-tree -O2 build."""
    here = os.path.dirname(os.path.abspath(__file__))
    out = os.path.join(tempfile.mkdtemp(prefix="mcx_cpu_mpi_"), "macroc_cpu_mpi")
    cmd = ["gcc", "-O3", "-march=native", "-ffp-contract=off", "-std=gnu11", "-o", out,
           os.path.join(here, "oracle", "cpu_mpi.c"), os.path.join(here, "oracle", "oracle.c"), "-lm",
           f"-I{MPI_DIR}/include", "-Wl,-rpath-link,/usr/lib/x86_64-linux-gnu", f"{MPI_DIR}/lib/libmpi.so",
           f"-Wl,-rpath,{MPI_DIR}/lib"]
    try:
        subprocess.run(cmd, check=True, timeout=120, capture_output=True)
        return out, "gcc -O3 -march=native -ffp-contract=off"
    except (OSError, subprocess.SubprocessError):
        exe = os.path.join(here, "oracle", "macroc_cpu_mpi")
        return (exe if os.path.exists(exe) else None), "gcc -O2 (in-tree build; the -march=native build failed)"


def cpu_baseline(G, cores, rtol, gpu_its, G_target, timeout):
    """The reference's path on the host cores the way the reference runs: oracle/cpu_mpi.c (the
    Newton step of src/main.c:61-79 with MPIAIJ storage, the inode MatMult, KSPSolve_CG + PCJacobi,
    MPI halo exchange and all-reduces) under `mpirun -np <cores>` with PETSC_DECIDE's processor
    grid, one full step to rtol on a G^3 grid: measured, not extrapolated.  The same step at the
    headline grid is estimated beside it (`extrapolated_target`): the measured per-element
    assembly time and per-(CG iteration x nonzero) solve time scaled with the GPU run's iteration
    count."""
    exe, build = cpu_mpi_build()
    mpirun = os.path.join(MPI_DIR, "bin", "mpirun")
    if not exe or not os.path.exists(mpirun):
        return {"error": "MPICH (mpirun) or the cpu_mpi build is not available"}
    cmd = [mpirun, "-np", str(cores), exe, "-da_grid_x", str(G), "-da_grid_y", str(G), "-da_grid_z", str(G),
           "-ksp_rtol", repr(rtol), "-steps", "1", "-warmup", "0"]
    t0 = time.perf_counter()
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout)
    wall = time.perf_counter() - t0
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    ph = rec["phases_s"]
    f = (G_target - 1) ** 3 / (G - 1) ** 3
    t_asm = ph["strains"] + ph["homogenize"] + ph["residual"] + ph["jacobian"] + ph["update"]
    t_target = t_asm * f + ph["solve"] * f * gpu_its / max(rec["its"], 1)
    return {
        "value": 3 * G ** 3 / rec["step_s"],
        "unit": "DOF/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"oracle/cpu_mpi.c ({build}): `mpirun -np {cores}` (MPICH, one rank per usable host core, "
                   f"processors {'x'.join(map(str, rec['procs']))}), one full Newton step at {G}^3 to rtol {rtol:g}: "
                   f"{rec['its']} CG its, measured (assembly {t_asm:.1f} s, solve {ph['solve']:.1f} s); the value is "
                   f"that grid's Newton-iter DOF/s"),
        "grid": [G, G, G],
        "measured_step_seconds": rec["step_s"],
        "cg_its": rec["its"],
        "reason": rec["reason"],
        "phases_s": ph,
        "mpirun_wall_seconds": wall,
        "extrapolated_target": {"grid": [G_target] * 3, "step_seconds": t_target,
                                "value": 3 * G_target ** 3 / t_target,
                                "how": f"assembly x (elements ratio {f:.2f}), solve x elements ratio x GPU CG its "
                                       f"{gpu_its} / {rec['its']}"},
    }


def room_for_warmup(t_step, steps, args, rank, world):
    """True when one more warmup step, the timed steps and the tail (true-residual check, CPU
    baseline) still fit the --wall budget of the invocation.  Decided by rank 0 and broadcast, so
    every rank runs the same number of warmup steps.  At 256^3 per GPU one step takes ~12 s on one
    GPU but ~25 s on 2-8 (the global grid doubles, and so do the CG iterations): there the driver's
    `--steps 20 --warmup 5` would not fit 600 s with every warmup run; the first warmup always runs."""
    ok = time.perf_counter() - T_START + (1 + steps) * t_step + args.tail <= args.wall
    if world > 1:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.broadcast(t, src=0)
        ok = bool(t[0])
    return ok


def measure(argv, rank, world, comm_id, args, steps, warmup):
    """Setup + warmup + timed steps of one configuration; returns the timings of this rank.
    Timing mode only records HIP events on the compute stream (no host waits): one event pair
    per phase and per SpMV launch of the first 256 CG iterations of each solve."""
    t_setup = time.perf_counter()
    m = M.Macroc(argv, rank=rank, nranks=world, comm_id=comm_id)
    # the ranks that really joined the communicator (ncclCommCount): n_gpus in the line is this
    comm_n, comm_r, comm_dev = m.comm_info()
    log(f"[rank {rank}] device {comm_dev}, communicator: rank {comm_r} of {comm_n}")
    if comm_n != world or comm_r != rank:
        raise SystemExit(f"rank {rank}: the communicator has {comm_n} ranks (this one {comm_r}), expected {world}")
    # a peer that stopped or a mismatched collective fails the waiting rank with its rank and the
    # operation named (communicator aborted) instead of hanging the job until the driver's timeout
    m.set_option("comm_timeout", args.comm_timeout)
    m.set_timing(True)
    info = m.info
    log(f"[rank {rank}] {' '.join(map(str, argv))}: setup {time.perf_counter() - t_setup:.1f}s, device GB "
        f"{info['device_bytes'] / 1e9:.1f}, local {info['nx']}x{info['ny']}x{info['nz']}")
    U = m.get_displacement(1)

    def step():
        m.zero_u()
        m.apply_bc_on_u(U)
        m.set_strains()
        m.homogenize()
        res = m.assembly_res()
        m.assembly_jac()
        its, rn, reason = m.solve_Ax()
        m.update_u()
        return res, its, rn, reason

    def barrier_sync():
        m.synchronize()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    t_warm = []
    for w in range(warmup):
        if w >= 1 and not room_for_warmup(max(t_warm), steps, args, rank, world):
            log(f"[rank {rank}] warmup: {warmup - w} of {warmup} skipped, {steps} timed steps would not fit "
                f"--wall {args.wall:.0f}s")
            break
        t = time.perf_counter()
        r = step()
        m.synchronize()
        t_warm.append(time.perf_counter() - t)
        log(f"[rank {rank}] warmup {w}: {t_warm[-1]:.2f}s its={r[1]}")
    barrier_sync()
    t0 = time.perf_counter()
    for s in range(steps):
        res, its, rn, reason = step()  # the solve's result readback already waited for the stream
        log(f"[rank {rank}] step {s}: its={its} reason={reason} |RES|={res:.6e} rnorm={rn:.3e}")
    barrier_sync()
    dt = time.perf_counter() - t0
    log(f"[rank {rank}] {steps} steps: {dt:.2f}s, its={its} reason={reason} |RES|={res:.6e} rnorm={rn:.3e}")
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])
    tm = m.timing()
    storage = m.get_info()
    spmv_avg_ms = tm["spmv_ms_total"] / max(tm["spmv_launches"], 1)
    spmv_bytes = tm["spmv_bytes_per_launch"]
    check = None
    if not args.no_check:
        # size-independent property: true residual of the solve, |A du - b| / |b| (collective)
        b, du = m.b(), m.du()
        r = m.spmv(du) - b
        loc = np.array([r @ r, b @ b])
        if world > 1:
            tt = torch.tensor(loc)
            dist.all_reduce(tt)
            loc = tt.numpy()
        check = {"true_rel_residual": float(np.sqrt(loc[0] / loc[1])), "ksp_reason": int(reason)}
    m.finish()
    nloc = info["ndofs_local"]
    # PETSc AIJ bytes of the same SpMV (int32 col, int64 rowptr, x once, y once): SURVEY §8(d)
    csr_bytes = info["nnz_local"] * 12 + (nloc + 1) * 8 + 2 * nloc * 8
    return {"its": its, "tm": tm, "info": info, "check": check, "spmv_avg_ms": spmv_avg_ms, "spmv_bytes": spmv_bytes,
            "exact": "-mat_vi_fma" in [str(a) for a in argv],
            "csr_bytes": csr_bytes, "storage": STORAGE_NAME[storage["storage"]], "storage_id": storage["storage"],
            "split_slots": storage["split_slots"], "split_bits": storage["split_bits"],
            "vi_values": storage["vi_values"], "vi_bits": storage["vi_bits"], "vi_blocks": storage["vi_blocks"],
            "st_listed": storage["st_listed"],
            "achieved": spmv_bytes / (spmv_avg_ms * 1e-3) / 1e9, "ms_step": dt / max(steps, 1) * 1e3,
            "warmup_s": t_warm, "comm_ranks": comm_n}


def cg_iter_roofline(r):
    """Bytes of one whole CG iteration of this rank (the SpMV's algorithmic bytes + the vector
    kernels' per iteration, mcx_timing.cg_vec_bytes_per_iter) over the measured solve time per CG
    iteration (every kernel, the reductions and the host polls included)."""
    tm, its = r["tm"], max(r["its"], 1)
    ms = tm["solve_ms"] / its
    b = tm["spmv_bytes_per_launch"] + tm["cg_vec_bytes_per_iter"]
    nown = r["info"]["ndofs_local"] // 3
    return {"bytes_per_iter": b, "bytes_per_node": b / nown, "spmv_bytes": tm["spmv_bytes_per_launch"],
            "vec_bytes": tm["cg_vec_bytes_per_iter"], "ms_per_cg_iter": ms, "achieved": b / (ms * 1e-3) / 1e9,
            "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": b / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS}


def nonlinear_leg(G, ts, dt, rtol, device, extra=()):
    """BASELINE config 5's path (G^3, the J2 Gauss-point law, non-linear Newton; tools/bench_nonlinear.py):
    time steps 0 .. ts-1 of src/main.c:49-109 in this process, default AIJ storage.  Reported beside
    the headline (config5 in the line), never the headline: per-GP tangents keep the plastic zone's
    nodes as exception nodes."""
    m = M.Macroc(["-da_grid_x", G, "-da_grid_y", G, "-da_grid_z", G, "-mat_law", "plastic", "-ksp_rtol", repr(rtol),
                  "-ts", ts, "-dt", dt, "-micro_n", 10, "-device", device, *extra])
    try:
        m.set_timing(True)
        steps, t0 = [], time.perf_counter()
        for t in range(ts):
            out = m.time_step(t)
            info = m.get_info()
            steps.append({"ts": t, "newton_its": out["newton_its"], "ksp_its": out["ksp_its"],
                          "nonlinear_gps": m.nonlinear_stats()[0], "storage": info["storage"],
                          "vi_exc_nodes": info["vi_exc_nodes"]})
        m.synchronize()
        sec = time.perf_counter() - t0
    finally:
        m.finish()
    nits = sum(s["newton_its"] for s in steps)
    mt = "sbaij" if "sbaij" in [str(e) for e in extra] else "aij"
    bc = "BC_BENDING" if "-bc_type" in [str(e) for e in extra] else "BC_CIRCLE"
    return {"workload": f"config 5 path: {G}^3 J2 law, {bc}, {ts} time steps (step 0: zero load), dt {dt}, rtol {rtol:g}",
            "mat_type": mt, "storage": {0: "aij-blocks", 1: "sbaij", 2: "aij-split", 3: "aij-vi"}[steps[-1]["storage"]],
            "newton_its": nits, "cg_its": sum(sum(s["ksp_its"]) for s in steps), "seconds": sec,
            "ms_per_newton_iter": sec / max(nits, 1) * 1e3, "dof_per_s": 3 * G ** 3 * nits / sec, "steps": steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = ranks (default: WORLD_SIZE under a launcher, else 1); N > 1 without a launcher "
                         "starts the N ranks itself (torch.distributed.run)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--grid", type=int, default=256, help="nodes per direction per GPU")
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--cpu-grid", type=int, default=128, help="grid of the CPU baseline's full MPI step (0 = skip)")
    ap.add_argument("--cpu-ranks", type=int, default=0, help="MPI ranks of the CPU baseline (0 = every usable core)")
    ap.add_argument("--cpu-timeout", type=float, default=600.0, help="seconds the CPU baseline may take")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--mat-type", default="aij", choices=list(STORAGE_ARGS), help="matrix storage of the headline")
    ap.add_argument("--variants", default=None,
                    help="other storages measured after the headline, 1 warmup + 1 step each, reported in the line's "
                         "'variants' (comma list; default aij-split on one GPU, none on several; skipped once "
                         "--budget would be exceeded)")
    ap.add_argument("--budget", type=float, default=480.0, help="wall seconds the optional variants may use up to")
    ap.add_argument("--config5", type=int, default=None,
                    help="grid of the config-5 leg (J2 law, non-linear Newton, 3 time steps) reported as 'config5' "
                         "(default 128 on one GPU, 0 = skip; within --budget)")
    ap.add_argument("--bending", type=int, default=None,
                    help="grid of the uniformly plastic leg (J2 law under -bc_type 0, BC_BENDING: the whole body "
                         "yields; default AIJ storage and SBAIJ) reported as 'bending' (default 128 on one GPU, 0 = skip)")
    ap.add_argument("--wall", type=float, default=570.0,
                    help="wall seconds the invocation must fit: warmup steps after the first are skipped when the "
                         "timed steps would not fit (reported as warmup_run); the timed steps are never cut")
    ap.add_argument("--comm-timeout", type=float, default=120.0,
                    help="seconds a rank's host wait on collective work may take before the communicator is aborted "
                         "and the run fails with the rank and the operation named")
    ap.add_argument("--tail", type=float, default=30.0, help="seconds reserved after the timed steps (check, CPU "
                                                             "baseline)")
    ap.add_argument("--dry-run", action="store_true",
                    help="bootstrap only: every rank joins the process group (gloo) and rank 0 prints the ranks that "
                         "joined; no GPU is touched (tests of the --gpus launch path on a CPU host)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:  # (launch_ranks handled the no-launcher case)
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.variants is None:
        args.variants = "aij-vi-exact,aij-split" if world == 1 and args.mat_type == "aij" else ""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            t = torch.ones(1)
            dist.all_reduce(t)
            joined = int(t[0])
            dist.destroy_process_group()
        else:
            joined = 1
        log(f"[rank {rank}] dry run: local rank {local}, {joined} ranks joined")
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": joined, "world_size": world}), flush=True)
        return
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        if torch.cuda.is_available():
            torch.cuda.set_device(local)  # torch's own synchronize() then targets this rank's GPU
    px, py, pz = rank_grid(world)
    G = args.grid
    NX, NY, NZ = G * px, G * py, G * pz
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ts", 2, "-ksp_rtol", repr(args.rtol), "-device", local]

    def new_comm_id():
        if world == 1:
            return None
        obj = [M.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return obj[0]

    r = measure(argv + STORAGE_ARGS[args.mat_type], rank, world, new_comm_id(), args, args.steps, args.warmup)
    its, tm, info, check = r["its"], r["tm"], r["info"], r["check"]
    spmv_avg_ms, spmv_bytes, achieved, ms_step = r["spmv_avg_ms"], r["spmv_bytes"], r["achieved"], r["ms_step"]
    ndofs = 3 * NX * NY * NZ
    # other storages of the same matrix, 1 warmup + 1 step each, while the budget lasts (reported
    # in the line so the headline's storage can be compared with them)
    variants = []
    per_step = max(r["warmup_s"] or [ms_step * 1e-3])
    for v in [v for v in args.variants.split(",") if v and v != args.mat_type]:
        if time.perf_counter() - T_START + 2 * 3 * per_step + 60 > args.budget:
            log(f"variant {v}: skipped (budget {args.budget:.0f}s)")
            continue
        vr = measure(argv + STORAGE_ARGS[v], rank, world, new_comm_id(), args, 1, 1)
        variants.append({
            "mat_type": v, "value": ndofs / (vr["ms_step"] * 1e-3), "ms_per_step": vr["ms_step"], "steps": 1,
            "warmup": 1, "storage": vr["storage"], "kernel": kernel_name(vr), "cg_its": vr["its"],
            "ms_per_cg_iter": vr["tm"]["solve_ms"] / max(vr["its"], 1), "spmv_avg_ms": vr["spmv_avg_ms"],
            "spmv_bytes_per_launch": vr["spmv_bytes"], "spmv_achieved_GBs": vr["achieved"],
            "spmv_frac": vr["achieved"] / PEAK_HBM_GBS, "spmv_traffic": pmc_traffic(vr["storage"], NX, NY, NZ),
            "phases_ms": {k: vr["tm"][k] for k in ("jacobian_ms", "solve_ms")}, "check": vr["check"]})
        log("variant " + json.dumps(variants[-1]))
    config5 = None
    c5 = args.config5 if args.config5 is not None else (128 if world == 1 else 0)
    if c5 > 0 and rank == 0:
        if time.perf_counter() - T_START + 60 > args.budget:
            log(f"config5 leg: skipped (budget {args.budget:.0f}s)")
        else:
            config5 = nonlinear_leg(c5, 3, 0.01, args.rtol, local)
            log("config5 " + json.dumps(config5))
    bending = None
    bg = args.bending if args.bending is not None else (128 if world == 1 else 0)
    if bg > 0 and rank == 0:
        # BC_BENDING (src/bcs.c:61-91) under the J2 law: the plastic zone grows from the clamped and
        # loaded faces (32,768 exception nodes, 1.6 %, in round 4's line); the AIJ storage stays
        # value-indexed with exception nodes below vi_exc_max, else AIJ-split; SBAIJ beside it
        bending = {}
        for mt in ("aij", "sbaij"):
            if time.perf_counter() - T_START + 60 > args.budget:
                log(f"bending leg {mt}: skipped (budget {args.budget:.0f}s)")
                continue
            bending[mt] = nonlinear_leg(bg, 3, 0.01, args.rtol, local,
                                        ["-bc_type", 0] + (["-dm_mat_type", "sbaij"] if mt == "sbaij" else []))
            log(f"bending {mt} " + json.dumps(bending[mt]))
    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_grid > 0:
            try:
                log(f"cpu_baseline: mpirun, {args.cpu_grid}^3 ...")
                cpu = cpu_baseline(args.cpu_grid, args.cpu_ranks or host_cores(), args.rtol, its, G, args.cpu_timeout)
                log("cpu_baseline " + json.dumps(cpu))
            except Exception as e:  # the baseline is reported, never the product path
                cpu = {"error": repr(e)}
        csr_ms_at_peak = r["csr_bytes"] / (PEAK_HBM_GBS * 1e9) * 1e3
        line = {
            "metric": "Newton-iter DOF/s (assembly+CG) at 256^3 grid per GPU; SpMV achieved HBM GB/s",
            "value": ndofs / (ms_step * 1e-3),
            "unit": "DOF/s",
            "n_gpus": r["comm_ranks"],
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_run": len(r["warmup_s"]),
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference defaults: lx=50 ly=1 lz=50, BC_CIRCLE, E=1e7 nu=0.25, time step 1)",
            "config": {"workload": f"MacroC Newton iteration, time step 1, CG/Jacobi rtol {args.rtol:g}",
                       "grid": [NX, NY, NZ], "grid_per_gpu": [G, G, G], "processors": [px, py, pz],
                       "dofs": ndofs, "nnz": info["nnz_global"], "parallelism": f"dmda{px}x{py}x{pz}",
                       "mat_type": "aij" if args.mat_type.startswith("aij") else "sbaij", "storage": r["storage"],
                       "split_slots": r["split_slots"], "split_bits": r["split_bits"],
                       "vi_values": r["vi_values"], "vi_bits": r["vi_bits"], "vi_blocks": r["vi_blocks"],
                       "st_listed": r["st_listed"],
                       "spmv_rows": "fused multiply-add (-mat_vi_fma 1)" if r["storage_id"] == 3 and not r["exact"]
                       else "multiply, add (MatMult inode order)"},
            "cg_its": its,
            "ms_per_cg_iter": tm["solve_ms"] / max(its, 1),
            # CG iterations grow ~linearly with the global grid edge (720 at 64^3, 2814 at 256^3),
            # so Newton-iter DOF/s cannot weak-scale; DOF x CG iterations / solve second can
            "dof_cg_iters_per_s": ndofs * its / (tm["solve_ms"] * 1e-3),
            "phases_ms": {k: tm[k] for k in ("strains_ms", "homogenize_ms", "residual_ms", "jacobian_ms",
                                             "solve_ms", "update_ms")},
            "device_gb": info["device_bytes"] / 1e9,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": pmc_traffic(r["storage"], NX, NY, NZ),
                         "traffic_source": "profiles/pmc_spmv.json (committed PMC passes, tools/pmc_spmv.sh)",
                         "traffic_measured_at_commit": pmc_commit(r["storage"], NX, NY, NZ),
                         "kernel": kernel_name(r), "bytes_per_launch": spmv_bytes,
                         "avg_launch_ms": spmv_avg_ms, "launches_timed": tm["spmv_launches"],
                         # what the reference's MatMult must stream for the same product (PETSc AIJ
                         # bytes), the time that takes at the 8 TB/s peak, and how many times faster
                         # this launch is than that bound (not a roofline fraction: it moves fewer bytes)
                         "csr_bytes_per_launch": r["csr_bytes"], "csr_ms_at_peak": csr_ms_at_peak,
                         "speedup_vs_csr_at_peak": csr_ms_at_peak / spmv_avg_ms,
                         "limiter": lds_limiter(r["storage"], NX, NY, NZ),
                         # the whole CG iteration: SpMV bytes + the vector kernels'
                         # (update, p update, amortised x update) per iteration over the measured
                         # solve time per iteration (reductions and the host polls included)
                         "cg_iter": cg_iter_roofline(r)},
            "cpu_baseline": cpu,
            "check": check,
            "variants": variants,
            "config5": config5,
            "bending": bending,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
