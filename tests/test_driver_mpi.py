"""The MPI build of the C host driver (make driver-mpi) under `mpirun -np N`, as the reference
runs (`mpirun -np N macroc ...`, tests/CMakeLists.txt:21-32): in -plan_only mode (no GPU) every
rank prints its DMDA corners, DOF offset, owned nonzeros and forward-halo plan, which must equal
the oracle's decomposition of the same -da_grid_* / -da_processors_* and be pairwise symmetric."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "macroc_amd", "driver", "macroc_amd_mpi")
MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"

pytestmark = pytest.mark.skipif(not (os.path.exists(EXE) and os.path.exists(MPIRUN)),
                                reason="MPI driver or mpirun not built/available")


def plan(nranks, grid, procs=None, tmp="."):
    cmd = [MPIRUN, "-np", str(nranks), EXE, "-plan_only", "-da_grid_x", str(grid[0]), "-da_grid_y", str(grid[1]),
           "-da_grid_z", str(grid[2])]
    if procs:
        cmd += ["-da_processors_x", str(procs[0]), "-da_processors_y", str(procs[1]), "-da_processors_z", str(procs[2])]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=tmp)
    assert r.returncode == 0, r.stderr
    rows = {}
    for ln in r.stdout.splitlines():
        m = re.match(r"PLAN rank (\d+) of (\d+) grid (\d+) (\d+) (\d+) corners ((?:\d+ ){6})dof_offset (\d+) ndofs (\d+) "
                     r"nnz (\d+) nelem (\d+) halo (\d+)(.*)", ln)
        assert m, ln
        rk = int(m.group(1))
        halo = {int(a): (int(b), int(c)) for a, b, c in re.findall(r" (\d+):(\d+):(\d+)", m.group(12))}
        assert len(halo) == int(m.group(11))
        rows[rk] = dict(size=int(m.group(2)), grid=tuple(int(m.group(i)) for i in (3, 4, 5)),
                        corners=tuple(int(v) for v in m.group(6).split()), off=int(m.group(7)),
                        ndofs=int(m.group(8)), nnz=int(m.group(9)), nelem=int(m.group(10)), halo=halo)
    assert sorted(rows) == list(range(nranks))
    return rows


@pytest.mark.parametrize("nranks,grid,procs", [(2, (5, 2, 2), None), (3, (5, 2, 2), None), (4, (9, 7, 6), (2, 2, 1)),
                                               (8, (5, 3, 4), None), (8, (10, 8, 8), (2, 2, 2))])
def test_mpi_plan_matches_oracle(nranks, grid, procs, tmp_path):
    rows = plan(nranks, grid, procs, tmp_path)
    m, n, p = procs or (0, 0, 0)
    P = O.Problem(*grid, nranks=nranks, m=m, n=n, p=p)
    rp, _ = P.csr()
    for r, row in rows.items():
        assert row["size"] == nranks and row["grid"] == P.decomp()
        assert row["corners"] == P.corners(r)[:6]
        assert row["off"] == P.dof_offset(r)
        assert row["ndofs"] == 3 * np.prod(row["corners"][3:])
        assert row["nnz"] == rp[row["off"] + row["ndofs"]] - rp[row["off"]]
        assert row["nelem"] == len(P.elements(r))
        for q, (send, recv) in row["halo"].items():
            assert rows[q]["halo"][r] == (recv, send)  # what r sends q is what q receives from r
    P.close()


def test_single_rank_build_refuses_a_rank_grid(tmp_path):
    exe = os.path.join(ROOT, "macroc_amd", "driver", "macroc_amd")
    r = subprocess.run([exe, "-da_grid_x", "5", "-da_grid_y", "2", "-da_grid_z", "2", "-da_processors_x", "2"],
                       capture_output=True, text=True, timeout=60, cwd=tmp_path)
    assert r.returncode != 0 and "driver-mpi" in r.stderr


@pytest.mark.gpu
def test_mpi_driver_one_rank_on_gpu(tmp_path):
    """The MPI build under `mpirun -np 1` on the GPU runs BASELINE config 1 (4x4x2, -ts 2) and
    prints the same |RES| / KSP lines as the single-rank build, and the same info.dat."""
    flags = ["-da_grid_x", "4", "-da_grid_y", "4", "-da_grid_z", "2", "-ts", "2"]
    single = os.path.join(ROOT, "macroc_amd", "driver", "macroc_amd")
    out = {}
    for name, cmd in (("mpi", [MPIRUN, "-np", "1", EXE, *flags]), ("single", [single, *flags])):
        d = tmp_path / name
        d.mkdir()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=d)
        assert r.returncode == 0, r.stderr
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith(("|RES|", "KSP", "Time Step", "Non-Linear"))]
        out[name] = (lines, (d / "info.dat").read_text())
    assert out["mpi"] == out["single"] and any(ln.startswith("KSP") for ln in out["mpi"][0])
