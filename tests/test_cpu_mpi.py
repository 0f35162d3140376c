"""The CPU baseline under MPI (oracle/cpu_mpi.c: the reference's Newton step on host cores,
`mpirun -np N` as tests/CMakeLists.txt:21-32 launches the reference) against the oracle on the
same rank grid: |RES|, CG iterations and du.  Test infrastructure for bench.py's cpu_baseline;
no GPU."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "macroc_cpu_mpi")
MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "macroc_cpu_mpi"], check=True,
                   capture_output=True, timeout=300)
    return os.path.exists(EXE) and os.path.exists(MPIRUN)


pytestmark = pytest.mark.skipif(not _build(), reason="MPICH or mpirun not available")


def run(np_, args, tmp_path):
    dump = str(tmp_path / f"du_{np_}.bin")
    out = subprocess.run([MPIRUN, "-np", str(np_), EXE, *map(str, args), "-dump", dump], check=True,
                         capture_output=True, text=True, timeout=300)
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    return rec, np.fromfile(dump, dtype=np.float64)


@pytest.mark.parametrize("grid,np_,procs,rtol", [((10, 8, 8), 1, (0, 0, 0), 1e-12), ((10, 8, 8), 2, (2, 1, 1), 1e-12),
                                                 ((9, 7, 8), 4, (0, 0, 0), 1e-12), ((8, 8, 8), 8, (2, 2, 2), 1e-12),
                                                 ((16, 16, 16), 3, (0, 0, 0), 1e-8)])
def test_cpu_mpi_vs_oracle(grid, np_, procs, rtol, tmp_path):
    NX, NY, NZ = grid
    m, n, p = procs
    args = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-ksp_rtol", repr(rtol)]
    if m:
        args += ["-da_processors_x", m, "-da_processors_y", n, "-da_processors_z", p]
    rec, du = run(np_, args, tmp_path)
    P = O.Problem(NX, NY, NZ, nranks=np_, m=m, n=n, p=p, rtol=rtol)
    assert tuple(rec["procs"]) == P.decomp() and rec["nnz"] == P.nnz
    out = P.newton_step1()
    assert abs(rec["res"] - out["res"]) <= 1e-12 * out["res"]
    assert rec["reason"] == out["reason"] and abs(rec["its"] - out["its"]) <= 1
    ref = P.du()  # PETSc order of this rank grid = the ranks' owned parts in rank order
    tol = 1e-10 if rtol <= 1e-12 else 50 * rtol
    assert np.linalg.norm(du - ref) <= tol * np.linalg.norm(ref)
    P.close()
