"""The RCCL transport between GPUs: one fresh process per GPU (started before anything touched
a GPU, as `mpirun -np N macroc` starts them, tests/CMakeLists.txt:21-32), a communicator built
from rank 0's id, grouped ncclSend/ncclRecv halos on the comm stream and ncclAllReduce of the CG
scalars.  For each option set (halo overlapped with the interior p update or serialised, the
Jacobi scaling from the diagonal-block index or the dinv/z vectors) du must be bitwise the same
and the iteration count equal, and du must match the one-rank oracle within the north-star bar.

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so this needs >= 2 GPUs; on a
one-GPU box it is skipped and the decomposed path is covered by the in-process transport
(tests/test_gpu_multirank.py), whose only difference is the two calls that move the bytes."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import macroc_amd as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def gpus():
    try:
        import torch  # device_count() does not initialise the GPU on this image

        return torch.cuda.device_count()
    except Exception:
        return 0


def run_ranks(nranks, argv, opts, tmp):
    cid = M.comm_unique_id().hex()  # host-side only (no GPU call)
    procs, outs = [], []
    for r in range(nranks):
        out = os.path.join(tmp, f"rank{r}.npz")
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "rccl_worker.py"), str(r), str(nranks), cid,
                                       out, json.dumps(opts)] + [str(a) for a in argv]))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0] * nranks, rcs
    return [np.load(o) for o in outs]


@pytest.mark.skipif(gpus() < 2, reason="RCCL needs one GPU per rank (>= 2 GPUs)")
@pytest.mark.parametrize("procs", [(2, 1, 1), (2, 2, 2)])
def test_rccl_halo_and_allreduce(procs, tmp_path):
    nr = procs[0] * procs[1] * procs[2]
    if gpus() < nr:
        pytest.skip(f"needs {nr} GPUs")
    NX, NY, NZ, rtol = 24, 14, 12, 1e-12
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", procs[0],
            "-da_processors_y", procs[1], "-da_processors_z", procs[2], "-ksp_rtol", repr(rtol)]
    ref = O.Problem(NX, NY, NZ, rtol=rtol)
    ref.newton_step1()
    results = []
    for opts in ([["halo_overlap", 1], ["cg_dix", 1]], [["halo_overlap", 0], ["cg_dix", 1]],
                 [["halo_overlap", 1], ["cg_dix", 0]]):
        outs = run_ranks(nr, argv, opts, str(tmp_path))
        du = np.zeros(ref.ndofs)
        for o in outs:
            du[o["nat"]] = o["du"]
            assert int(o["its"]) == int(outs[0]["its"]) and int(o["reason"]) == 2
        results.append((int(outs[0]["its"]), du))
    for its, du in results[1:]:
        assert its == results[0][0] and np.array_equal(du, results[0][1])
    assert np.linalg.norm(results[0][1] - ref.du()) <= 1e-10 * np.linalg.norm(ref.du())


def test_rccl_worker_one_rank(tmp_path):
    """The same fresh-process worker as a one-rank RCCL communicator (runs on one GPU): every
    reduction takes the communicator path; du matches the oracle within the north-star bar."""
    NX, NY, NZ, rtol = 24, 14, 12, 1e-12
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-ksp_rtol", repr(rtol)]
    ref = O.Problem(NX, NY, NZ, rtol=rtol)
    ref.newton_step1()
    (o,) = run_ranks(1, argv, [["halo_overlap", 1]], str(tmp_path))
    du = np.zeros(ref.ndofs)
    du[o["nat"]] = o["du"]
    assert int(o["reason"]) == 2
    assert np.linalg.norm(du - ref.du()) <= 1e-10 * np.linalg.norm(ref.du())
