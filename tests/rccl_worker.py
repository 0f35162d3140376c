"""One rank of tests/test_gpu_rccl.py: a fresh process (nothing touched the GPU before it) that
joins an RCCL communicator on its own GPU and runs time step 1's Newton iteration of a
decomposed grid, writing its owned du in natural order and the KSP result to an .npz file.

    python tests/rccl_worker.py RANK NRANKS ID_HEX OUT.npz OPTS_JSON ARG..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import macroc_amd as M  # noqa: E402


def main():
    rank, nranks, cid, out, opts = int(sys.argv[1]), int(sys.argv[2]), bytes.fromhex(sys.argv[3]), sys.argv[4], \
        json.loads(sys.argv[5])
    argv = sys.argv[6:] + ["-device", str(rank)]
    with M.Macroc(argv, rank=rank, nranks=nranks, comm_id=cid) as m:
        for k, v in opts:
            m.set_option(k, v)
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains()
        m.homogenize()
        res = m.assembly_res()
        m.assembly_jac()
        its, rn, reason = m.solve_Ax()
        _, nat = m.owned_dofs()
        np.savez(out, du=m.du(), nat=nat, its=its, reason=reason, res=res)


if __name__ == "__main__":
    main()
