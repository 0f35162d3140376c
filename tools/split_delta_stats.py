"""How exact the AIJ-split lower corrections are in bf16: for an oracle J2 state (time step 1 after
one solved Newton iteration, BC_BENDING = bc 0 or the load circle = bc 1), every lower entry's
delta d = A(r, c) - A(c, r) and the significant bits it needs.  Diagnosis tool (CPU, oracle only).

    python tools/split_delta_stats.py N BC
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402

N, bc = int(sys.argv[1]), int(sys.argv[2])
P = O.Problem(N, N, N, rtol=1e-10, law=1, dt=0.05 if bc == 0 else 0.01, bc_type=bc)
P.apply_bc_u(P.get_displacement(1))
P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac(); P.solve(); P.update_u()
P.set_strains(); P.homogenize(); P.assembly_jac()
print("plastic Gauss points", P.nonlinear_gps()[0], "of", P.ngp)
rp, ci = P.csr()
v = P.A_values()
n = len(rp) - 1
rows = np.repeat(np.arange(n), np.diff(rp))
A = sp.csr_matrix((v, ci, rp), shape=(n, n))
lo = ci < rows
d = v[lo] - np.asarray(A.T.tocsr()[rows[lo], ci[lo]]).ravel()
b = d.astype(np.float32).view(np.uint32)
hi = (b & 0xffff0000).view(np.float32).astype(np.float64)  # the truncated bf16 the split stores
print("lower entries", lo.sum(), "non-zero deltas", (d != 0).sum(), "bf16-exact", (hi == d).sum(),
      "f32-exact", (d.astype(np.float32).astype(np.float64) == d).sum())
bits = []
for x in d[d != 0][:200000]:
    m, k = np.frexp(x)[0], 0
    while m != 0 and k < 60:
        m *= 2
        m -= np.trunc(m)
        k += 1
    bits.append(k)
print("significant bits (histogram from 0):", np.bincount(np.minimum(np.array(bits, dtype=int), 40)).tolist())
