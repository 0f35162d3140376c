import sys; sys.path.insert(0,'.')
import numpy as np, macroc_amd as M
from oracle import oracle as O
NX,NY,NZ,dt,rtol=12,10,12,0.01,1e-12
P=O.Problem(NX,NY,NZ,law=1,dt=dt,rtol=rtol)
m=M.Macroc(["-da_grid_x",NX,"-da_grid_y",NY,"-da_grid_z",NZ,"-dt",dt,"-ksp_rtol",repr(rtol),"-mat_law","plastic"])
for ts in (0,1):
    m.apply_bc_on_u(m.get_displacement(ts)); P.apply_bc_u(P.get_displacement(ts))
print("U", m.get_displacement(1), P.get_displacement(1), "u eq", np.array_equal(m.u(),P.u()))
m.set_strains(); m.homogenize(); n=m.assembly_res(); P.set_strains(); P.homogenize(); P.assembly_res()
print("strain eq", np.array_equal(m.strain(),P.strain()), "stress maxdiff", np.abs(m.stress()-P.stress()).max(), np.abs(P.stress()).max())
print("b maxdiff", np.abs(m.b()-P.b()).max(), np.abs(P.b()).max(), "nl", m.nonlinear_stats(), P.nonlinear_gps())
m.assembly_jac(); P.assembly_jac()
v=m.dump_csr()[2]; a=P.A_values(); d=np.abs(v-a); i=d.argmax()
print("A maxdiff", d.max(), "at", i, v[i], a[i], "maxA", np.abs(a).max(), "n mismatched", (d>1e-6*np.abs(a).max()).sum(), len(a))
its=m.solve_Ax(); o=P.solve(history=True)
du=m.du(); dr=P.du()
print("solve gpu", its, "oracle", o["its"], o["reason"], "rel du diff", np.linalg.norm(du-dr)/np.linalg.norm(dr))
x=np.random.default_rng(1).uniform(-1,1,m.n); print("spmv eq", np.array_equal(m.spmv(x), P.spmv(x)))
print("hist oracle", o["history"][:5])
