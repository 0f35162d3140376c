"""Host sanitizer run (SURVEY.md §5 "race detection / sanitizers"; the reference forces a Debug
build for its tests, tests/CMakeLists.txt:2): `make asan` builds every library source with
AddressSanitizer + UndefinedBehaviorSanitizer on the host side (device code unchanged) into the
C driver, and the oracle's CLI under the same sanitizers.  No GPU is needed: the driver's
-plan_only runs the DMDA decomposition and forward-halo planner (mcx_plan / mcx_plan_halo) of
every rank on 1-8 rank grids, and must print exactly what the product build prints; the oracle
runs the reference's time loop (src/main.c:49-109) on BASELINE config 1 and a 3-rank grid.
Any sanitizer report aborts the process (-fno-sanitize-recover=all) and fails the test."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "build", "asan")
DRIVER = os.path.join(ASAN, "macroc_amd_asan")
ORACLE = os.path.join(ASAN, "macroc_oracle_asan")
PLAIN = os.path.join(ROOT, "macroc_amd", "driver", "macroc_amd")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")

pytestmark = pytest.mark.skipif(not (os.path.exists(DRIVER) and os.path.exists(ORACLE)),
                                reason="sanitizer build missing (make asan)")


def run(cmd, tmp):
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True, timeout=300, cwd=tmp, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    return r.stdout


@pytest.mark.parametrize("grid,procs", [((4, 4, 2), (1, 1, 1)), ((5, 2, 2), (2, 1, 1)), ((9, 7, 6), (3, 1, 1)),
                                        ((9, 7, 6), (2, 2, 1)), ((10, 8, 8), (2, 2, 2)), ((17, 9, 5), (3, 2, 1)),
                                        ((12, 10, 14), (1, 2, 4)), ((64, 6, 5), (4, 1, 2))])
def test_plan_only_under_asan(grid, procs, tmp_path):
    args = ["-plan_only", "-da_grid_x", grid[0], "-da_grid_y", grid[1], "-da_grid_z", grid[2],
            "-da_processors_x", procs[0], "-da_processors_y", procs[1], "-da_processors_z", procs[2]]
    out = run([DRIVER] + args, tmp_path)
    lines = [ln for ln in out.splitlines() if ln.startswith("PLAN ")]
    assert len(lines) == procs[0] * procs[1] * procs[2]
    if os.path.exists(PLAIN):
        assert lines == [ln for ln in run([PLAIN] + args, tmp_path).splitlines() if ln.startswith("PLAN ")]


@pytest.mark.parametrize("args", [["-da_grid_x", 4, "-da_grid_y", 4, "-da_grid_z", 2, "-ts", 2],
                                  ["-da_grid_x", 6, "-da_grid_y", 5, "-da_grid_z", 4, "-ts", 3, "-nranks", 3],
                                  ["-da_grid_x", 6, "-da_grid_y", 4, "-da_grid_z", 5, "-ts", 2, "-bc_type", 0,
                                   "-mat_law", 1, "-dt", 0.05]])
def test_oracle_under_asan(args, tmp_path):
    out = run([ORACLE] + args, tmp_path)
    assert "newton_solve_iter_s" in out
