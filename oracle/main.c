/* macroc_oracle — CLI of the CPU restatement (TEST INFRASTRUCTURE / CPU baseline only).
 * Accepts the reference's flag names (src/init.c:66-83, DMSetFromOptions -da_*,
 * KSPSetFromOptions -ksp_*) and runs src/main.c:49-109. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

int main(int argc, char** argv) {
  orc_opts o;
  orc_default_opts(&o);
  const char* log = NULL;
  const char* info = NULL;
  const char* gauss = NULL;
  for (int a = 1; a < argc; a++) {
    const char* k = argv[a];
    const char* v = a + 1 < argc ? argv[a + 1] : "0";
#define I64(name, field) if (!strcmp(k, name)) { o.field = atoll(v); a++; continue; }
#define INT(name, field) if (!strcmp(k, name)) { o.field = atoi(v); a++; continue; }
#define DBL(name, field) if (!strcmp(k, name)) { o.field = atof(v); a++; continue; }
    I64("-da_grid_x", NX) I64("-da_grid_y", NY) I64("-da_grid_z", NZ)
    INT("-da_processors_x", m) INT("-da_processors_y", n) INT("-da_processors_z", p)
    INT("-nranks", nranks) DBL("-lx", lx) DBL("-ly", ly) DBL("-lz", lz) DBL("-dt", dt)
    INT("-ts", ts) INT("-bc_type", bc_type) INT("-newton_max_its", newton_max_its)
    DBL("-newton_min_tol", newton_min_tol) DBL("-newton_rel_tol", newton_rel_tol)
    DBL("-ksp_rtol", rtol) DBL("-ksp_atol", abstol) DBL("-ksp_divtol", dtol) INT("-ksp_max_it", maxits)
    if (!strcmp(k, "-log")) { log = v; a++; continue; }
    if (!strcmp(k, "-info")) { info = v; a++; continue; }
    if (!strcmp(k, "-gauss")) { gauss = v; a++; continue; }
    INT("-mat_law", law)
    fprintf(stderr, "warning: unknown option %s ignored\n", k);
  }
  orc_problem* P = orc_create(&o);
  if (!P) { fprintf(stderr, "bad options / partition\n"); return 1; }
  double t = 0;
  orc_run_files(P, log, info, gauss, &t);
  printf("newton_solve_iter_s %.6f ndofs %lld\n", t, (long long)orc_ndofs(P));
  orc_destroy(P);
  return 0;
}
