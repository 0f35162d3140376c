// vtu.cpp — ParaView output of the MI355X MacroC path: write_pvtu (src/output.c:25-267).
//
// Same files as the reference: "<prefix>.pvtu" naming one "<prefix>-subdo-<rank>.vtu" piece per
// rank, each piece holding the rank's DMDA ghosted box as points, its own elements (as
// DMDAGetElements lists them) as hexahedra, the ghosted displacement, and per-cell data.  The
// cell data are computed on the device (k_vtu_cells: wg-weighted Gauss-point sums of the strain
// recomputed from u and of the stress, non-linear GP counts); this file only formats text.
// "cost" is MicroPP's micro-solver cost (micropp_C_get_sigma_cost3, :180-187): the device
// Gauss-point laws have no micro solve, so it is 0, as in the oracle.
#include <cstdio>
#include <string>
#include <vector>

#include "mcx_internal.h"

namespace mcx {

static int write_pvtu_index(const char* prefix, int nranks) {
  const std::string name = std::string(prefix) + ".pvtu";
  FILE* fp = std::fopen(name.c_str(), "w");
  if (!fp) {
    set_error("cannot open " + name);
    return 40;
  }
  std::fprintf(fp,
               "<?xml version=\"1.0\"?>\n"
               "<VTKFile type=\"PUnstructuredGrid\" version=\"0.1\" "
               "byte_order=\"LittleEndian\">\n"
               "<PUnstructuredGrid GhostLevel=\"0\">\n"
               "<PPoints>\n"
               "  <PDataArray type=\"Float64\" Name=\"Position\"   NumberOfComponents=\"3\"/>\n"
               "</PPoints>\n"
               "<PCells>\n"
               "  <PDataArray type=\"Int32\" Name=\"connectivity\" NumberOfComponents=\"1\"/>\n"
               "  <PDataArray type=\"Int32\" Name=\"offsets\"      NumberOfComponents=\"1\"/>\n"
               "  <PDataArray type=\"UInt8\" Name=\"types\"        NumberOfComponents=\"1\"/>\n"
               "</PCells>\n"
               "<PPointData Vectors=\"displ\">\n"
               "  <PDataArray type=\"Float64\" Name=\"displ\"      NumberOfComponents=\"3\" />\n"
               "</PPointData>\n"
               "<PCellData>\n"
               "  <PDataArray type=\"Int32\"   Name=\"part\"       NumberOfComponents=\"1\"/>\n"
               "  <PDataArray type=\"Float64\" Name=\"cost\"       NumberOfComponents=\"1\"/>\n"
               "  <PDataArray type=\"Int32\"   Name=\"non-linear\" NumberOfComponents=\"1\"/>\n"
               "<PDataArray type=\"Float64\" Name=\"strain\"       NumberOfComponents=\"6\"/>\n"
               "<PDataArray type=\"Float64\" Name=\"stress\"       NumberOfComponents=\"6\"/>\n"
               "</PCellData>\n");
  for (int r = 0; r < nranks; ++r) std::fprintf(fp, "  <Piece Source=\"%s-subdo-%d.vtu\"/>\n", prefix, r);
  std::fprintf(fp,
               "</PUnstructuredGrid>\n"
               "</VTKFile>\n");
  std::fclose(fp);
  return 0;
}

int write_vtu(Ctx& c, const char* prefix) {
  const Geo& g = c.g;
  int rc = halo_exchange(c, c.u_pad);  // DMGlobalToLocal of u (src/output.c:152-154)
  if (rc) return rc;
  // the rank's elements (DMDAGetElements) and ghosted box (DMDAGetGhostCorners)
  const int s[3] = {g.xs, g.ys, g.zs}, w[3] = {g.nx, g.ny, g.nz}, N[3] = {g.NX, g.NY, g.NZ};
  int lo[3], cnt[3], gs[3], gw[3];
  for (int d = 0; d < 3; d++) {
    lo[d] = s[d] > 0 ? s[d] - 1 : s[d];
    cnt[d] = std::max(0, s[d] + w[d] - 1 - lo[d]);
    gs[d] = lo[d];
    gw[d] = (s[d] + w[d] < N[d] ? s[d] + w[d] + 1 : N[d]) - gs[d];
  }
  const int64_t nelem = (int64_t)cnt[0] * cnt[1] * cnt[2];
  const int64_t npts = (int64_t)gw[0] * gw[1] * gw[2];
  std::vector<double> cells(13 * nelem), upad((size_t)3 * g.PX * g.PY * g.PZ);
  double* d_cells = nullptr;
  if (nelem > 0) {
    MCX_HIP(hipMalloc(&d_cells, sizeof(double) * cells.size()));
    launch_vtu_cells(c, lo, cnt, d_cells);
    MCX_HIP(hipMemcpyAsync(cells.data(), d_cells, sizeof(double) * cells.size(), hipMemcpyDeviceToHost, c.stream));
  }
  MCX_HIP(hipMemcpyAsync(upad.data(), c.u_pad, sizeof(double) * upad.size(), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  if (d_cells) MCX_HIP(hipFree(d_cells));

  if (c.rank == 0 && (rc = write_pvtu_index(prefix, c.nranks))) return rc;
  const std::string name = std::string(prefix) + "-subdo-" + std::to_string(c.rank) + ".vtu";
  FILE* fp = std::fopen(name.c_str(), "w");
  if (!fp) {
    set_error("cannot open " + name);
    return 40;
  }
  std::fprintf(fp,
               "<?xml version=\"1.0\"?>\n"
               "<VTKFile type=\"UnstructuredGrid\" version=\"0.1\" "
               "byte_order=\"LittleEndian\">\n"
               "<UnstructuredGrid>\n"
               "<Piece NumberOfPoints=\"%d\" NumberOfCells=\"%d\">\n"
               "<Points>\n",
               (int)npts, (int)nelem);
  std::fprintf(fp,
               "<DataArray type=\"Float64\" "
               "Name=\"Position\" NumberOfComponents=\"3\" "
               "format=\"ascii\">\n");
  for (int k = gs[2]; k < gs[2] + gw[2]; ++k)
    for (int j = gs[1]; j < gs[1] + gw[1]; ++j)
      for (int i = gs[0]; i < gs[0] + gw[0]; ++i) std::fprintf(fp, "%01.6e\t%01.6e\t%01.6e\n", i * g.dx, j * c.dy, k * g.dz);
  std::fprintf(fp,
               "</DataArray>\n"
               "</Points>\n"
               "<Cells>\n");
  std::fprintf(fp,
               "<DataArray type=\"Int32\" Name=\"connectivity\" "
               "NumberOfComponents=\"1\" format=\"ascii\">\n");
  // Q1 node order of DMDAGetElements (---, +--, ++-, -+-, --+, +-+, +++, -++), ghosted-local ids
  static const int q1[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};
  for (int64_t e = 0; e < nelem; ++e) {
    const int ex = lo[0] + (int)(e % cnt[0]), ey = lo[1] + (int)((e / cnt[0]) % cnt[1]),
              ez = lo[2] + (int)(e / ((int64_t)cnt[0] * cnt[1]));
    for (int n = 0; n < 8; ++n) {
      const int id = (ex + q1[n][0] - gs[0]) + (ey + q1[n][1] - gs[1]) * gw[0] + (ez + q1[n][2] - gs[2]) * gw[0] * gw[1];
      std::fprintf(fp, "%-6d\t", id);
    }
    std::fprintf(fp, "\n");
  }
  std::fprintf(fp, "</DataArray>\n");
  std::fprintf(fp,
               "<DataArray type=\"Int32\" Name=\"offsets\" "
               "NumberOfComponents=\"1\" format=\"ascii\">\n");
  for (int64_t e = 1; e < nelem + 1; ++e) std::fprintf(fp, "%d\t", (int)(e * 8));
  std::fprintf(fp, "\n</DataArray>\n");
  std::fprintf(fp,
               "<DataArray type=\"UInt8\"  Name=\"types\" "
               "NumberOfComponents=\"1\" format=\"ascii\">\n");
  for (int64_t e = 0; e < nelem; ++e) std::fprintf(fp, "12\t");
  std::fprintf(fp, "\n</DataArray>\n");
  std::fprintf(fp, "</Cells>\n");
  std::fprintf(fp, "<PointData Vectors=\"displ\">\n");
  std::fprintf(fp,
               "<DataArray type=\"Float64\" Name=\"displ\" "
               "NumberOfComponents=\"3\" format=\"ascii\" >\n");
  for (int k = gs[2]; k < gs[2] + gw[2]; ++k)
    for (int j = gs[1]; j < gs[1] + gw[1]; ++j)
      for (int i = gs[0]; i < gs[0] + gw[0]; ++i) {
        const int64_t p = (i - g.xs + 1) + (int64_t)(j - g.ys + 1) * g.PX + (int64_t)(k - g.zs + 1) * g.PX * g.PY;
        std::fprintf(fp, "%01.6e\t%01.6e\t%01.6e\n", upad[3 * p], upad[3 * p + 1], upad[3 * p + 2]);
      }
  std::fprintf(fp, "</DataArray>\n");
  std::fprintf(fp, "</PointData>\n");
  std::fprintf(fp, "<CellData>\n");
  std::fprintf(fp,
               "<DataArray type=\"Int32\" Name=\"part\" "
               "NumberOfComponents=\"1\" format=\"ascii\">\n");
  for (int64_t e = 0; e < nelem; ++e) std::fprintf(fp, "%d\t", c.rank);
  std::fprintf(fp, "\n</DataArray>\n");
  std::fprintf(fp,
               "<DataArray type=\"Float64\" Name=\"cost\" "
               "NumberOfComponents=\"1\" format=\"ascii\">\n");
  for (int64_t e = 0; e < nelem; ++e) std::fprintf(fp, "%lf\t", 0. / 8);
  std::fprintf(fp, "\n</DataArray>\n");
  std::fprintf(fp,
               "<DataArray type=\"Int32\" Name=\"non-linear\" "
               "NumberOfComponents=\"1\" format=\"ascii\">\n");
  for (int64_t e = 0; e < nelem; ++e) std::fprintf(fp, "%d\t", (int)cells[13 * e + 12]);
  std::fprintf(fp, "\n</DataArray>\n");
  std::fprintf(fp,
               "<DataArray type=\"Float64\" Name=\"strain\" "
               "NumberOfComponents=\"6\" format=\"ascii\">");
  for (int64_t e = 0; e < nelem; ++e)
    for (int i = 0; i < 6; ++i) std::fprintf(fp, "%e\t", cells[13 * e + i]);
  std::fprintf(fp, "\n</DataArray>\n");
  std::fprintf(fp,
               "<DataArray type=\"Float64\" Name=\"stress\" "
               "NumberOfComponents=\"6\" format=\"ascii\">");
  for (int64_t e = 0; e < nelem; ++e)
    for (int i = 0; i < 6; ++i) std::fprintf(fp, "%e\t", cells[13 * e + 6 + i]);
  std::fprintf(fp, "\n</DataArray>\n");
  std::fprintf(fp, "</CellData>\n");
  std::fprintf(fp,
               "</Piece>\n"
               "</UnstructuredGrid>\n"
               "</VTKFile>\n");
  std::fclose(fp);
  return 0;
}

}  // namespace mcx

extern "C" int mcx_write_vtu(void* ctx, const char* file_prefix) try {
  MCX_ENTRY();
  using namespace mcx;
  if (!ctx || !file_prefix) {
    set_error("mcx_write_vtu: null argument");
    return 1;
  }
  Ctx& c = *reinterpret_cast<Ctx*>(ctx);
  MCX_HIP(hipSetDevice(c.device));
  return write_vtu(c, file_prefix);
} MCX_CATCH
