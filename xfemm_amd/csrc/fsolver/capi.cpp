// extern "C" surface of FSolver (include/xfemm_fsolver.h).
#include "../../../include/xfemm_fsolver.h"

#include <algorithm>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>

#include "fsolver.h"

struct xfemm_fsolver {
    xfemm::FSolver s;
};

// No C++ exception crosses the C-ABI: a host allocation failure (or any
// other exception) of a step becomes its false return, with the reason in
// last_error.
template <class F>
int guarded(xfemm_fsolver *h, F &&f)
{
    if (!h) return 0;
    try {
        return f() ? 1 : 0;
    } catch (const std::bad_alloc &) {
        h->s.join_removals();
        h->s.lastError = "out of host memory\n";
    } catch (const std::exception &e) {
        h->s.join_removals();
        h->s.lastError = std::string(e.what()) + "\n";
    }
    h->s.WarnMessage("%s", h->s.lastError.c_str());
    return 0;
}

extern "C" {

xfemm_fsolver *xfemm_fsolver_create(void) { return new xfemm_fsolver(); }

void xfemm_fsolver_destroy(xfemm_fsolver *h) { delete h; }

void xfemm_fsolver_set_message_handlers(xfemm_fsolver *h, xfemm_message_fn warn, xfemm_message_fn print)
{
    if (!h) return;
    if (warn) h->s.WarnMessage = warn;
    if (print) h->s.PrintMessage = print;
}

int xfemm_fsolver_set_pathname(xfemm_fsolver *h, const char *path)
{
    if (!h || !path) return 0;
    std::string p(path);
    if (p.size() > 4 && p.compare(p.size() - 4, 4, ".fem") == 0) p.resize(p.size() - 4);
    h->s.PathName = p;
    return 1;
}

int xfemm_fsolver_set_device(xfemm_fsolver *h, int device)
{
    if (!h || device < 0) return 0;
    h->s.device = device;
    return 1;
}

int xfemm_fsolver_set_comm(xfemm_fsolver *h, xfk_comm *comm)
{
    if (!h) return 0;
    h->s.comm = comm;
    return 1;
}

int xfemm_fsolver_set_delete_mesh_files(xfemm_fsolver *h, int del)
{
    if (!h) return 0;
    h->s.deleteMeshFiles = del != 0;
    return 1;
}

int xfemm_fsolver_load_problem_file(xfemm_fsolver *h)
{
    return guarded(h, [&] { return h->s.LoadProblemFile(); });
}

int xfemm_fsolver_run_solver(xfemm_fsolver *h, int verbose)
{
    return guarded(h, [&] { return h->s.runSolver(verbose != 0); });
}

int xfemm_fsolver_load_mesh(xfemm_fsolver *h)
{
    return guarded(h, [&] {
        xfemm::LoadMeshErr err = h->s.LoadMesh(h->s.deleteMeshFiles);
        h->s.join_removals();
        if (err != xfemm::NOERROR) {
            h->s.lastError = xfemm::FSolver::getErrorString(err);
            return false;
        }
        return true;
    });
}

int xfemm_fsolver_cuthill(xfemm_fsolver *h)
{
    return guarded(h, [&] {
        const int ok = h->s.Cuthill(h->s.deleteMeshFiles);
        h->s.join_removals();
        return ok != 0;
    });
}

int xfemm_fsolver_get_nodes(xfemm_fsolver *h, double *x, double *y, int *marker)
{
    if (!h) return 0;
    for (int i = 0; i < h->s.NumNodes; i++) {
        if (x) x[i] = h->s.meshnode[i].x;
        if (y) y[i] = h->s.meshnode[i].y;
        if (marker) marker[i] = h->s.meshnode[i].BoundaryMarker;
    }
    return 1;
}

int xfemm_fsolver_get_element_edges(xfemm_fsolver *h, int *e)
{
    if (!h || !e) return 0;
    for (int i = 0; i < h->s.NumEls; i++)
        for (int q = 0; q < 3; q++) e[3 * i + q] = h->s.meshele[i].e[q];
    return 1;
}

int xfemm_fsolver_num_pbcs(xfemm_fsolver *h) { return h ? h->s.NumPBCs : 0; }

int xfemm_fsolver_get_pbcs(xfemm_fsolver *h, int *pbc3)
{
    if (!h || !pbc3) return 0;
    for (int k = 0; k < h->s.NumPBCs; k++) {
        pbc3[3 * k] = h->s.pbclist[k].x;
        pbc3[3 * k + 1] = h->s.pbclist[k].y;
        pbc3[3 * k + 2] = h->s.pbclist[k].t;
    }
    return 1;
}

int xfemm_fsolver_bandwidth(xfemm_fsolver *h) { return h ? h->s.BandWidth : 0; }

int xfemm_fsolver_num_air_gaps(xfemm_fsolver *h) { return h ? (int)h->s.agelist.size() : 0; }

int xfemm_fsolver_get_air_gap_nodes(xfemm_fsolver *h, int *counts, int *quad4)
{
    if (!h) return 0;
    int total = 0;
    for (size_t i = 0; i < h->s.agelist.size(); i++) {
        const std::vector<int> &qn = h->s.agelist[i].qn;
        const int nq = (int)(qn.size() / 4);
        if (counts) counts[i] = nq;
        if (quad4) std::copy(qn.begin(), qn.end(), quad4 + 4 * (size_t)total);
        total += nq;
    }
    return total;
}

int xfemm_fsolver_get_block_bh(xfemm_fsolver *h, int k, double *B, double *H, double *slope, double *mu_x)
{
    if (!h || k < 0 || k >= (int)h->s.blockproplist.size()) return -1;
    const xfemm::CMSolverMaterialProp &m = h->s.blockproplist[k];
    for (int i = 0; i < m.BHpoints && i < (int)m.slope.size(); i++) {
        if (B) B[i] = m.Bdata[i];
        if (H) H[i] = m.Hdata[i];
        if (slope) slope[i] = m.slope[i];
    }
    if (mu_x) *mu_x = m.mu_x;
    return m.BHpoints;
}

int xfemm_fsolver_num_nodes(xfemm_fsolver *h) { return h ? h->s.NumNodes : 0; }

int xfemm_fsolver_num_elements(xfemm_fsolver *h) { return h ? h->s.NumEls : 0; }

int xfemm_fsolver_get_solution(xfemm_fsolver *h, double *x, double *y, double *A)
{
    if (!h || (int)h->s.A.size() != h->s.NumNodes) return 0;
    const double unitconv[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    const double cf = unitconv[h->s.LengthUnits];
    for (int i = 0; i < h->s.NumNodes; i++) {
        if (x) x[i] = h->s.meshnode[i].x / cf;
        if (y) y[i] = h->s.meshnode[i].y / cf;
        if (A) A[i] = h->s.A[i];
    }
    return 1;
}

int xfemm_fsolver_get_elements(xfemm_fsolver *h, int *p, int *lbl)
{
    if (!h) return 0;
    for (int i = 0; i < h->s.NumEls; i++) {
        for (int q = 0; q < 3; q++)
            if (p) p[3 * i + q] = h->s.meshele[i].p[q];
        if (lbl) lbl[i] = h->s.meshele[i].lbl;
    }
    return 1;
}

int xfemm_fsolver_get_stats(xfemm_fsolver *h, xfk_result *out)
{
    if (!h || !out) return 0;
    *out = h->s.stats;
    return 1;
}

int xfemm_fsolver_get_times(xfemm_fsolver *h, double *ms)
{
    if (!h || !ms) return 0;
    for (int k = 0; k < 5; ++k) ms[k] = h->s.ms_phase[k];
    return 1;
}

const char *xfemm_fsolver_last_error(xfemm_fsolver *h) { return h ? h->s.lastError.c_str() : ""; }

int xfemm_fsolver_set_previous_solution_file(xfemm_fsolver *h, const char *path)
{
    if (!h) return 0;
    h->s.previousSolutionFile = path ? path : "";
    return 1;
}

const char *xfemm_fsolver_previous_solution_file(xfemm_fsolver *h)
{
    return h ? h->s.previousSolutionFile.c_str() : "";
}

int xfemm_fsolver_ac_solver(xfemm_fsolver *h) { return h ? h->s.ACSolver : -1; }

double xfemm_fsolver_frequency(xfemm_fsolver *h) { return h ? h->s.Frequency : 0.0; }

int xfemm_fsolver_num_line_props(xfemm_fsolver *h) { return h ? (int)h->s.lineproplist.size() : -1; }

int xfemm_fsolver_num_node_props(xfemm_fsolver *h) { return h ? (int)h->s.nodeproplist.size() : -1; }

int xfemm_fsolver_num_block_props(xfemm_fsolver *h) { return h ? (int)h->s.blockproplist.size() : -1; }

int xfemm_fsolver_num_circ_props(xfemm_fsolver *h) { return h ? (int)h->s.circproplist.size() : -1; }

int xfemm_fsolver_num_block_labels(xfemm_fsolver *h) { return h ? (int)h->s.labellist.size() : -1; }

int xfemm_bh_get_slopes(int n, double *B, double *H, double *slope, int lam_type, double lam_fill, double *mu_x)
{
    if (n < 2 || !B || !H || !slope) return 0;
    xfemm::CMSolverMaterialProp m;
    m.BHpoints = n;
    m.Bdata.assign(B, B + n);
    m.Hdata.assign(H, H + n);
    m.LamType = lam_type;
    m.LamFill = lam_fill;
    if (!m.GetSlopes()) return 0;
    for (int i = 0; i < n; i++) {
        B[i] = m.Bdata[i];
        H[i] = m.Hdata[i];
        slope[i] = m.slope[i];
    }
    if (mu_x) *mu_x = m.mu_x;
    return 1;
}

int xfemm_bh_get_slopes_ac(int n, double *B, double *H, double *H_im, double *slope, double *slope_im, double omega,
                           int lam_type, double lam_fill, double theta_hn, double lam_d, double cduct, double *mu_x,
                           double *mu_max)
{
    if (n < 2 || !B || !H || !H_im || !slope || !slope_im || !(omega >= 0)) return 0;
    xfemm::CMSolverMaterialProp m;
    m.BHpoints = n;
    m.Bdata.assign(B, B + n);
    m.Hdata.assign(H, H + n);
    m.LamType = lam_type;
    m.LamFill = lam_fill;
    m.Theta_hn = theta_hn;
    m.Lam_d = lam_d;
    m.Cduct = cduct;
    if (!m.GetSlopesAC(omega)) return 0;
    for (int i = 0; i < n; i++) {
        B[i] = m.Bdata[i];
        H[i] = m.Hdata[i];
        H_im[i] = m.Hdata_im[i];
        slope[i] = m.slope[i];
        slope_im[i] = m.slope_im[i];
    }
    if (mu_x) *mu_x = m.mu_x;
    if (mu_max) *mu_max = m.MuMax;
    return 1;
}

}  // extern "C"
