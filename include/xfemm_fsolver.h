/* xfemm_fsolver.h -- C-ABI of the file-based magnetics solver (FSolver) whose
 * static-2D hot path runs on MI355X (include/xfemm_kernels.h).
 *
 * This is the surface the reference's own foreign-function binding drives:
 * mfemm/mexfsolver.cpp (the MATLAB/Octave MEX gateway) creates an FSolver,
 * sets PathName and the WarnMessage/PrintMessage hooks, calls
 * LoadProblemFile() and runSolver(verbose), and returns 1/2 on failure.
 * Each entry point below replaces one step of that sequence:
 *
 *   xfemm_fsolver_create / _destroy     std::make_shared<FSolver>()        mexfsolver.cpp:31
 *   xfemm_fsolver_set_message_handlers  SolveObj->WarnMessage/PrintMessage mexfsolver.cpp:100-111
 *   xfemm_fsolver_set_pathname          SolveObj->PathName                 mexfsolver.cpp:115
 *   xfemm_fsolver_load_problem_file     FSolver::LoadProblemFile()         fsolver/fsolver.cpp:202
 *   xfemm_fsolver_run_solver            FSolver::runSolver(verbose)        fsolver/fsolver.cpp:1213
 *   xfemm_fsolver_set_delete_mesh_files FSolver::LoadMesh(deleteFiles)     fsolver/fsolver.cpp:350
 *
 * Boolean results follow the reference: 1 = success (true), 0 = failure.
 * Output: <PathName>.ans in the reference's WriteStatic2D layout
 * (fsolver/static2d.cpp:1038-1195).
 */
#ifndef XFEMM_FSOLVER_H
#define XFEMM_FSOLVER_H

#include "xfemm_kernels.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct xfemm_fsolver xfemm_fsolver;
typedef int (*xfemm_message_fn)(const char *fmt, ...);

xfemm_fsolver *xfemm_fsolver_create(void);
void xfemm_fsolver_destroy(xfemm_fsolver *s);
void xfemm_fsolver_set_message_handlers(xfemm_fsolver *s, xfemm_message_fn warn, xfemm_message_fn print);
int xfemm_fsolver_set_pathname(xfemm_fsolver *s, const char *path_without_extension);
int xfemm_fsolver_set_device(xfemm_fsolver *s, int device);
int xfemm_fsolver_set_delete_mesh_files(xfemm_fsolver *s, int delete_files);
/* Sharded solve (north_star: large meshes shard across up to 8 GPUs under the
 * same FSolver API).  Every rank of `comm` (include/xfemm_kernels.h:
 * xfk_comm_create_rccl, one process per GPU, or xfk_comm_create_local)
 * creates its own FSolver on the same PathName and calls
 * load_problem_file / run_solver; runSolver (reference fsolver.cpp:1213-1340)
 * then builds the rank's row block with xfk_problem_create_dist /
 * xfk_problem_create_harmonic_dist, the solve is collective, every rank holds
 * the global solution afterwards, rank 0 writes the .ans and deletes the mesh
 * files (after the collective solve, so every rank has read them).  The
 * communicator stays the caller's.  NULL: one device (the default). */
int xfemm_fsolver_set_comm(xfemm_fsolver *s, xfk_comm *comm);
int xfemm_fsolver_load_problem_file(xfemm_fsolver *s);
int xfemm_fsolver_run_solver(xfemm_fsolver *s, int verbose);

/* Host-only steps of runSolver, for callers that drive them one by one:
 * FSolver::LoadMesh (fsolver.cpp:350) and FSolver::Cuthill (cuthill.cpp:88). */
int xfemm_fsolver_load_mesh(xfemm_fsolver *s);
int xfemm_fsolver_cuthill(xfemm_fsolver *s);
int xfemm_fsolver_get_nodes(xfemm_fsolver *s, double *x_cm, double *y_cm, int *marker);
int xfemm_fsolver_get_element_edges(xfemm_fsolver *s, int *e);
int xfemm_fsolver_get_pbcs(xfemm_fsolver *s, int *pbc3);
int xfemm_fsolver_num_pbcs(xfemm_fsolver *s);
int xfemm_fsolver_bandwidth(xfemm_fsolver *s);
/* Air gaps (FEASolver::agelist, feasolver.h:141): the number of quadNodes of
 * each (totalArcElements + 1) into counts[num_air_gaps], and their node ids
 * n0..n3 (CQuadPoint, libfemm/CQuadPoint.h) air gap by air gap into quad4 --
 * after Cuthill in the renumbered ids (cuthill.cpp:320-330).  Returns the
 * total number of quadNodes; either array may be NULL to query sizes. */
int xfemm_fsolver_num_air_gaps(xfemm_fsolver *s);
int xfemm_fsolver_get_air_gap_nodes(xfemm_fsolver *s, int *counts, int *quad4);
/* processed B-H curve of block k after LoadProblemFile (GetSlopes); returns BHpoints */
int xfemm_fsolver_get_block_bh(xfemm_fsolver *s, int k, double *B, double *H, double *slope, double *mu_x);

/* state after run_solver (renumbered order, as written to the .ans) */
int xfemm_fsolver_num_nodes(xfemm_fsolver *s);
int xfemm_fsolver_num_elements(xfemm_fsolver *s);
int xfemm_fsolver_get_solution(xfemm_fsolver *s, double *x, double *y, double *A);
int xfemm_fsolver_get_elements(xfemm_fsolver *s, int *p, int *lbl);
int xfemm_fsolver_get_stats(xfemm_fsolver *s, xfk_result *out);
/* Wall milliseconds of the last runSolver (fsolver.cpp:1213-1340 is the
 * reference's sequence): ms[0] LoadMesh, ms[1] Cuthill-McKee, ms[2] problem
 * creation (descriptor, host -> HBM upload), ms[3] solve (device work and the
 * solution read-back), ms[4] .ans write. */
int xfemm_fsolver_get_times(xfemm_fsolver *s, double *ms);
const char *xfemm_fsolver_last_error(xfemm_fsolver *s);

/* femmcli's binding (cfemm/femmcli/LuaMagneticsCommands.cpp:817-842, mi_analyze):
 * it sets FSolver::previousSolutionFile from the document before
 * LoadProblemFile (:824) -- kept unless the .fem carries its own [PrevSoln]
 * line, as FEASolver::CleanUp leaves the member alone (feasolver.cpp:134-172)
 * -- and then asserts the loaded solver against the document (:830-838):
 * ACSolver, Frequency and the sizes of the property lists (circuits may grow
 * by the serial expansion; labels exclude holes).  Getters return -1 (0.0
 * for the frequency) on a NULL handle. */
int xfemm_fsolver_set_previous_solution_file(xfemm_fsolver *s, const char *path);   /* fsolver.h previousSolutionFile */
const char *xfemm_fsolver_previous_solution_file(xfemm_fsolver *s);
int xfemm_fsolver_ac_solver(xfemm_fsolver *s);               /* FSolver::ACSolver */
double xfemm_fsolver_frequency(xfemm_fsolver *s);            /* FSolver::Frequency (Hz) */
int xfemm_fsolver_num_line_props(xfemm_fsolver *s);          /* lineproplist.size() */
int xfemm_fsolver_num_node_props(xfemm_fsolver *s);          /* nodeproplist.size() */
int xfemm_fsolver_num_block_props(xfemm_fsolver *s);         /* blockproplist.size() */
int xfemm_fsolver_num_circ_props(xfemm_fsolver *s);          /* circproplist.size(), after the serial expansion */
int xfemm_fsolver_num_block_labels(xfemm_fsolver *s);        /* labellist.size() */

/* CMMaterialProp::GetSlopes(0) (libfemm/CMaterialProp.cpp:127): processes a
 * B-H curve in place (B, H: n points) and writes the knot slopes; returns the
 * initial relative permeability in *mu_x.  1 on success. */
int xfemm_bh_get_slopes(int n, double *B, double *H, double *slope, int lam_type, double lam_fill,
                        double *mu_x);
/* CMMaterialProp::GetSlopes(omega > 0) with CMSolverMaterialProp::LaminatedBH
 * (CMaterialProp.cpp:127-348, 1060-1160): the harmonic solver's complex curve.
 * B, H in place (H gets its real part, H_im the imaginary part), complex knot
 * slopes in slope / slope_im; *mu_x the initial relative permeability, *mu_max
 * MuMax.  theta_hn: hysteresis lag (deg); lam_d (mm) and cduct (MS/m) drive
 * the lamination eddy-current correction.  1 on success. */
int xfemm_bh_get_slopes_ac(int n, double *B, double *H, double *H_im, double *slope, double *slope_im,
                           double omega, int lam_type, double lam_fill, double theta_hn, double lam_d,
                           double cduct, double *mu_x, double *mu_max);

#ifdef __cplusplus
}
#endif
#endif
