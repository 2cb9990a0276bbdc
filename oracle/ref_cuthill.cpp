// C adapter over the REFERENCE's own renumbering, compiled from /root/reference
// by oracle/Makefile into oracle/_ref/libref_cuthill.so.
//
// TEST INFRASTRUCTURE ONLY (pins the product FSolver's node / element order,
// bandwidth, periodic-pair and air-gap quad-node remap -- index work, so
// array-equal).  Nothing of the reference is copied: like the reference's
// fsolver/fsolver.cpp:55-56 this file #includes libfemm/feasolver.cpp and
// libfemm/cuthill.cpp to instantiate FEASolver<...> with the fsolver's own
// CM* types, and supplies the three pure virtuals of feasolver.h:146,153,207
// as harness code:
//   LoadMesh   -- not used (the arrays come in through ref_cuthill_run),
//   runSolver  -- not used,
//   SortNodes  -- records the node numbering newnum that Cuthill hands over.
// FEASolver::Cuthill (cuthill.cpp:94-391) reads PathName.edge itself, exactly
// as the reference fsolver does after LoadMesh, then calls SortNodes and
// SortElements (the comb sort, cuthill.cpp:33-85).
#include <cstring>
#include <vector>

#include "feasolver.cpp"
#include "cuthill.cpp"

#include "CBlockLabel.h"
#include "CBoundaryProp.h"
#include "CCircuit.h"
#include "CElement.h"
#include "CMaterialProp.h"
#include "CPointProp.h"

namespace {

using RefBase = FEASolver<femm::CMPointProp, femm::CMBoundaryProp, femm::CMSolverMaterialProp,
                          femm::CMCircuit, femm::CMBlockLabel, femmsolver::CMElement>;

class RefRenumber : public RefBase
{
public:
    std::vector<int> newnum;
    LoadMeshErr LoadMesh(bool) override { return NOERROR; }
    bool runSolver(bool) override { return false; }

private:
    void SortNodes(std::vector<int> nn) override { newnum = nn; }
};

int quiet(const char *, ...) { return 0; }

}  // namespace

extern "C" {

// Run the reference's Cuthill(deletefiles = false) on one mesh.
//   path       : PathName (the mesh's .edge file is read from path + ".edge")
//   p          : 3 * num_els node ids in LoadMesh order; overwritten with the
//                renumbered, SortElements-ordered corners
//   elem_order : num_els; elem_order[k] = LoadMesh index of the element that
//                ends at position k
//   newnum     : num_nodes; LoadMesh node id -> solver node id
//   pbc        : 2 * num_pbcs (x, y) node ids, remapped in place
//   age_quad   : 4 * num_quad node ids (n0..n3 of every quadNode of every air
//                gap, air gap by air gap), remapped in place; age_counts[i] is
//                the number of quadNodes of air gap i (totalArcElements + 1)
// Returns the reference's BandWidth, or -1 when Cuthill returns false.
int ref_cuthill_run(const char *path, int num_nodes, int num_els, int *p, int *elem_order,
                    int *newnum, int num_pbcs, int *pbc, int num_ages, const int *age_counts,
                    int *age_quad)
{
    RefRenumber s;
    s.WarnMessage = &quiet;
    s.PrintMessage = &quiet;
    s.PathName = path;
    s.NumNodes = num_nodes;
    s.NumEls = num_els;
    s.meshele.resize(num_els);
    for (int k = 0; k < num_els; k++) {
        femmsolver::CMElement &e = s.meshele[k];
        e.p[0] = p[3 * k];
        e.p[1] = p[3 * k + 1];
        e.p[2] = p[3 * k + 2];
        e.blk = k;   // carried through the swaps: the element's LoadMesh index
    }
    s.NumPBCs = num_pbcs;
    s.pbclist.resize(num_pbcs);
    for (int i = 0; i < num_pbcs; i++) {
        s.pbclist[i].x = pbc[2 * i];
        s.pbclist[i].y = pbc[2 * i + 1];
    }
    s.NumAirGapElems = num_ages;
    s.agelist.resize(num_ages);
    int q = 0;
    for (int i = 0; i < num_ages; i++) {
        femmsolver::CAirGapElement &g = s.agelist[i];
        g.totalArcElements = age_counts[i] - 1;
        g.quadNode.resize(age_counts[i]);
        for (int k = 0; k < age_counts[i]; k++, q++) {
            g.quadNode[k].n0 = age_quad[4 * q];
            g.quadNode[k].n1 = age_quad[4 * q + 1];
            g.quadNode[k].n2 = age_quad[4 * q + 2];
            g.quadNode[k].n3 = age_quad[4 * q + 3];
        }
    }
    if (!s.Cuthill(false))
        return -1;
    for (int k = 0; k < num_els; k++) {
        p[3 * k] = s.meshele[k].p[0];
        p[3 * k + 1] = s.meshele[k].p[1];
        p[3 * k + 2] = s.meshele[k].p[2];
        elem_order[k] = s.meshele[k].blk;
    }
    std::memcpy(newnum, s.newnum.data(), sizeof(int) * num_nodes);
    for (int i = 0; i < num_pbcs; i++) {
        pbc[2 * i] = s.pbclist[i].x;
        pbc[2 * i + 1] = s.pbclist[i].y;
    }
    q = 0;
    for (int i = 0; i < num_ages; i++)
        for (const femm::CQuadPoint &qp : s.agelist[i].quadNode) {
            age_quad[4 * q] = qp.n0;
            age_quad[4 * q + 1] = qp.n1;
            age_quad[4 * q + 2] = qp.n2;
            age_quad[4 * q + 3] = qp.n3;
            q++;
        }
    return s.BandWidth;
}

}  // extern "C"
