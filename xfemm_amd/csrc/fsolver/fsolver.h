// FSolver: the magnetics solver object of the reference (cfemm/fsolver/fsolver.h),
// re-hosted over the MI355X kernels (include/xfemm_kernels.h).
//
// Same public surface and behaviour for the static planar path:
//   PathName, LoadProblemFile(), LoadMesh(), Cuthill(), runSolver(verbose),
//   Static2D(), WriteStatic2D(), WarnMessage / PrintMessage hooks,
//   meshnode / meshele / *proplist / pbclist state.
// The linear system never exists on the host: Static2D() uploads the mesh
// and property tables and runs assembly + PCG + Newton on the GPU.
#pragma once

#include <array>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/xfemm_kernels.h"
#include "femm_problem.h"
#include "hostmem.h"

namespace xfemm {

enum LoadMeshErr { NOERROR, BADFEMFILE, BADNODEFILE, BADPBCFILE, BADELEMENTFILE, BADEDGEFILE, MISSINGMATPROPS,
                   ELMLABELTOOBIG, UNSUPPORTEDMESH };

int PrintWarningMsg(const char *fmt, ...);

class FSolver : public FemmProblemData {
public:
    FSolver();
    ~FSolver();
    FSolver(const FSolver &) = delete;
    FSolver &operator=(const FSolver &) = delete;

    // General problem attributes (fsolver.h / feasolver.h)
    std::string PathName;
    double Relax = 0.0;
    int NumNodes = 0, NumEls = 0, BandWidth = 0, NumPBCs = 0, NumAirGapElems = 0, NumCircPropsOrig = 0;
    BigVec<CNode> meshnode;      // (parallel first touch: hostmem.h)
    BigVec<CMElement> meshele;
    std::vector<CCommonPoint> pbclist;
    // CAirGapElement as read from the .pbc file (fsolver.cpp:425-515)
    struct AirGap {
        std::string name;
        int format = 0, n_arc = 0;
        double inner_angle = 0, outer_angle = 0, ri = 0, ro = 0, arc = 0, agc_re = 0, agc_im = 0;
        double inner_shift = 0, outer_shift = 0;
        std::vector<int> qn;       // 4 per quadNode
        std::vector<double> qw;
    };
    std::vector<AirGap> agelist;

    int (*WarnMessage)(const char *, ...);
    int (*PrintMessage)(const char *, ...);

    // GPU selection and file handling
    int device = 0;
    bool deleteMeshFiles = true;
    // sharded solve over comm's ranks (xfk_problem_create_dist): every rank
    // runs its own FSolver on the same files; rank 0 writes the .ans and
    // deletes the mesh files.  nullptr: one device.
    xfk_comm *comm = nullptr;
    bool writes_output() const;

    bool LoadProblemFile();                              // fsolver.cpp:202-348
    bool loadPreviousSolution(bool loadAprev);           // fsolver.cpp:990-1081
    LoadMeshErr LoadMesh(bool deleteFiles = true);       // fsolver.cpp:350-718
    int Cuthill(bool deleteFiles = true);                // cuthill.cpp:88-390
    int SortElements();                                  // cuthill.cpp:39-86
    bool runSolver(bool verbose = false);                // fsolver.cpp:1213-1338
    int Static2D();                                      // static2d.cpp:53-1033 (on the GPU)
    int WriteStatic2D();                                 // static2d.cpp:1038-1195
    int Harmonic2D();                                    // harmonic2d.cpp:36-790 (on the GPU: linear, successive approximation, Newton AC)
    int WriteHarmonic2D();                               // harmonic2d.cpp:793-960
    void WriteAirGapElements(FILE *fp) const;            // static2d.cpp:1161-1190, harmonic2d.cpp:1002-1030
    void GetFillFactor(int lbl);                         // fsolver.cpp:1083-1193 (incl. ProximityMu)
    static std::string getErrorString(LoadMeshErr err);
    void join_removals();   // wait for the mesh-file deletions LoadMesh / Cuthill started
    // .ans text formatted in parallel chunks (fsolver.cpp: format_lines)
    struct Formatted {
        std::vector<HugeBuf<char>> buf;
        std::vector<size_t> len;
        // every chunk's buffer was allocated (a failed chunk is left empty)
        bool ok() const
        {
            for (const auto &b : buf)
                if (!b.data()) return false;
            return true;
        }
    };

    // result of the last Static2D: A (= V*c) per node, in meshnode order;
    // Harmonic2D: A holds the real parts and A_im the imaginary parts
    std::vector<double> A, A_im;
    // previous-solution problems ([PrevSoln]): A of the previous solution
    // (PrevType != 0), and whether the mesh came from it (fsolver.h:149)
    std::vector<double> Aprev;
    bool meshLoadedFromPrevSolution = false;
    xfk_result stats{};
    // wall milliseconds of the last runSolver: LoadMesh, Cuthill, problem
    // creation (descriptor + host -> HBM upload), solve (device + solution
    // read-back), write (.ans)
    double ms_phase[5] = {};
    std::string lastError;

private:
    BigVec<std::array<int, 3>> edges_;        // .edge content: n0, n1, marker
    std::vector<std::thread> removers_;       // mesh-file deletions in flight (joined by runSolver)
    void remove_async(std::vector<std::string> paths);
    template <class Src>
    bool permute_elements(Src src);
    std::thread ele_fmt_;                     // the .ans element section, formatted beside the solve
    // HIP runtime / device / code-object bring-up (xfk_device_init) started by
    // LoadProblemFile on a thread of its own, so a fresh process pays it beside
    // LoadMesh and Cuthill instead of inside the first device call; joined
    // before the first device use (SortElements, Static2D, Harmonic2D)
    std::thread hip_warm_;
    void start_hip_warmup();
    void join_hip_warmup();
    Formatted ele_text_;
    Formatted format_static_elements() const;
    // the .ans node lines without A (x, y before it; the marker and the
    // previous-solution A after it), formatted beside the solve: the lines of
    // chunk t are [lo[t], lo[t + 1]) with pre[i] / suf[i] bytes around A
    struct NodeParts {
        Formatted f;
        std::vector<int> lo;
        std::vector<unsigned char> pre, suf;
    };
    NodeParts node_parts_;
    NodeParts format_static_node_parts() const;
    void clear_old_output(const std::string &path);
    void remove_mesh_files_after_collective_solve();
    void warn(const std::string &msg);
    struct DescStore;                         // property tables + mesh arrays behind an xfk_problem_desc
    bool make_desc(DescStore &ds);
};

}  // namespace xfemm
