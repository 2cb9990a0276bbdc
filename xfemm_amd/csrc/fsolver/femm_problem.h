// Problem description of a magnetostatic .fem file, as the reference's
// FEASolver/FSolver hold it after LoadProblemFile.
//
// Mirrors (names and meaning): femm::CMPointProp (CPointProp.h),
// femm::CMBoundaryProp (CBoundaryProp.h), femm::CMSolverMaterialProp
// (CMaterialProp.h:193), femm::CMCircuit (CCircuit.h), femm::CMBlockLabel
// (CBlockLabel.h:153) and femm::CNode / femmsolver::CMElement
// (CNode.h, CElement.h).  The parser restates FEASolver::LoadProblemFile
// (cfemm/libfemm/feasolver.cpp:223-520) and the property fromStream readers.
#pragma once

#include <string>
#include <vector>

namespace xfemm {

constexpr double kMuo = 1.2566370614359173e-6;
constexpr double kPi = 3.141592653589793238462643383;
constexpr double kDeg = 0.01745329251994329576923690768;
constexpr double kLengthConvMeters[6] = {0.0254, 0.001, 0.01, 1., 2.54e-05, 1.e-06};

enum LengthUnit { LengthInches = 0, LengthMillimeters, LengthCentimeters, LengthMeters, LengthMils,
                  LengthMicrometers };
enum CoordsType { CART = 0, POLAR = 1 };
enum ProblemType { PLANAR = 0, AXISYMMETRIC = 1 };

struct CMPointProp {
    std::string PointName = "New Point Property";
    double A_re = 0, A_im = 0;   // prescribed A
    double J_re = 0, J_im = 0;   // point current
};

struct CMBoundaryProp {
    std::string BdryName = "New Boundary";
    int BdryFormat = 0;
    double A0 = 0, A1 = 0, A2 = 0, phi = 0;
    double Mu = 0, Sig = 0;
    double c0_re = 0, c0_im = 0, c1_re = 0, c1_im = 0;
    double InnerAngle = 0, OuterAngle = 0;
};

struct CMSolverMaterialProp {
    std::string BlockName = "New Material";
    double mu_x = 1., mu_y = 1.;
    double H_c = 0., Theta_m = 0.;
    double J_re = 0., J_im = 0.;
    double Cduct = 0., Lam_d = 0.;
    double Theta_hn = 0., Theta_hx = 0., Theta_hy = 0.;
    int LamType = 0;
    double LamFill = 1.;
    int NStrands = 0;
    double WireD = 0;
    int BHpoints = 0;
    std::vector<double> Bdata, Hdata;   // H real parts (static problems)
    std::vector<double> slope;
    std::vector<double> Hdata_im, slope_im;   // imaginary parts (GetSlopesAC)
    double MuMax = 0;

    // CMMaterialProp::GetSlopes(omega = 0) (CMaterialProp.cpp:127-348)
    bool GetSlopes();
    // CMMaterialProp::GetSlopes(omega > 0) with CMSolverMaterialProp::LaminatedBH
    // (CMaterialProp.cpp:127-348, 1060-1160): the effective B-H curve for a
    // sinusoidal H, the hysteresis-lag kludge, the 1-D lamination eddy-current
    // solve per curve point, the lamination fill.  Complex H and slopes come
    // back in Hdata / Hdata_im and slope / slope_im; MuMax is set.
    bool GetSlopesAC(double omega);
};

struct CMCircuit {
    std::string CircName = "New Circuit";
    int CircType = 0;
    double Amps_re = 0, Amps_im = 0;
    double dVolts_re = 0, dVolts_im = 0;
    int OrigCirc = 0;
    // outputs of Static2D / Harmonic2D (imaginary parts: Harmonic2D only)
    int Case = 0;
    double J = 0, dV = 0;
    double J_im = 0, dV_im = 0;
};

struct CMBlockLabel {
    double x = 0, y = 0;
    int BlockType = -1;
    double MaxArea = 0;
    int InCircuit = -1;
    double MagDir = 0;
    int InGroup = 0;
    int Turns = 1;
    bool IsDefault = false, IsExternal = false;
    std::string MagDirFctn;
    bool bIsWound = false;
    double ProxMu_re = 1, ProxMu_im = 0;   // ProximityMu (GetFillFactor, AC wound LamType > 2 regions)
};

struct CNode {
    double x = 0, y = 0;     // cm after LoadMesh
    int BoundaryMarker = -1;
};

struct CMElement {
    int p[3] = {0, 0, 0};
    int e[3] = {-1, -1, -1};
    int blk = 0, lbl = 0;
    double Jprev = 0;   // previous-solution problems: the element's J column of the .ans
};

struct CCommonPoint {
    int x = 0, y = 0, t = 0;
};

// The .fem content (FEASolver attributes, feasolver.h).
struct FemmProblemData {
    double FileFormat = -1;
    double Frequency = 0;
    double Precision = 1.e-08;
    double MinAngle = 0.;
    double Depth = -1;
    LengthUnit LengthUnits = LengthInches;
    CoordsType Coords = CART;
    ProblemType ProblemTypeV = PLANAR;
    double extZo = 0, extRo = 0, extRi = 0;   // axisymmetric exterior region, user units
    int ACSolver = 0;
    int PrevType = 0;
    std::string previousSolutionFile;
    bool prevSolnInFile = false;       // the .fem had a [PrevSoln] line
    std::string comment;
    std::vector<CMPointProp> nodeproplist;
    std::vector<CMBoundaryProp> lineproplist;
    std::vector<CMSolverMaterialProp> blockproplist;
    std::vector<CMCircuit> circproplist;
    std::vector<CMBlockLabel> labellist;
};

// FEASolver::LoadProblemFile: returns false and fills `err` on a parse error.
bool ParseFemFile(const std::string &path, FemmProblemData &out, std::string &err);

}  // namespace xfemm
