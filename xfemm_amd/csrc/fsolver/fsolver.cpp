// FSolver host logic over the MI355X kernels (see fsolver.h).
#include "fsolver.h"

#include <algorithm>
#include <atomic>
#include <cctype>
#include <charconv>
#include <chrono>
#include <complex>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <type_traits>
#include <thread>
#include <unordered_map>
#include <utility>

#include <fcntl.h>
#include <immintrin.h>
#include <sys/stat.h>
#include <unistd.h>

#include "fastnum.h"
#include "hostmem.h"
#include "hostpool.h"

namespace xfemm {

int PrintWarningMsg(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    int r = vfprintf(stderr, fmt, ap);
    va_end(ap);
    return r;
}

FSolver::FSolver() : WarnMessage(&PrintWarningMsg), PrintMessage(&PrintWarningMsg) {}

FSolver::~FSolver()
{
    if (ele_fmt_.joinable()) ele_fmt_.join();
    join_hip_warmup();
    join_removals();
}

void FSolver::start_hip_warmup()
{
    // a sharded FSolver's communicator has brought the device up already;
    // XFEMM_NO_HIP_WARMUP=1 leaves the bring-up to the first device call
    if (comm || hip_warm_.joinable() || std::getenv("XFEMM_NO_HIP_WARMUP")) return;
    const int dev = device;
    hip_warm_ = std::thread([dev] { (void)xfk_device_init(dev); });
}

void FSolver::join_hip_warmup()
{
    if (hip_warm_.joinable()) hip_warm_.join();
}

// The mesh files the reference deletes once read (fsolver.cpp:711-716,
// cuthill.cpp:140): unlinking ~170 MB of page cache costs tens of ms, so it
// runs beside the rest of runSolver and is joined before runSolver returns.
void FSolver::remove_async(std::vector<std::string> paths)
{
    removers_.emplace_back([paths = std::move(paths)] {
        for (const auto &p : paths) remove(p.c_str());
    });
}

bool FSolver::writes_output() const { return !comm || xfk_comm_rank(comm) == 0; }

void FSolver::remove_mesh_files_after_collective_solve()
{
    // what a one-device run deletes: LoadMesh's four files whenever it read
    // them (not for a mesh taken from the previous solution, fsolver.cpp:357-360),
    // the .edge only after Cuthill (which runs without a previous solution)
    if (!comm || !deleteMeshFiles || xfk_comm_rank(comm) != 0 || meshLoadedFromPrevSolution) return;
    std::vector<std::string> v;
    for (const char *ext : {".ele", ".node", ".pbc", ".poly"}) v.push_back(PathName + ext);
    if (previousSolutionFile.empty()) v.push_back(PathName + ".edge");
    remove_async(std::move(v));
}

void FSolver::join_removals()
{
    for (auto &t : removers_) t.join();
    removers_.clear();
}

void FSolver::warn(const std::string &msg)
{
    lastError = msg;
    WarnMessage("%s", msg.c_str());
}

std::string FSolver::getErrorString(LoadMeshErr err)
{
    switch (err) {
    case NOERROR: return std::string();
    case BADEDGEFILE: return "problem loading mesh:\nCould not open .edge file.\n";
    case BADELEMENTFILE: return "problem loading mesh:\nCould not open .ele file.\n";
    case BADFEMFILE: return "problem loading mesh:\nCould not open .fem file.\n";
    case BADNODEFILE: return "problem loading mesh:\nCould not open .node file.\n";
    case BADPBCFILE: return "problem loading mesh:\nCould not open .pbc file.\n";
    case MISSINGMATPROPS: return "problem loading mesh:\nMaterial properties have not been defined for all regions.\n";
    case ELMLABELTOOBIG:
        return "problem loading mesh:\nElemnet label number was greater than the number of labels in the problem.\n";
    case UNSUPPORTEDMESH: return "problem loading mesh:\nmalformed air-gap element data.\n";
    }
    return std::string();
}

bool FSolver::LoadProblemFile()
{
    start_hip_warmup();
    Relax = 1.;
    std::string err;
    FemmProblemData &base = *this;
    // a previous-solution file set by the caller survives the parse unless the
    // .fem names one itself (FEASolver::CleanUp keeps previousSolutionFile,
    // feasolver.cpp:134-172; femmcli sets it before LoadProblemFile,
    // LuaMagneticsCommands.cpp:824)
    const std::string presetPrev = previousSolutionFile;
    if (!ParseFemFile(PathName + ".fem", base, err)) {
        warn(err);
        return false;
    }
    if (!prevSolnInFile) previousSolutionFile = presetPrev;
    meshLoadedFromPrevSolution = false;
    if (!previousSolutionFile.empty()) {
        // fsolver.cpp:224-238: the mesh (and A, for PrevType != 0) come from
        // the previous solution, and LoadProblemFile returns right there --
        // before GetSlopes and the serial-circuit expansion below.  On a B-H
        // block or a serial circuit the reference then runs on uncomputed
        // slopes / an unexpanded circuit (undefined); refused here.
        for (auto &prop : blockproplist)
            if (prop.BHpoints > 0) {
                warn("B-H curves with a previous solution: the reference never computes their slopes "
                     "(fsolver.cpp:224-238)\n");
                return false;
            }
        for (auto &c : circproplist)
            if (c.CircType == 1) {
                warn("serial circuits with a previous solution: the reference skips their expansion "
                     "(fsolver.cpp:224-238)\n");
                return false;
            }
        return loadPreviousSolution(PrevType != 0);
    }
    // B-H curves: GetSlopes(Frequency * 2 pi) (fsolver.cpp:241-276; the
    // harmonic curve is complex: effective sinusoidal-H amplitude, hysteresis
    // lag, lamination eddy currents)
    for (auto &prop : blockproplist)
        if (prop.BHpoints > 0) {
            if (!(Frequency != 0 ? prop.GetSlopesAC(Frequency * 2. * kPi) : prop.GetSlopes())) {
                warn("bad B-H curve in material " + prop.BlockName + "\n");
                return false;
            }
            prop.MuMax = 0;
        }
    const int NumBlockLabels = (int)labellist.size();
    for (auto &lb : labellist)
        if (lb.InCircuit >= (int)circproplist.size()) {
            warn("block label refers to an undefined circuit\n");
            return false;
        }
    int NumCircProps = (int)circproplist.size();
    if (NumCircProps == 0) return true;
    // serial circuits -> one parallel circuit per block label (fsolver.cpp:280-317)
    for (auto &c : circproplist) c.OrigCirc = -1;
    NumCircPropsOrig = NumCircProps;
    for (int k = 0; k < NumBlockLabels; k++)
        if (labellist[k].InCircuit >= 0) {
            int ic = labellist[k].InCircuit;
            if (circproplist[ic].CircType == 1) {
                CMCircuit ncirc = circproplist[ic];
                ncirc.OrigCirc = ic;
                ncirc.Amps_im *= labellist[k].Turns;
                ncirc.Amps_re *= labellist[k].Turns;
                circproplist.push_back(ncirc);
                labellist[k].InCircuit = NumCircProps;
                NumCircProps++;
            }
        }
    for (auto &c : circproplist)
        if (c.CircType == 1) c.CircType = 0;
    return true;
}

// FSolver::loadPreviousSolution (fsolver.cpp:990-1081) and its readers
// (:801-988).  A WriteStatic2D .ans has p0 p1 p2 lbl per element, so the
// 8-field scan leaves e[] and Jprev at the CMElement defaults of the
// reference -- e = {0, 0, 0} (CElement.cpp:30-39): every edge carries boundary
// property 0 -- and Jprev = 0.
bool FSolver::loadPreviousSolution(bool loadAprev)
{
    if (previousSolutionFile.empty()) return false;
    FILE *fp = fopen(previousSolutionFile.c_str(), "rt");
    if (!fp) {
        warn("Failed to open the specified previous solution file, file path was:\n" + previousSolutionFile + "\n");
        return false;
    }
    char s[1024];
    bool hasSolution = false;
    while (fgets(s, 1024, fp) != nullptr) {
        char q[256] = {0};
        sscanf(s, "%255s", q);
        std::string key(q);
        for (auto &ch : key) ch = (char)tolower((unsigned char)ch);
        if (key.compare(0, 11, "[frequency]") == 0) {
            double prevFreq = 0;
            const char *v = strchr(s, '=');
            if (v) sscanf(v + 1, "%lf", &prevFreq);
            if (prevFreq != 0) {
                fclose(fp);
                warn("Previous solution file (" + previousSolutionFile +
                     ") appears to be an AC problem, only DC previous solutions are presently supported\n");
                return false;
            }
        }
        if (key.compare(0, 10, "[solution]") == 0) {
            hasSolution = true;
            break;
        }
    }
    if (!hasSolution) {
        fclose(fp);
        warn("No solution was found in previous solution file, file path was:\n" + previousSolutionFile + "\n");
        return false;
    }
    auto fail = [&](const char *what) {
        fclose(fp);
        warn(std::string("malformed previous solution file (") + what + "): " + previousSolutionFile + "\n");
        return false;
    };
    // nodes: x y A marker, lengths back to cm (fsolver.cpp:801-840)
    if (!fgets(s, 1024, fp) || sscanf(s, "%i", &NumNodes) != 1 || NumNodes < 0) return fail("node count");
    Aprev.clear();
    meshnode.assign(NumNodes, CNode());
    const double conv = 100 * kLengthConvMeters[LengthUnits];
    for (int i = 0; i < NumNodes; i++) {
        CNode node;
        double a = 0;
        if (!fgets(s, 1024, fp) || sscanf(s, "%lf %lf %lf %i", &node.x, &node.y, &a, &node.BoundaryMarker) < 3)
            return fail("node line");
        node.x *= conv;
        node.y *= conv;
        if (loadAprev) Aprev.push_back(a);
        meshnode[i] = node;
    }
    // elements: p0 p1 p2 lbl [e0 e1 e2 Jprev] (fsolver.cpp:842-880)
    if (!fgets(s, 1024, fp) || sscanf(s, "%i", &NumEls) != 1 || NumEls < 0) return fail("element count");
    meshele.assign(NumEls, CMElement());
    for (int i = 0; i < NumEls; i++) {
        CMElement elm;
        elm.e[0] = elm.e[1] = elm.e[2] = 0;
        if (!fgets(s, 1024, fp) ||
            sscanf(s, "%i %i %i %i %i %i %i %lf", &elm.p[0], &elm.p[1], &elm.p[2], &elm.lbl, &elm.e[0], &elm.e[1],
                   &elm.e[2], &elm.Jprev) < 4)
            return fail("element line");
        if (elm.lbl < 0 || elm.lbl >= (int)labellist.size()) return fail("element label");
        for (int q = 0; q < 3; q++)
            if (elm.p[q] < 0 || elm.p[q] >= NumNodes) return fail("element node");
        elm.blk = labellist[elm.lbl].BlockType;
        meshele[i] = elm;
    }
    // block-label circuit lines: skipped
    int numLabels = 0;
    if (!fgets(s, 1024, fp) || sscanf(s, "%i", &numLabels) != 1) return fail("label count");
    for (int i = 0; i < numLabels; i++)
        if (!fgets(s, 1024, fp)) return fail("label line");
    // periodic pairs (fsolver.cpp:882-909)
    NumPBCs = 0;
    pbclist.clear();
    if (fgets(s, 1024, fp) != nullptr) {
        sscanf(s, "%i", &NumPBCs);
        for (int i = 0; i < NumPBCs; i++) {
            CCommonPoint pbc;
            if (!fgets(s, 1024, fp) || sscanf(s, "%i %i %i", &pbc.x, &pbc.y, &pbc.t) != 3) return fail("pbc line");
            pbclist.push_back(pbc);
        }
    }
    // air-gap elements (fsolver.cpp:911-988): name (80 characters), parameters, quadNodes
    NumAirGapElems = 0;
    agelist.clear();
    if (fgets(s, 1024, fp) != nullptr) sscanf(s, "%i", &NumAirGapElems);
    for (int i = 0; i < NumAirGapElems; i++) {
        AirGap g;
        if (!fgets(s, 80, fp)) return fail("air-gap name");
        g.name = s;
        if (!fgets(s, 1024, fp) ||
            sscanf(s, "%i %lf %lf %lf %lf %lf %lf %lf %i %lf %lf", &g.format, &g.inner_angle, &g.outer_angle, &g.ri,
                   &g.ro, &g.arc, &g.agc_re, &g.agc_im, &g.n_arc, &g.inner_shift, &g.outer_shift) != 11 ||
            g.n_arc <= 0)
            return fail("air-gap parameters");
        for (int k = 0; k <= g.n_arc; k++) {
            int n[4];
            double w[4];
            if (!fgets(s, 1024, fp) ||
                sscanf(s, "%i %lf %i %lf %i %lf %i %lf", &n[0], &w[0], &n[1], &w[1], &n[2], &w[2], &n[3], &w[3]) != 8)
                return fail("air-gap quadNode");
            for (int m = 0; m < 4; m++) {
                if (n[m] < 0 || n[m] >= NumNodes) {
                    fclose(fp);
                    warn("An error occured while reading pbc file, quadNode has negative node number.\n");
                    return false;
                }
                g.qn.push_back(n[m]);
                g.qw.push_back(w[m]);
            }
        }
        agelist.push_back(g);
    }
    fclose(fp);
    BandWidth = 0;
    meshLoadedFromPrevSolution = true;
    return true;
}

namespace {
// XFEMM_TRACE_LOAD=1: host milliseconds of the mesh-loading / renumbering stages on stderr
struct LoadTrace {
    bool on = std::getenv("XFEMM_TRACE_LOAD") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char *what)
    {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[load] %-24s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

// Token readers with fscanf's semantics: "%i" (strtol base 0: decimal, 0x..,
// leading-0 octal) and "%lf" (strtod).  Digit strings take a direct decimal
// path (the value strtol gives); everything else goes through strtol /
// strtod, so every value is the reference's fscanf value to the bit.  `nl`:
// the token must lie on the current line (line-parallel parsing).
inline bool ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f'; }
inline bool skip_ws(const char *&p, bool nl)
{
    if (nl) {
        while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f') ++p;
        return *p && *p != '\n';
    }
    while (ws(*p)) ++p;
    return *p != 0;
}
inline bool read_int(const char *&p, int &v, bool nl)
{
    if (!skip_ws(p, nl)) return false;
    const char *q = p + (*p == '-' || *p == '+');
    if (*q >= '1' && *q <= '9') {   // plain decimal (no octal / hex prefix)
        long long a = 0;
        const char *r = q;
        while (*r >= '0' && *r <= '9' && r - q < 18) a = 10 * a + (*r++ - '0');
        if (!(*r >= '0' && *r <= '9') && a <= 2147483648LL) {
            v = (int)(*p == '-' ? -a : a);
            p = r;
            return true;
        }
    }
    char *end = nullptr;
    const long x = std::strtol(p, &end, 0);
    if (end == p) return false;
    v = (int)x;
    p = end;
    return true;
}
inline bool read_double(const char *&p, double &v, bool nl)
{
    if (!skip_ws(p, nl)) return false;
    const char *end = nullptr;   // (strtod's value and extent, exact fast path: fastnum.h)
    if (!fastnum::parse_double(p, v, &end)) return false;
    p = end;
    return true;
}

// [0, n) split over the host's cores (at most 16), f(begin, end) per part,
// on the persistent pool (hostpool.h)
template <class F>
void par_for(long long n, long long min_per_thread, F f)
{
    HostPool &pool = HostPool::get();
    const int T = (int)std::max<long long>(1, std::min<long long>((long long)pool.size(), n / std::max(1LL, min_per_thread)));
    if (T <= 1) {
        f(0LL, n);
        return;
    }
    pool.run(T, [&](int t) { f(n * t / T, n * (t + 1) / T); });
}

// v = n copies of val, the storage first-touched by the pool's threads
template <class T>
void par_assign(BigVec<T> &v, size_t n, const T &val)
{
    huge_reserve(v, n);
    v.clear();
    v.resize(n);   // (NoInitAlloc: nothing written)
    par_for((long long)n, 1 << 16, [&](long long a, long long b) {
        for (long long k = a; k < b; k++) ::new (&v[k]) T(val);
    });
}

// A whole mesh file in memory, read as the token stream fscanf sees.
struct TextBuf {
    // the file's bytes + a terminating NUL; not value-initialised (the
    // parallel reads below fill it, each thread faulting in its own pages),
    // on huge pages, kept for the next file of the mesh
    struct Bytes {
        HugeBuf<char> b;
        size_t n = 0;   // bytes incl. the NUL
        char *data() { return b.data(); }
        const char *data() const { return b.data(); }
        size_t size() const { return n; }
        char &operator[](size_t i) { return b[i]; }
    } d;
    size_t pos = 0;
    size_t hint = 0;      // bytes to allocate at least (the largest file to come)
    double ms_count = 0;  // (trace: the record-count pass of the last records())
    bool load(const std::string &path)
    {
        const int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) return false;
        struct stat st;
        if (::fstat(fd, &st) != 0) {
            ::close(fd);
            return false;
        }
        const size_t n = (size_t)std::max<off_t>(0, st.st_size);
        // (sized for the largest mesh file at the first load: .edge > .ele > .node for fmesher output)
        if (!d.b.allocate(std::max<size_t>(n + 1, hint))) {
            ::close(fd);
            return false;
        }
        // chunks of >= 4 MiB read side by side (pread: no shared file offset)
        const int T = (int)std::max<size_t>(1, std::min<size_t>(16, n >> 22));
        std::vector<size_t> got(T, 0);
        par_for(T, 1, [&](long long a, long long b) {
            for (long long t = a; t < b; ++t) {
                size_t o = n * t / T;
                const size_t e = n * (t + 1) / T;
                while (o < e) {
                    const ssize_t r = ::pread(fd, d.b.data() + o, e - o, (off_t)o);
                    if (r <= 0) break;
                    o += (size_t)r;
                    got[t] += (size_t)r;
                }
            }
        });
        ::close(fd);
        size_t tot = 0;
        for (size_t g : got) tot += g;
        if (tot != n) return false;
        d.b[n] = '\0';
        d.n = n + 1;
        pos = 0;
        return true;
    }
    bool next_int(int &v)
    {
        const char *p = d.data() + pos;
        if (!read_int(p, v, false)) return false;
        pos = (size_t)(p - d.data());
        return true;
    }
    // the first line's leading integer (fgets + sscanf "%i"), then the stream after that line
    bool header_int(int &v)
    {
        const char *nl = std::strchr(d.data(), '\n');
        std::string line(d.data(), nl ? (size_t)(nl - d.data()) : std::strlen(d.data()));
        pos = nl ? (size_t)(nl - d.data()) + 1 : d.size() - 1;
        return std::sscanf(line.c_str(), "%i", &v) == 1;
    }
    // `count` records from pos on, rec(p, index, nl) reading one record.
    // When every record sits on a line of its own (fmesher's layout) the lines
    // are parsed in parallel chunks -- the same values as the token stream;
    // any other layout (a record over several lines, extra tokens on a line)
    // is parsed as one sequential token stream, as fscanf reads it.
    template <class Rec>
    bool records(int count, Rec rec)
    {
        const char *base = d.data() + pos, *end = d.data() + d.size() - 1;
        const long long len = end - base;
        const int T = (int)std::max<long long>(1, std::min<long long>(HostPool::get().size(), len / (1 << 20)));
        bool ok = T > 1;
        const auto tc = std::chrono::steady_clock::now();
        ms_count = 0;
        if (ok) {
            // chunk starts at line starts; records (non-blank lines) per chunk
            std::vector<const char *> cs(T + 1);
            cs[0] = base;
            cs[T] = end;
            for (int t = 1; t < T; ++t) {
                const char *q = base + len * t / T;
                while (q < end && q[-1] != '\n') ++q;
                cs[t] = std::max(q, cs[t - 1]);
            }
            std::vector<long long> cnt(T + 1, 0);
            par_for(T, 1, [&](long long a, long long b) {
                for (long long t = a; t < b; ++t) {
                    // lines found by memchr; a line counts when a non-blank
                    // character precedes its end (leading blanks are few)
                    long long c = 0;
                    const char *q = cs[t], *const e = cs[t + 1];
                    while (q < e) {
                        const char *nl = static_cast<const char *>(std::memchr(q, '\n', (size_t)(e - q)));
                        const char *le = nl ? nl : e;
                        while (q < le && ws(*q)) ++q;
                        c += q < le;
                        q = nl ? nl + 1 : e;
                    }
                    cnt[t + 1] = c;
                }
            });
            for (int t = 0; t < T; ++t) cnt[t + 1] += cnt[t];
            ms_count = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc).count();
            ok = cnt[T] >= count;
            std::vector<char> good(T, 1);
            if (ok)
                par_for(T, 1, [&](long long a, long long b) {
                    for (long long t = a; t < b; ++t) {
                        long long k = cnt[t];
                        const char *q = cs[t];
                        while (q < cs[t + 1] && k < count) {
                            const char *p = q;
                            if (!skip_ws(p, true)) {   // blank line
                                q = p + (*p == '\n');
                                continue;
                            }
                            if (!rec(p, (int)k, true) || skip_ws(p, true)) {   // short record or extra tokens
                                good[t] = 0;
                                return;
                            }
                            ++k;
                            q = p + (*p == '\n');
                        }
                    }
                });
            for (char g : good) ok = ok && g;
        }
        if (!ok) {   // the token stream, sequentially
            const char *p = base;
            for (int k = 0; k < count; ++k)
                if (!rec(p, k, false)) return false;
        }
        return true;
    }
};
}  // namespace

LoadMeshErr FSolver::LoadMesh(bool deleteFiles)
{
    if (meshLoadedFromPrevSolution) return NOERROR;   // fsolver.cpp:357-360
    LoadTrace tr;
    char s[1024];
    std::string infile = PathName + ".node";
    TextBuf tb;
    {   // one buffer for the three mesh files: the largest one's size
        struct stat st;
        for (const char *ext : {".node", ".ele", ".edge"})
            if (::stat((PathName + ext).c_str(), &st) == 0) tb.hint = std::max(tb.hint, (size_t)st.st_size + 1);
    }
    if (!tb.load(infile)) return BADNODEFILE;
    tr.mark("  .node read");
    int k = 0, j = 0;
    if (!tb.header_int(k)) return BADNODEFILE;
    NumNodes = k;
    par_assign(meshnode, (size_t)std::max(0, k), CNode());
    const double conv = 100 * kLengthConvMeters[LengthUnits];
    if (!tb.records(k, [&](const char *&p, int i, bool nl) {
            int a, m;
            CNode &node = meshnode[i];
            if (!read_int(p, a, nl) || !read_double(p, node.x, nl) || !read_double(p, node.y, nl) ||
                !read_int(p, m, nl))
                return false;
            node.BoundaryMarker = (m > 1) ? m - 2 : -1;
            node.x *= conv;   // lengths in cm (fsolver.cpp:386-388)
            node.y *= conv;
            return true;
        }))
        return BADNODEFILE;
    if (tr.on) std::fprintf(stderr, "[load]   (record count pass %.1f ms)\n", tb.ms_count);
    tr.mark("nodes");

    infile = PathName + ".pbc";
    FILE *fp = fopen(infile.c_str(), "rt");
    if (!fp) return BADPBCFILE;
    NumPBCs = 0;
    if (fgets(s, 1024, fp)) sscanf(s, "%i", &NumPBCs);
    pbclist.clear();
    for (int i = 0; i < NumPBCs; i++) {
        CCommonPoint pbc;
        if (!fgets(s, 1024, fp) || sscanf(s, "%i %i %i %i", &j, &pbc.x, &pbc.y, &pbc.t) != 4) {
            fclose(fp);
            return BADPBCFILE;
        }
        pbclist.push_back(pbc);
    }
    // air-gap elements: name, parameter line, totalArcElements + 1 quadNodes
    NumAirGapElems = 0;
    if (fgets(s, 1024, fp)) sscanf(s, "%i", &NumAirGapElems);
    agelist.clear();
    for (int i = 0; i < NumAirGapElems; i++) {
        AirGap g;
        bool ok = fgets(s, 1024, fp) != nullptr;
        g.name = s;
        ok = ok && fgets(s, 1024, fp) &&
             sscanf(s, "%i %lf %lf %lf %lf %lf %lf %lf %i %lf %lf", &g.format, &g.inner_angle, &g.outer_angle,
                    &g.ri, &g.ro, &g.arc, &g.agc_re, &g.agc_im, &g.n_arc, &g.inner_shift, &g.outer_shift) == 11;
        ok = ok && g.n_arc > 0;
        for (int k = 0; ok && k <= g.n_arc; k++) {
            int n[4];
            double w[4];
            ok = fgets(s, 1024, fp) && sscanf(s, "%i %lf %i %lf %i %lf %i %lf", &n[0], &w[0], &n[1], &w[1], &n[2],
                                              &w[2], &n[3], &w[3]) == 8;
            for (int m = 0; ok && m < 4; m++) {
                ok = n[m] >= 0 && n[m] < NumNodes;   // negative quadNode: the reference rejects the file too
                g.qn.push_back(n[m]);
                g.qw.push_back(w[m]);
            }
        }
        if (!ok) {
            fclose(fp);
            return BADPBCFILE;
        }
        agelist.push_back(g);
    }
    fclose(fp);

    infile = PathName + ".ele";
    if (!tb.load(infile)) return BADELEMENTFILE;
    tr.mark("  .ele read");
    if (!tb.header_int(k)) return BADELEMENTFILE;
    NumEls = k;
    par_assign(meshele, (size_t)std::max(0, k), CMElement());
    tr.mark("  element array");
    int defaultLabel = -1;
    for (int i = 0; i < (int)labellist.size(); i++)
        if (labellist[i].IsDefault) defaultLabel = i;
    auto remove_files = [&]() {
        for (const char *ext : {".ele", ".node", ".pbc", ".poly", ".edge"}) remove((PathName + ext).c_str());
    };
    if (!tb.records(k, [&](const char *&p, int i, bool nl) {
            int a;
            CMElement &elm = meshele[i];
            return read_int(p, a, nl) && read_int(p, elm.p[0], nl) && read_int(p, elm.p[1], nl) &&
                   read_int(p, elm.p[2], nl) && read_int(p, elm.lbl, nl);
        }))
        return BADELEMENTFILE;
    if (tr.on) std::fprintf(stderr, "[load]   (record count pass %.1f ms)\n", tb.ms_count);
    tr.mark("  element records");
    {
        // labels and node ids checked per element, in parallel; the first
        // failing element (in file order) decides the error, as the
        // reference's sequential loop does (fsolver.cpp:593-626)
        const int nl = (int)labellist.size();
        const int T = 64;
        std::vector<int> bad_at(T, -1), bad_code(T, 0);
        par_for(T, 1, [&](long long t0, long long t1) {
            for (long long t = t0; t < t1; ++t) {
                const int a = (int)((long long)k * t / T), b = (int)((long long)k * (t + 1) / T);
                for (int i = a; i < b; i++) {
                    CMElement &elm = meshele[i];
                    elm.lbl--;
                    if (elm.lbl < 0) elm.lbl = defaultLabel;
                    int code = 0;
                    if (elm.lbl < 0) code = 1;
                    else if (elm.lbl >= nl) code = 2;
                    else
                        for (int q = 0; q < 3; q++)
                            if (elm.p[q] < 0 || elm.p[q] >= NumNodes) code = 3;
                    if (code) {
                        bad_at[t] = i;
                        bad_code[t] = code;
                        break;
                    }
                    elm.blk = labellist[elm.lbl].BlockType;
                }
            }
        });
        for (int t = 0; t < T; ++t) {
            if (bad_at[t] < 0) continue;
            const int i = bad_at[t];
            if (bad_code[t] == 1) {
                char buf[256];
                snprintf(buf, sizeof buf, "The element number %i had label %i\n", i, meshele[i].lbl);
                warn(std::string("Material properties have not been defined for all regions.\n") + buf);
                if (deleteFiles) remove_files();
                return MISSINGMATPROPS;
            }
            if (bad_code[t] == 2) {
                if (deleteFiles) remove_files();
                return ELMLABELTOOBIG;
            }
            return BADELEMENTFILE;
        }
    }
    tr.mark("elements");

    infile = PathName + ".edge";
    if (!tb.load(infile)) return BADEDGEFILE;
    tr.mark("  .edge read");
    int nedge = 0, flag = 0;
    if (!tb.next_int(nedge) || !tb.next_int(flag)) return BADEDGEFILE;
    par_assign(edges_, (size_t)std::max(0, nedge), std::array<int, 3>{0, 0, 0});
    if (nedge > 0 && !tb.records(nedge, [&](const char *&p, int i, bool nl) {
            int a;
            auto &e = edges_[i];
            return read_int(p, a, nl) && read_int(p, e[0], nl) && read_int(p, e[1], nl) && read_int(p, e[2], nl);
        }))
        return BADEDGEFILE;
    if (tr.on) std::fprintf(stderr, "[load]   (record count pass %.1f ms)\n", tb.ms_count);
    tr.mark("edge records");
    // boundary-marked edges (marker < 0) set the boundary property of the
    // element sides they match (fsolver.cpp:660-704: per edge, every element
    // around its first node whose side k joins the two nodes).  The last such
    // edge in file order wins a side, so the side takes the property of the
    // last marked edge with its node pair: a map from the (unordered) pair,
    // filled in file order, looked up per element side in parallel -- no
    // node -> element membership lists
    {
        const int T = 64;
        std::vector<char> bad(T, 0);
        std::vector<std::vector<int>> marked(T);
        par_for(T, 1, [&](long long t0, long long t1) {
            for (long long t = t0; t < t1; ++t) {
                const int a = (int)((long long)nedge * t / T), b = (int)((long long)nedge * (t + 1) / T);
                for (int i = a; i < b; i++) {
                    const auto &e = edges_[i];
                    if (e[0] < 0 || e[1] < 0 || e[0] >= NumNodes || e[1] >= NumNodes) {
                        bad[t] = 1;
                        break;
                    }
                    if (e[2] < 0) marked[t].push_back(i);
                }
            }
        });
        for (char c : bad)
            if (c) return BADEDGEFILE;
        std::unordered_map<unsigned long long, int> side_bc;
        std::vector<char> on_marked(NumNodes, 0);
        auto pair_key = [](int a, int b) {
            return ((unsigned long long)(unsigned)std::min(a, b) << 32) | (unsigned)std::max(a, b);
        };
        for (auto &m : marked)
            for (int i : m) {
                const auto &e = edges_[i];
                side_bc[pair_key(e[0], e[1])] = -(e[2] + 2);
                on_marked[e[0]] = on_marked[e[1]] = 1;
            }
        if (!side_bc.empty())
            par_for(NumEls, 1 << 15, [&](long long a, long long b) {
                for (long long i = a; i < b; i++) {
                    CMElement &el = meshele[i];
                    for (int q = 0; q < 3; q++) {
                        const int n0 = el.p[q], n1 = el.p[(q + 1) % 3];
                        if (!on_marked[n0] || !on_marked[n1]) continue;
                        auto it = side_bc.find(pair_key(n0, n1));
                        if (it != side_bc.end()) el.e[q] = it->second;
                    }
                }
            });
    }
    tr.mark("edges");
    if (deleteFiles) remove_async({PathName + ".ele", PathName + ".node", PathName + ".pbc", PathName + ".poly"});
    return NOERROR;
}

namespace {
// one run of comb-sort compare-swaps x[i] <-> y[i] (score = high 32 bits,
// swap on a strict decrease); x and y do not overlap.  Branch-free: a wide
// pass meets random data, whose swaps mispredict half the time.  Returns
// nonzero when anything moved.
__attribute__((target("avx2"))) unsigned long long comb_swap_run_avx2(unsigned long long *__restrict x,
                                                                       unsigned long long *__restrict y, int n)
{
    __m256i anyv = _mm256_setzero_si256();
    int i = 0;
    for (; i + 4 <= n; i += 4) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(x + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(y + i));
        // (scores < 2^32: the signed 64-bit compare of the shifted keys is the unsigned one)
        const __m256i m = _mm256_cmpgt_epi64(_mm256_srli_epi64(a, 32), _mm256_srli_epi64(b, 32));
        _mm256_storeu_si256(reinterpret_cast<__m256i *>(x + i), _mm256_blendv_epi8(a, b, m));
        _mm256_storeu_si256(reinterpret_cast<__m256i *>(y + i), _mm256_blendv_epi8(b, a, m));
        anyv = _mm256_or_si256(anyv, m);
    }
    unsigned long long any = (unsigned long long)_mm256_movemask_epi8(anyv);
    for (; i < n; ++i) {
        const unsigned long long a = x[i], b = y[i];
        const unsigned long long m = 0ULL - (unsigned long long)((a >> 32) > (b >> 32));
        x[i] = (a & ~m) | (b & m);
        y[i] = (b & ~m) | (a & m);
        any |= m;
    }
    return any;
}
unsigned long long comb_swap_run_plain(unsigned long long *__restrict x, unsigned long long *__restrict y, int n)
{
    unsigned long long any = 0;
    for (int i = 0; i < n; ++i) {
        const unsigned long long a = x[i], b = y[i];
        const unsigned long long m = 0ULL - (unsigned long long)((a >> 32) > (b >> 32));
        x[i] = (a & ~m) | (b & m);
        y[i] = (b & ~m) | (a & m);
        any |= m;
    }
    return any;
}
unsigned long long comb_swap_run(unsigned long long *x, unsigned long long *y, int n)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    return avx2 ? comb_swap_run_avx2(x, y, n) : comb_swap_run_plain(x, y, n);
}

// Narrow comb passes as scans (see SortElements).  op(c, x): the carried
// entry c stays only on a strictly greater score; the all-zero key (score 0)
// is its identity from the left, so a class's first entry needs no special
// case.  Rows of g positions: lane c of a row is class c.
inline unsigned long long scan_op(unsigned long long c, unsigned long long x)
{
    const unsigned long long m = 0ULL - (unsigned long long)((c >> 32) > (x >> 32));
    return (c & m) | (x & ~m);
}
// red[c] = op(red[c], key[r g + c]) over `rows` rows
__attribute__((target("avx2"))) void scan_reduce_avx2(unsigned long long *red, const unsigned long long *key,
                                                       long long rows, int g)
{
    int c = 0;
    for (; c + 4 <= g; c += 4) {
        __m256i r = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(red + c));
        const unsigned long long *k = key + c;
        for (long long i = 0; i < rows; ++i, k += g) {
            const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(k));
            const __m256i m = _mm256_cmpgt_epi64(_mm256_srli_epi64(r, 32), _mm256_srli_epi64(x, 32));
            r = _mm256_blendv_epi8(x, r, m);
        }
        _mm256_storeu_si256(reinterpret_cast<__m256i *>(red + c), r);
    }
    for (; c < g; ++c) {
        unsigned long long r = red[c];
        const unsigned long long *k = key + c;
        for (long long i = 0; i < rows; ++i, k += g) r = scan_op(r, *k);
        red[c] = r;
    }
}
// car[c] = op(car[c], key[r g + c]) = c_k; out[r g + c] = the smaller-score of
// c_k and key[(r + 1) g + c] (c_k on ties) -- `rows` rows, each with its
// next row present; returns nonzero when some position took the next entry
__attribute__((target("avx2"))) unsigned long long scan_rows_avx2(unsigned long long *car,
                                                                   const unsigned long long *key,
                                                                   unsigned long long *out, long long rows, int g)
{
    unsigned long long any = 0;
    int c = 0;
    __m256i anyv = _mm256_setzero_si256();
    for (; c + 4 <= g; c += 4) {
        __m256i cv = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(car + c));
        const unsigned long long *k = key + c;
        unsigned long long *o = out + c;
        for (long long i = 0; i < rows; ++i, k += g, o += g) {
            const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(k));
            const __m256i nx = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(k + g));
            const __m256i m0 = _mm256_cmpgt_epi64(_mm256_srli_epi64(cv, 32), _mm256_srli_epi64(x, 32));
            cv = _mm256_blendv_epi8(x, cv, m0);
            const __m256i m = _mm256_cmpgt_epi64(_mm256_srli_epi64(cv, 32), _mm256_srli_epi64(nx, 32));
            _mm256_storeu_si256(reinterpret_cast<__m256i *>(o), _mm256_blendv_epi8(cv, nx, m));
            anyv = _mm256_or_si256(anyv, m);
        }
        _mm256_storeu_si256(reinterpret_cast<__m256i *>(car + c), cv);
    }
    any = (unsigned long long)_mm256_movemask_epi8(anyv);
    for (; c < g; ++c) {
        unsigned long long cc = car[c];
        const unsigned long long *k = key + c;
        unsigned long long *o = out + c;
        for (long long i = 0; i < rows; ++i, k += g, o += g) {
            cc = scan_op(cc, *k);
            const unsigned long long nx = k[g];
            const unsigned long long m = 0ULL - (unsigned long long)((cc >> 32) > (nx >> 32));
            *o = (nx & m) | (cc & ~m);
            any |= m;
        }
        car[c] = cc;
    }
    return any;
}
void scan_reduce_plain(unsigned long long *red, const unsigned long long *key, long long rows, int g)
{
    for (int c = 0; c < g; ++c) {
        unsigned long long r = red[c];
        const unsigned long long *k = key + c;
        for (long long i = 0; i < rows; ++i, k += g) r = scan_op(r, *k);
        red[c] = r;
    }
}
unsigned long long scan_rows_plain(unsigned long long *car, const unsigned long long *key, unsigned long long *out,
                                   long long rows, int g)
{
    unsigned long long any = 0;
    for (int c = 0; c < g; ++c) {
        unsigned long long cc = car[c];
        const unsigned long long *k = key + c;
        unsigned long long *o = out + c;
        for (long long i = 0; i < rows; ++i, k += g, o += g) {
            cc = scan_op(cc, *k);
            const unsigned long long nx = k[g];
            const unsigned long long m = 0ULL - (unsigned long long)((cc >> 32) > (nx >> 32));
            *o = (nx & m) | (cc & ~m);
            any |= m;
        }
        car[c] = cc;
    }
    return any;
}
void scan_reduce(unsigned long long *red, const unsigned long long *key, long long rows, int g)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2 && g >= 4) scan_reduce_avx2(red, key, rows, g);
    else scan_reduce_plain(red, key, rows, g);
}
unsigned long long scan_rows(unsigned long long *car, const unsigned long long *key, unsigned long long *out,
                             long long rows, int g)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    return (avx2 && g >= 4) ? scan_rows_avx2(car, key, out, rows, g) : scan_rows_plain(car, key, out, rows, g);
}
}  // namespace

// meshele[k] = the old meshele[src(k)]: a second element array copy-constructed
// in parallel (no serial value-initialisation), then swapped in
template <class Src>
bool FSolver::permute_elements(Src src)
{
    BigVec<CMElement> out;
    huge_reserve(out, (size_t)std::max(0, NumEls));
    out.resize((size_t)std::max(0, NumEls));   // (NoInitAlloc: written below, in parallel)
    par_for(NumEls, 1 << 16, [&](long long a, long long b) {
        // (the sources are scattered: each 40-B record is a cache miss, so the
        // one kPf ahead is requested while this one is copied)
        constexpr long long kPf = 16;
        for (long long k = a; k < b; k++) {
            if (k + kPf < b) __builtin_prefetch(&meshele[src(k + kPf)], 0, 0);
            ::new (&out[k]) CMElement(meshele[src(k)]);
        }
    });
    meshele.swap(out);
    static_assert(std::is_trivially_destructible<CMElement>::value, "uninitialised storage");
    return true;
}

int FSolver::SortElements()
{
    // comb sort on p0+p1+p2 (cuthill.cpp:39-86); not stable, restated exactly:
    // the same comparisons and swaps, on packed (score, element) keys instead
    // of the element records, which are permuted once at the end.  With a
    // GPU (the solve needs one anyway) every pass runs on the device
    // (xfk_sort_elements: ~2 ms instead of ~45 on 16 host cores); without
    // one, or with XFEMM_HOST_SORT set, on the host below.
    LoadTrace tr;
    join_hip_warmup();
    if (NumEls > 1 && !std::getenv("XFEMM_HOST_SORT") && xfk_device_count() > 0) {
        HugeBuf<unsigned> score;
        HugeBuf<int> perm;
        if (!score.allocate((size_t)NumEls) || !perm.allocate((size_t)NumEls)) return false;
        par_for(NumEls, 1 << 16, [&](long long a, long long b) {
            for (long long k = a; k < b; k++) {
                const CMElement &e = meshele[k];
                score[k] = (unsigned)((long long)e.p[0] + e.p[1] + e.p[2]);
            }
        });
        if (xfk_sort_elements(NumEls, score.data(), device, perm.data()) != XFK_OK) {
            warn(std::string("device element sort failed: ") + xfk_last_error() + "\n");
            return false;
        }
        tr.mark("  device comb sort");
        permute_elements([&](long long k) { return perm[k]; });
        tr.mark("  permute");
        return true;
    }
    std::vector<unsigned long long> key, tmp;
    huge_reserve(key, (size_t)NumEls);
    huge_reserve(tmp, (size_t)NumEls);
    key.resize(NumEls);
    par_for(NumEls, 1 << 16, [&](long long a, long long b) {
        for (long long k = a; k < b; k++) {
            const CMElement &e = meshele[k];
            const unsigned long long sc = (unsigned long long)((long long)e.p[0] + e.p[1] + e.p[2]);
            key[k] = (sc << 32) | (unsigned)k;
        }
    });
    // A pass with gap g compares (j, j + g) for j ascending: the steps of one
    // residue class j mod g touch only that class's entries, in ascending
    // order, so classes are independent.  Wide passes split the classes over
    // threads.  Narrow passes (few classes) use that a pass over one class is
    // a bubble pass: the element carried to position k is the prefix
    // "maximum" c_k = op(c_{k-1}, x_k), op(a, b) = score(a) > score(b) ? a : b
    // (a swap happens exactly when the carried score exceeds the next one:
    // ties keep their order), and position k receives
    // score(c_k) > score(x_{k+1}) ? x_{k+1} : c_k -- an associative scan, so
    // chunks of rows run in parallel from their classes' carries (computed
    // from per-chunk reductions): out of place, the same result as the
    // sequential pass
    HostPool &pool = HostPool::get();
    const int T = pool.size();
    auto scan_pass = [&](int g) -> bool {
        // chunks of whole rows (g positions each); every chunk but the last
        // holds every class, so the carries need no presence flags
        const long long n = NumEls;
        const long long R = (n + g - 1) / g;
        const int TT = (int)std::max<long long>(1, std::min<long long>(T, R / 64));
        std::vector<long long> q0(TT + 1);
        for (int t = 0; t <= TT; ++t) q0[t] = std::min(n, (R * t / TT) * g);
        std::vector<unsigned long long> red((size_t)TT * g), cin((size_t)TT * g);
        std::vector<char> sw(TT, 0);
        auto run = [&](auto fn) { pool.run(TT, fn); };
        run([&](int t) {   // per chunk and class: the op-reduction of its entries (from the identity 0)
            if (t == TT - 1) return;   // (the last chunk feeds no carry; the others are whole rows)
            unsigned long long *rd = red.data() + (size_t)t * g;
            std::fill(rd, rd + g, 0ULL);
            scan_reduce(rd, key.data() + q0[t], (q0[t + 1] - q0[t]) / g, g);
        });
        for (int t = 1; t < TT; ++t)   // carries into each chunk
            for (int c = 0; c < g; ++c) {
                const size_t i1 = (size_t)(t - 1) * g + c, i2 = (size_t)t * g + c;
                cin[i2] = t == 1 ? red[i1] : scan_op(cin[i1], red[i1]);
            }
        tmp.resize(NumEls);
        run([&](int t) {
            const long long a = q0[t], e = q0[t + 1];
            if (a >= e) return;
            std::vector<unsigned long long> car(g, 0ULL);   // chunk 0: the identity
            if (t > 0) std::copy(cin.begin() + (size_t)t * g, cin.begin() + (size_t)(t + 1) * g, car.begin());
            // whole rows whose next row is complete, then position by position
            const long long full = std::max(0LL, std::min((e - a) / g, (n - g - a) / g));
            unsigned long long any = scan_rows(car.data(), key.data() + a, tmp.data() + a, full, g);
            int c = 0;
            long long q = a + full * g;
            const long long lim = std::min(e, n - g);   // positions with a partner one gap on
            for (; q < lim; ++q) {
                const unsigned long long cc = scan_op(car[c], key[q]);   // c_k
                car[c] = cc;
                const unsigned long long nx = key[q + g];                 // x_{k+1}
                const unsigned long long m = 0ULL - (unsigned long long)((cc >> 32) > (nx >> 32));
                tmp[q] = (nx & m) | (cc & ~m);
                any |= m;
                if (++c == g) c = 0;
            }
            for (; q < e; ++q) {   // the last g positions: the carried entry lands
                tmp[q] = scan_op(car[c], key[q]);
                if (++c == g) c = 0;
            }
            sw[t] = any != 0;
        });
        key.swap(tmp);
        bool any = false;
        for (char c : sw) any |= c != 0;
        return any;
    };
    int gap = NumEls, i = 0;
    double ms_wide = 0, ms_narrow = 0;
    int n_wide = 0, n_narrow = 0;
    do {
        const auto tp = std::chrono::steady_clock::now();
        if (gap > 1) {
            gap = (gap * 10) / 13;
            if ((gap == 10) || (gap == 9)) gap = 11;
        }
        i = 0;
        if (T > 1 && gap >= 8 * T && NumEls >= (1 << 16)) {
            std::vector<char> sw(T, 0);
            const int g = gap;
            auto part = [&](int t) {
                const int r0 = (int)((long long)g * t / T), r1 = (int)((long long)g * (t + 1) / T);
                unsigned long long any = 0;
                for (long long b = 0; b + g < NumEls; b += g) {
                    // (the class range [r0, r1) of this block and its partners one gap on:
                    // disjoint, so the compare-swaps are independent -- branch-free)
                    const int re = (int)std::min<long long>(r1, NumEls - g - b);
                    any |= comb_swap_run(key.data() + b + r0, key.data() + b + r0 + g, re - r0);
                }
                sw[t] = any != 0;
            };
            pool.run(T, part);
            for (char c : sw) i |= c;
        } else if (T > 1 && NumEls >= (1 << 16)) {   // (narrow passes: few classes)
            i = scan_pass(gap) ? 1 : 0;
        } else {
            for (int j = 0; (j + gap) < NumEls; j++) {
                if ((key[j] >> 32) > (key[j + gap] >> 32)) {
                    std::swap(key[j], key[j + gap]);
                    i = 1;
                }
            }
        }
        const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
        if (T > 1 && gap >= 8 * T && NumEls >= (1 << 16)) ms_wide += dt, ++n_wide;
        else ms_narrow += dt, ++n_narrow;
    } while ((gap > 1) && (i > 0));
    if (tr.on)
        std::fprintf(stderr, "[load]   comb passes: %d wide %.1f ms, %d narrow %.1f ms\n", n_wide, ms_wide, n_narrow,
                     ms_narrow);
    tr.mark("  comb sort");
    // the permutation applied through a second element array (permute_elements)
    if (!permute_elements([&](long long k) { return (int)(key[k] & 0xffffffffu); })) return false;
    tr.mark("  permute");
    return true;
}

int FSolver::Cuthill(bool deleteFiles)
{
    // reverse-less Cuthill-McKee of cuthill.cpp:88-390, on the .edge connectivity
    LoadTrace tr;
    const int n_lines = (int)edges_.size();
    BigVec<int> numcon, newnum, nxtnum;
    par_assign(numcon, (size_t)NumNodes, 0);
    par_assign(newnum, (size_t)NumNodes, -1);
    par_assign(nxtnum, (size_t)NumNodes, -1);
    // neighbour lists as CSR, each in the order the reference's lists get
    // their entries (edge order).  Thread t takes the edges of its range and
    // bins both ends by the node range that owns them (bucket (t, u)); owner u
    // then reads its buckets in t order -- every list in edge order, as the
    // sequential loop appends it -- counts, scans and fills its own nodes.
    // The edge array is read twice in all (not once per thread).
    BigVec<int> aptr, adj;
    par_assign(aptr, (size_t)NumNodes + 1, 0);
    huge_reserve(adj, 2 * edges_.size());
    adj.resize(2 * edges_.size());   // (every slot written by the fill below)
    {
        const int T = (int)std::max<long long>(1, std::min<long long>(HostPool::get().size(), (long long)n_lines / 65536));
        const int chunk = (int)std::max<long long>(1, ((long long)NumNodes + T - 1) / T);
        auto lo = [&](int u) { return (int)std::min<long long>(NumNodes, (long long)chunk * u); };
        auto elo = [&](int t) { return (long long)n_lines * t / T; };
        std::vector<long long> bc((size_t)T * T + 1, 0);   // bucket (t, u) at t * T + u: ends counted, then offsets
        par_for(T, 1, [&](long long t0, long long t1) {
            for (long long t = t0; t < t1; ++t) {
                long long *c = bc.data() + t * T;
                for (long long i = elo((int)t); i < elo((int)t + 1); ++i) {
                    c[edges_[i][0] / chunk]++;
                    c[edges_[i][1] / chunk]++;
                }
            }
        });
        // layout: owner u's region holds its buckets t = 0 .. T-1 in order
        std::vector<long long> off((size_t)T * T), ubase(T + 1, 0);
        long long o = 0;
        for (int u = 0; u < T; ++u) {
            ubase[u] = o;
            for (int t = 0; t < T; ++t) {
                off[(size_t)t * T + u] = o;
                o += bc[(size_t)t * T + u];
            }
        }
        ubase[T] = o;
        BigVec<std::array<int, 2>> ends;   // (owned end, other end)
        huge_reserve(ends, (size_t)o);
        ends.resize((size_t)o);
        par_for(T, 1, [&](long long t0, long long t1) {
            for (long long t = t0; t < t1; ++t) {
                long long *w = off.data() + t * T;
                for (long long i = elo((int)t); i < elo((int)t + 1); ++i) {
                    const int e0 = edges_[i][0], e1 = edges_[i][1];
                    ends[w[e0 / chunk]++] = {e0, e1};
                    ends[w[e1 / chunk]++] = {e1, e0};
                }
            }
        });
        par_for(T, 1, [&](long long u0, long long u1) {
            for (long long u = u0; u < u1; ++u) {
                for (long long k = ubase[u]; k < ubase[u + 1]; ++k) numcon[ends[k][0]]++;
                long long q = ubase[u];   // (= the ends owned by the ranges before u)
                for (int v = lo((int)u); v < lo((int)u + 1); ++v) {
                    aptr[v] = (int)q;
                    q += numcon[v];
                }
                std::vector<int> cur(aptr.begin() + lo((int)u), aptr.begin() + lo((int)u + 1));
                for (long long k = ubase[u]; k < ubase[u + 1]; ++k) adj[cur[ends[k][0] - lo((int)u)]++] = ends[k][1];
            }
        });
        aptr[NumNodes] = (int)ubase[T];
    }
    if (deleteFiles) remove_async({PathName + ".edge"});
    tr.mark("adjacency");
    // bubble sort by increasing connectivity: swaps only on a strict decrease,
    // so it is the stable sort of the list by numcon -- an insertion sort per
    // list gives the same order; lists are independent
    par_for(NumNodes, 1 << 14, [&](long long a, long long b) {
        for (long long n0 = a; n0 < b; n0++) {
            int *l = adj.data() + aptr[n0];
            const int m = aptr[n0 + 1] - aptr[n0];
            for (int q = 1; q < m; q++) {
                const int v = l[q], kv = numcon[v];
                int r = q;
                for (; r > 0 && numcon[l[r - 1]] > kv; --r) l[r] = l[r - 1];
                l[r] = v;
            }
        }
    });
    tr.mark("neighbour sort");
    long long j = numcon[0];
    int n0 = 0;
    for (long long i = 1; i < NumNodes; i++) {
        if (numcon[i] < j) {
            j = numcon[i];
            n0 = (int)i;
        }
        if (j == 2) i = n_lines;
    }
    newnum[n0] = 0;
    int n = 1;
    nxtnum[0] = n0;
    if (NumNodes > 1) {
        do {
            for (int t = aptr[n0]; t < aptr[n0 + 1]; ++t)
                if (const int c = adj[t]; newnum[c] < 0) {
                    newnum[c] = n;
                    nxtnum[n] = c;
                    n++;
                }
            const int nextpos = newnum[n0] + 1;
            if (nextpos >= NumNodes || nxtnum[nextpos] < 0) {
                if (n >= NumNodes) break;
                for (int i = 0; i < NumNodes; i++)
                    if (newnum[i] < 0) {
                        j = numcon[i];
                        n0 = i;
                        break;
                    }
                for (int i = 0; i < NumNodes; i++) {
                    if ((newnum[i] < 0) && (numcon[i] < j)) {
                        j = numcon[i];
                        n0 = i;
                    }
                    if (j == 2) break;
                }
                newnum[n0] = n;
                nxtnum[n] = n0;
                n++;
            } else {
                n0 = nxtnum[nextpos];
            }
        } while (n < NumNodes);
    }
    tr.mark("numbering");
    for (auto &p : pbclist) {
        p.x = newnum[p.x];
        p.y = newnum[p.y];
    }
    for (auto &g : agelist)   // cuthill.cpp:321-330
        for (int &q : g.qn) q = newnum[q];
    int newwide = 0;
    {
        std::mutex mu;
        par_for(NumNodes, 1 << 16, [&](long long a0, long long a1) {
            int w = 0;
            for (long long a = a0; a < a1; a++)
                for (int t = aptr[a]; t < aptr[a + 1]; ++t) w = std::max(w, std::abs(newnum[a] - newnum[adj[t]]));
            std::lock_guard<std::mutex> g(mu);
            newwide = std::max(newwide, w);
        });
    }
    BandWidth = newwide + 1;
    par_for(NumEls, 1 << 16, [&](long long a, long long b) {
        for (long long k = a; k < b; k++)
            for (int q = 0; q < 3; q++) meshele[k].p[q] = newnum[meshele[k].p[q]];
    });
    // SortNodes (fsolver.cpp:1341-1353): node i moves to slot newnum[i]
    BigVec<CNode> sorted;
    huge_reserve(sorted, (size_t)NumNodes);
    sorted.resize(NumNodes);   // (every slot written below: newnum is a permutation)
    par_for(NumNodes, 1 << 16, [&](long long a, long long b) {
        for (long long k = a; k < b; k++) ::new (&sorted[newnum[k]]) CNode(meshnode[k]);
    });
    meshnode.swap(sorted);
    tr.mark("bandwidth + renumber");
    SortElements();
    tr.mark("SortElements");
    return true;
}

void FSolver::GetFillFactor(int lbl)
{
    // bIsWound, and at AC the proximity-effect permeability of a wound
    // LamType > 2 region (fsolver.cpp:1083-1193): an equivalent-foil model for
    // rectangular wire, a fitted frequency-dependent permeability for round
    // wire (magnet, stranded, litz, copper-clad aluminium)
    CMBlockLabel &bl = labellist[lbl];
    const int lt = (bl.BlockType >= 0) ? blockproplist[bl.BlockType].LamType : 0;
    bl.bIsWound = (std::abs(bl.Turns) > 1) || (lt > 2);
    bl.ProxMu_re = 1;
    bl.ProxMu_im = 0;
    if (Frequency == 0 || lt < 3) return;
    // the region's area, m^2 (ElmArea, fsolver.cpp:1196-1210)
    double atot = 0;
    for (const auto &el : meshele) {
        if (el.lbl != lbl) continue;
        const CNode &a = meshnode[el.p[0]], &b = meshnode[el.p[1]], &c = meshnode[el.p[2]];
        const double b0 = b.y - c.y, b1 = c.y - a.y, c0 = c.x - b.x, c1 = a.x - c.x;
        atot += 0.0001 * (b0 * c1 - b1 * c0) / 2.;
    }
    if (atot == 0) return;   // ProximityMu keeps its previous value (1 here)
    const CMSolverMaterialProp &bp = blockproplist[bl.BlockType];
    if (bp.Cduct == 0) return;
    using cd = std::complex<double>;
    const cd I(0, 1);
    const double muo = 4.e-7 * kPi;
    const int wiretype = lt - 3;
    cd mu;
    if (wiretype == 3) {   // rectangular wire: equivalent foil
        const double W = 2. * kPi * Frequency, d = bp.WireD * 0.001;
        double fill = std::fabs(d * d * (double)bl.Turns / atot);
        const double pitch = d / std::sqrt(fill);
        fill = d / pitch;
        const double o = bp.Cduct * fill * 1.e6;
        const cd k = std::sqrt(I * W * o * muo) * d / 2.;
        const cd ufd = muo * std::tanh(k) / k;
        mu = (fill * ufd + (1. - fill) * muo) / muo;
    } else {
        double R = 0, awire = 0;
        const double turns = (double)bl.Turns, ns = (double)bp.NStrands;
        if (wiretype == 0 || wiretype == 2) {   // magnet wire, litz: NStrands strands of WireD
            R = bp.WireD * 0.0005;
            awire = kPi * R * R * ns * turns;
        } else if (wiretype == 1) {             // stranded, non-litz: one conductor of the bundle's area
            R = bp.WireD * 0.0005 * std::sqrt(ns);
            awire = kPi * R * R * turns;
        }                                       // CCA (4, 5): the reference leaves R and awire at 0
        const double fill = std::fabs(awire / atot);
        const double W = 2. * kPi * Frequency * bp.Cduct * 1.e6 * muo * R * R / 2.;
        double c1 = 0, c2 = 0;
        if (wiretype <= 2) {
            c1 = 0.7756067409818643 + fill * (0.6873854335408803 + fill * (0.06841584481674128 - 0.07143732702512284 * fill));
            c2 = 1.5 * fill / c1;
        } else if (wiretype == 4) {
            c1 = 0.7270741505617485 + 0.8902950067721367 * fill + 0.11894736885885195 * fill * fill -
                 0.12247276254503957 * fill * fill * fill;
            c2 = 0.006784920229549677 + 1.8942880489198526 * fill - 1.3631438759519217 * fill * fill +
                 0.504431701685587 * fill * fill * fill;
        } else if (wiretype == 5) {
            c1 = 0.7486913529860821 + 0.9042845510838825 * fill + 0.1361040321433224 * fill * fill -
                 0.10652380745682069 * fill * fill * fill;
            c2 = 0.006790468527313965 + 1.8945509985370095 * fill - 1.3643501010185972 * fill * fill +
                 0.5036765577982594 * fill * fill * fill;
        }
        const cd z = std::sqrt(c1 * I * W);
        mu = c2 * (std::tanh(z) / z) + (1. - c2);
    }
    bl.ProxMu_re = mu.real();
    bl.ProxMu_im = mu.imag();
}

// the C-ABI descriptor of the current problem and the arrays it points into
struct FSolver::DescStore {
    std::vector<xfk_block_desc> blk;
    std::vector<xfk_label_desc> lab;
    std::vector<xfk_line_desc> lin;
    std::vector<xfk_point_desc> pts;
    std::vector<xfk_circuit_desc> cir;
    std::vector<double> x, y;
    std::vector<int> marker, p, e, lbl, pbc;
    std::vector<xfk_age_desc> age;
    xfk_problem_desc d{};
};

bool FSolver::make_desc(DescStore &ds)
{
    for (int i = 0; i < (int)labellist.size(); i++) GetFillFactor(i);
    ds.blk.resize(blockproplist.size());
    for (size_t k = 0; k < blockproplist.size(); k++) {
        const CMSolverMaterialProp &m = blockproplist[k];
        xfk_block_desc &d = ds.blk[k];
        d.mu_x = m.mu_x; d.mu_y = m.mu_y; d.H_c = m.H_c; d.J_re = m.J_re; d.Cduct = m.Cduct;
        d.LamFill = m.LamFill; d.LamType = m.LamType; d.BHpoints = m.BHpoints;
        d.B = m.Bdata.empty() ? nullptr : m.Bdata.data();
        d.H = m.Hdata.empty() ? nullptr : m.Hdata.data();
        d.slope = m.slope.empty() ? nullptr : m.slope.data();
    }
    if (ds.blk.empty()) {
        warn("no block properties defined\n");
        return false;
    }
    ds.lab.resize(labellist.size());
    for (size_t k = 0; k < labellist.size(); k++) {
        ds.lab[k].block = labellist[k].BlockType >= 0 ? labellist[k].BlockType : 0;
        ds.lab[k].in_circuit = labellist[k].InCircuit;
        ds.lab[k].mag_dir = labellist[k].MagDir;
        ds.lab[k].is_wound = labellist[k].bIsWound ? 1 : 0;
        ds.lab[k].is_external = labellist[k].IsExternal ? 1 : 0;
        ds.lab[k].mag_dir_fctn = labellist[k].MagDirFctn.empty() ? nullptr : labellist[k].MagDirFctn.c_str();
    }
    ds.lin.resize(lineproplist.size());
    for (size_t k = 0; k < lineproplist.size(); k++) {
        const CMBoundaryProp &b = lineproplist[k];
        ds.lin[k] = xfk_line_desc{b.BdryFormat, b.A0, b.A1, b.A2, b.phi, b.c0_re, b.c1_re};
    }
    ds.pts.resize(nodeproplist.size());
    for (size_t k = 0; k < nodeproplist.size(); k++)
        ds.pts[k] = xfk_point_desc{nodeproplist[k].A_re, nodeproplist[k].A_im, nodeproplist[k].J_re,
                                   nodeproplist[k].J_im};
    ds.cir.resize(circproplist.size());
    for (size_t k = 0; k < circproplist.size(); k++)
        ds.cir[k] = xfk_circuit_desc{circproplist[k].CircType, circproplist[k].Amps_re, circproplist[k].dVolts_re};
    // the mesh arrays: huge-page storage, filled in parallel
    huge_reserve(ds.x, (size_t)NumNodes);
    huge_reserve(ds.y, (size_t)NumNodes);
    huge_reserve(ds.marker, (size_t)NumNodes);
    huge_reserve(ds.p, 3ull * NumEls);
    huge_reserve(ds.e, 3ull * NumEls);
    huge_reserve(ds.lbl, (size_t)NumEls);
    ds.x.resize(NumNodes);
    ds.y.resize(NumNodes);
    ds.marker.resize(NumNodes);
    ds.p.resize(3LL * NumEls);
    ds.e.resize(3LL * NumEls);
    ds.lbl.resize(NumEls);
    ds.pbc.resize(3LL * NumPBCs);
    const int nnp = (int)nodeproplist.size(), nlp = (int)lineproplist.size();
    par_for(NumNodes, 1 << 16, [&](long long a, long long b) {
        for (long long i = a; i < b; i++) {
            ds.x[i] = meshnode[i].x;
            ds.y[i] = meshnode[i].y;
            const int m = meshnode[i].BoundaryMarker;
            ds.marker[i] = m >= nnp ? -1 : m;
        }
    });
    std::atomic<bool> hole{false};
    par_for(NumEls, 1 << 16, [&](long long a, long long b) {
        for (long long i = a; i < b; i++) {
            const CMElement &el = meshele[i];
            if (labellist[el.lbl].BlockType < 0) hole = true;
            for (int q = 0; q < 3; q++) {
                ds.p[3 * i + q] = el.p[q];
                const int eq = el.e[q];
                ds.e[3 * i + q] = (eq >= 0 && eq < nlp) ? eq : -1;
            }
            ds.lbl[i] = el.lbl;
        }
    });
    if (hole) {
        warn("an element lies in a region without material (hole label)\n");
        return false;
    }
    for (int k = 0; k < NumPBCs; k++) {
        ds.pbc[3 * k] = pbclist[k].x;
        ds.pbc[3 * k + 1] = pbclist[k].y;
        ds.pbc[3 * k + 2] = pbclist[k].t;
    }
    xfk_problem_desc &d = ds.d;
    d.n_nodes = NumNodes; d.x = ds.x.data(); d.y = ds.y.data(); d.marker = ds.marker.data();
    d.n_elems = NumEls; d.p = ds.p.data(); d.e = ds.e.data(); d.lbl = ds.lbl.data();
    d.n_blocks = (int)ds.blk.size(); d.blocks = ds.blk.data();
    d.n_labels = (int)ds.lab.size(); d.labels = ds.lab.data();
    d.n_lines = (int)ds.lin.size(); d.lines = ds.lin.empty() ? nullptr : ds.lin.data();
    d.n_points = (int)ds.pts.size(); d.points = ds.pts.empty() ? nullptr : ds.pts.data();
    d.n_circs = (int)ds.cir.size(); d.circs = ds.cir.empty() ? nullptr : ds.cir.data();
    d.n_pbc = NumPBCs; d.pbc = NumPBCs ? ds.pbc.data() : nullptr;
    ds.age.clear();
    for (const AirGap &g : agelist) {
        xfk_age_desc a{};
        a.format = g.format; a.ri = g.ri; a.ro = g.ro; a.total_arc_length = g.arc;
        a.inner_shift = g.inner_shift; a.outer_shift = g.outer_shift; a.n_arc = g.n_arc;
        a.qn = g.qn.data(); a.qw = g.qw.data();
        ds.age.push_back(a);
    }
    d.n_ages = (int)ds.age.size(); d.ages = ds.age.empty() ? nullptr : ds.age.data();
    d.precision = Precision;
    d.length_units = (int)LengthUnits;
    d.coords = (int)Coords;
    d.relax = Relax;
    d.problem_type = ProblemTypeV == AXISYMMETRIC ? XFK_AXISYMMETRIC : XFK_PLANAR;
    d.ext_zo = extZo;
    d.ext_ro = extRo;
    d.ext_ri = extRi;
    return true;
}

namespace {
double ms_since(std::chrono::steady_clock::time_point &t)
{
    const auto n = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(n - t).count();
    t = n;
    return ms;
}
}  // namespace

int FSolver::Static2D()
{
    join_hip_warmup();
    auto t = std::chrono::steady_clock::now();
    DescStore ds;
    if (!make_desc(ds)) return false;
    // the .ans element section depends on the mesh only: formatted while the
    // device solves (joined by WriteStatic2D, or below on failure)
    if (ele_fmt_.joinable()) ele_fmt_.join();
    if (writes_output())
        ele_fmt_ = std::thread([this] {
            ele_text_ = format_static_elements();
            node_parts_ = format_static_node_parts();
        });
    xfk_problem *prob = nullptr;
    int rc = comm ? xfk_problem_create_dist(&ds.d, device, comm, &prob) : xfk_problem_create(&ds.d, device, &prob);
    ms_phase[2] = ms_since(t);
    if (rc == XFK_OK) rc = xfk_static2d(prob, 0, &stats);
    if (rc == XFK_OK) {
        A.assign(NumNodes, 0.0);
        rc = xfk_get_solution(prob, A.data());
    }
    if (rc == XFK_OK && !circproplist.empty()) {
        std::vector<int> cc(circproplist.size());
        std::vector<double> J(circproplist.size()), dV(circproplist.size());
        rc = xfk_get_circuits(prob, cc.data(), J.data(), dV.data());
        for (size_t k = 0; rc == XFK_OK && k < circproplist.size(); k++) {
            circproplist[k].Case = cc[k];
            circproplist[k].J = J[k];
            circproplist[k].dV = dV[k];
        }
    }
    if (rc != XFK_OK) {
        warn(std::string("GPU solver error: ") + xfk_last_error() + "\n");
        if (ele_fmt_.joinable()) ele_fmt_.join();
        ele_text_ = Formatted();
        node_parts_ = NodeParts();
    }
    if (prob) xfk_problem_destroy(prob);
    ms_phase[3] = ms_since(t);
    return rc == XFK_OK;
}

int FSolver::Harmonic2D()
{
    join_hip_warmup();
    auto t = std::chrono::steady_clock::now();
    DescStore ds;
    if (!make_desc(ds)) return false;
    std::vector<xfk_block_ac_desc> bac(blockproplist.size());
    for (size_t k = 0; k < blockproplist.size(); k++) {
        const CMSolverMaterialProp &m = blockproplist[k];
        const bool bh = m.BHpoints > 0;
        bac[k] = xfk_block_ac_desc{m.J_im, m.Theta_hx, m.Theta_hy, m.Lam_d, bh ? m.Hdata_im.data() : nullptr,
                                   bh ? m.slope_im.data() : nullptr};
    }
    std::vector<xfk_line_ac_desc> lac(lineproplist.size());
    for (size_t k = 0; k < lineproplist.size(); k++) {
        const CMBoundaryProp &b = lineproplist[k];
        lac[k] = xfk_line_ac_desc{b.c0_im, b.c1_im, b.Mu, b.Sig};
    }
    std::vector<xfk_circuit_ac_desc> cac(circproplist.size());
    for (size_t k = 0; k < circproplist.size(); k++)
        cac[k] = xfk_circuit_ac_desc{circproplist[k].Amps_im, circproplist[k].dVolts_im};
    std::vector<double> prox(2 * std::max<size_t>(1, labellist.size()), 0.0);
    for (size_t k = 0; k < labellist.size(); k++) {
        if (!std::isfinite(labellist[k].ProxMu_re) || !std::isfinite(labellist[k].ProxMu_im)) {
            // copper-clad aluminium wire (LamType 7, 8): the reference's
            // GetFillFactor leaves the wire radius at 0, ProximityMu = 0/0
            warn("copper-clad aluminium windings (LamType 7, 8) have no defined proximity permeability "
                 "(the reference computes 0/0); not supported\n");
            return false;
        }
        prox[2 * k] = labellist[k].ProxMu_re;
        prox[2 * k + 1] = labellist[k].ProxMu_im;
    }
    xfk_harmonic_desc ac{Frequency, bac.data(), lac.empty() ? nullptr : lac.data(),
                         cac.empty() ? nullptr : cac.data(), ACSolver, prox.data()};
    xfk_problem *prob = nullptr;
    int rc = comm ? xfk_problem_create_harmonic_dist(&ds.d, &ac, device, comm, &prob)
                  : xfk_problem_create_harmonic(&ds.d, &ac, device, &prob);
    ms_phase[2] = ms_since(t);
    if (rc == XFK_OK) rc = xfk_harmonic2d(prob, 0, &stats);
    std::vector<double> Ac;
    if (rc == XFK_OK) {
        Ac.assign(2 * (size_t)NumNodes, 0.0);
        rc = xfk_get_solution_complex(prob, Ac.data());
    }
    if (rc == XFK_OK) {
        A.resize(NumNodes);
        A_im.resize(NumNodes);
        for (int i = 0; i < NumNodes; i++) {
            A[i] = Ac[2 * i];
            A_im[i] = Ac[2 * i + 1];
        }
    }
    if (rc == XFK_OK && !circproplist.empty()) {
        const size_t nc = circproplist.size();
        std::vector<int> cc(nc);
        std::vector<double> J(2 * nc), dV(2 * nc);
        rc = xfk_get_circuits_complex(prob, cc.data(), J.data(), dV.data());
        for (size_t k = 0; rc == XFK_OK && k < nc; k++) {
            circproplist[k].Case = cc[k];
            circproplist[k].J = J[2 * k];
            circproplist[k].J_im = J[2 * k + 1];
            circproplist[k].dV = dV[2 * k];
            circproplist[k].dV_im = dV[2 * k + 1];
        }
    }
    if (rc != XFK_OK) warn(std::string("GPU solver error: ") + xfk_last_error() + "\n");
    if (prob) xfk_problem_destroy(prob);
    ms_phase[3] = ms_since(t);
    return rc == XFK_OK;
}

namespace {
// "%.17g" and "%i" as printf writes them (std::to_chars: the same correctly
// rounded digits and the same %g form), for the .ans's large sections
inline char *put_g17(char *p, double v) { return fastnum::put_g17(p, v); }   // (exact: fastnum.h)
inline char *put_i(char *p, int v) { return std::to_chars(p, p + 16, v).ptr; }
// lines [0, n): line(i, buf) writes line i (at most max_line chars) and returns
// its end; formatted in parallel chunks into huge-page buffers, then written
// in order by fwrite (one write of ~10 GB/s on the box; a shared mapping of
// the file was measured 5x slower, tools/lab/io_probe.cpp)
int format_chunks(int n) { return (int)std::max(1, std::min<int>(HostPool::get().size(), n / 8192)); }
template <class F>
FSolver::Formatted format_lines(int n, int max_line, F line)
{
    const int T = format_chunks(n);
    FSolver::Formatted f;
    f.buf.resize(T);
    f.len.assign(T, 0);
    par_for(T, 1, [&](long long t0, long long t1) {
        for (long long t = t0; t < t1; ++t) {
            const int a = (int)((long long)n * t / T), b = (int)((long long)n * (t + 1) / T);
            if (!f.buf[t].allocate((size_t)(b - a) * max_line + 1)) continue;   // (Formatted::ok() fails)
            char *q = f.buf[t].data();
            for (int i = a; i < b; ++i) q = line(i, q);
            f.len[t] = (size_t)(q - f.buf[t].data());
        }
    });
    return f;
}
bool write_formatted(FILE *fp, const FSolver::Formatted &f)
{
    if (!f.ok()) return false;   // (a chunk's buffer could not be allocated)
    for (size_t t = 0; t < f.buf.size(); ++t)
        if (f.len[t]) fwrite(f.buf[t].data(), 1, f.len[t], fp);
    return true;
}
template <class F>
bool write_lines(FILE *fp, int n, int max_line, F line)
{
    return write_formatted(fp, format_lines(n, max_line, line));
}
}  // namespace

FSolver::Formatted FSolver::format_static_elements() const
{
    return format_lines(NumEls, 64, [&](int i, char *q) {
        for (int m = 0; m < 3; ++m) {
            q = put_i(q, meshele[i].p[m]);
            *q++ = '\t';
        }
        q = put_i(q, meshele[i].lbl);
        *q++ = '\n';
        return q;
    });
}

FSolver::NodeParts FSolver::format_static_node_parts() const
{
    const double unitconv[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    const double cf = unitconv[LengthUnits];
    NodeParts np;
    const int n = NumNodes, T = format_chunks(n);
    np.lo.resize(T + 1);
    for (int t = 0; t <= T; ++t) np.lo[t] = (int)((long long)n * t / T);
    np.pre.resize(n);
    np.suf.resize(n);
    np.f = format_lines(n, 104, [&](int i, char *q) {
        char *q0 = q;
        q = put_g17(q, meshnode[i].x / cf);
        *q++ = '\t';
        q = put_g17(q, meshnode[i].y / cf);
        *q++ = '\t';
        np.pre[i] = (unsigned char)(q - q0);
        q0 = q;
        *q++ = '\t';
        q = put_i(q, meshnode[i].BoundaryMarker);
        // static2d.cpp:1093-1101: Aprev follows the marker with no separator
        if (!Aprev.empty()) q = put_g17(q, Aprev[i]);
        *q++ = '\n';
        np.suf[i] = (unsigned char)(q - q0);
        return q;
    });
    return np;
}

// an existing .ans is moved aside and unlinked beside the write (truncating
// ~130 MB of page cache in fopen costs ~7 ms); the new file is written whole.
// A symlinked or hard-linked .ans keeps the reference's fopen("wt") behaviour
// (truncated in place: the link target, inode and permissions stay); the
// aside name is unique (mkstemp in the same directory, replaced by rename).
void FSolver::clear_old_output(const std::string &path)
{
    struct stat st;
    if (::lstat(path.c_str(), &st) != 0 || !S_ISREG(st.st_mode) || st.st_nlink > 1 || st.st_size < (1 << 20))
        return;
    std::string aside = path + ".xfemm-old-XXXXXX";
    const int fd = ::mkstemp(&aside[0]);
    if (fd < 0) return;
    ::close(fd);
    if (::rename(path.c_str(), aside.c_str()) == 0) remove_async({aside});
    else ::unlink(aside.c_str());
}

int FSolver::WriteStatic2D()
{
    LoadTrace tr;
    const double unitconv[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    std::string fin = PathName + ".fem", fout = PathName + ".ans";
    FILE *fz = fopen(fin.c_str(), "rt");
    if (!fz) {
        warn("Couldn't open " + fin + "\n");
        return false;
    }
    clear_old_output(fout);
    FILE *fp = fopen(fout.c_str(), "wt");
    if (!fp) {
        fclose(fz);
        warn("Couldn't write to " + fout + "\n");
        return false;
    }
    char c[1024];
    while (fgets(c, 1024, fz) != nullptr) fputs(c, fp);
    fclose(fz);
    tr.mark("  .fem echo");
    fprintf(fp, "[Solution]\n");
    const double cf = unitconv[LengthUnits];
    fprintf(fp, "%i\n", NumNodes);
    fflush(fp);
    if (ele_fmt_.joinable()) ele_fmt_.join();   // (element text and node parts formatted beside the device solve)
    Formatted nodes_text;
    NodeParts &np = node_parts_;
    if (np.lo.size() >= 2 && np.lo.back() == NumNodes && (int)np.f.buf.size() == (int)np.lo.size() - 1) {
        // the parts around A, with A put in between
        const int T = (int)np.lo.size() - 1;
        nodes_text.buf.resize(T);
        nodes_text.len.assign(T, 0);
        par_for(T, 1, [&](long long t0, long long t1) {
            for (long long t = t0; t < t1; ++t) {
                const int a = np.lo[t], b = np.lo[t + 1];
                if (!nodes_text.buf[t].allocate(np.f.len[t] + (size_t)(b - a) * 25 + 1)) continue;
                const char *p = np.f.buf[t].data();
                char *q = nodes_text.buf[t].data();
                for (int i = a; i < b; ++i) {
                    std::memcpy(q, p, np.pre[i]);
                    q += np.pre[i];
                    p += np.pre[i];
                    q = put_g17(q, A[i]);
                    std::memcpy(q, p, np.suf[i]);
                    q += np.suf[i];
                    p += np.suf[i];
                }
                nodes_text.len[t] = (size_t)(q - nodes_text.buf[t].data());
            }
        });
    } else {
        nodes_text = format_lines(NumNodes, 128, [&](int i, char *q) {
            q = put_g17(q, meshnode[i].x / cf);
            *q++ = '\t';
            q = put_g17(q, meshnode[i].y / cf);
            *q++ = '\t';
            q = put_g17(q, A[i]);
            *q++ = '\t';
            q = put_i(q, meshnode[i].BoundaryMarker);
            // static2d.cpp:1093-1101: Aprev follows the marker with no separator
            if (!Aprev.empty()) q = put_g17(q, Aprev[i]);
            *q++ = '\n';
            return q;
        });
    }
    node_parts_ = NodeParts();
    tr.mark("  .ans nodes formatted");
    if (!write_formatted(fp, nodes_text)) {
        fclose(fp);
        warn("couldn't allocate the .ans node text\n");
        return false;
    }
    tr.mark("  .ans nodes written");
    fprintf(fp, "%i\n", NumEls);
    fflush(fp);
    if (ele_text_.buf.empty()) ele_text_ = format_static_elements();
    tr.mark("  .ans element text joined");
    const bool ele_ok = write_formatted(fp, ele_text_);
    ele_text_ = Formatted();
    if (!ele_ok) {
        fclose(fp);
        warn("couldn't allocate the .ans element text\n");
        return false;
    }
    tr.mark("  .ans elements");
    fprintf(fp, "%i\n", (int)labellist.size());
    for (size_t k = 0; k < labellist.size(); k++) {
        int i = labellist[k].InCircuit;
        if (i < 0) fprintf(fp, "1\t0\n");
        else {
            if (circproplist[i].Case == 0) fprintf(fp, "0\t%.17g\n", circproplist[i].dV);
            if (circproplist[i].Case == 1) fprintf(fp, "1\t%.17g\n", circproplist[i].J);
        }
    }
    fprintf(fp, "%i\n", NumPBCs);
    for (int k = 0; k < NumPBCs; k++) fprintf(fp, "%i\t%i\t%i\n", pbclist[k].x, pbclist[k].y, pbclist[k].t);
    WriteAirGapElements(fp);
    fclose(fp);
    tr.mark("  .ans close");
    return true;
}

void FSolver::WriteAirGapElements(FILE *fp) const
{
    // static2d.cpp:1161-1190 / harmonic2d.cpp:1002-1030: per AGE its name as
    // read from the .pbc (newline kept), the parameter line, and the
    // totalArcElements + 1 quadNodes in the renumbered node ids -- the input
    // fpproc's gap integrals (torque, force) read back
    fprintf(fp, "%i\n", NumAirGapElems);
    for (const AirGap &g : agelist) {
        fprintf(fp, "%s", g.name.c_str());
        fprintf(fp, "%i %.17g %.17g %.17g %.17g %.17g %.17g %.17g %i %.17g %.17g\n", g.format, g.inner_angle,
                g.outer_angle, g.ri, g.ro, g.arc, g.agc_re, g.agc_im, g.n_arc, g.inner_shift, g.outer_shift);
        for (int k = 0; k <= g.n_arc; k++)
            fprintf(fp, "%i %.17g %i %.17g %i %.17g %i %.17g\n", g.qn[4 * k], g.qw[4 * k], g.qn[4 * k + 1],
                    g.qw[4 * k + 1], g.qn[4 * k + 2], g.qw[4 * k + 2], g.qn[4 * k + 3], g.qw[4 * k + 3]);
    }
}

int FSolver::WriteHarmonic2D()
{
    // harmonic2d.cpp:793-960: echo the .fem, then nodes (x, y, A re, A im,
    // marker), elements (p, label, edge markers), circuit data per label,
    // periodic pairs, air-gap elements
    const double unitconv[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    std::string fin = PathName + ".fem", fout = PathName + ".ans";
    FILE *fz = fopen(fin.c_str(), "rt");
    if (!fz) {
        warn("Couldn't open " + fin + "\n");
        return false;
    }
    FILE *fp = fopen(fout.c_str(), "wt");
    if (!fp) {
        fclose(fz);
        warn("Couldn't write to " + fout + "\n");
        return false;
    }
    char c[1024];
    while (fgets(c, 1024, fz) != nullptr) fputs(c, fp);
    fclose(fz);
    fprintf(fp, "[Solution]\n");
    const double cf = unitconv[LengthUnits];
    fprintf(fp, "%i\n", NumNodes);
    // incremental problems add A of the previous solution per node and J per
    // element (harmonic2d.cpp:929-949)
    fflush(fp);
    bool text_ok = write_lines(fp, NumNodes, 160, [&](int i, char *q) {
        for (double v : {meshnode[i].x / cf, meshnode[i].y / cf, A[i], A_im[i]}) {
            q = put_g17(q, v);
            *q++ = '\t';
        }
        q = put_i(q, meshnode[i].BoundaryMarker);
        if (!Aprev.empty()) {
            *q++ = '\t';
            q = put_g17(q, Aprev[i]);
        }
        *q++ = '\n';
        return q;
    });
    if (text_ok) fprintf(fp, "%i\n", NumEls);
    fflush(fp);
    text_ok = text_ok && write_lines(fp, NumEls, 128, [&](int i, char *q) {
        const CMElement &e = meshele[i];
        for (int v : {e.p[0], e.p[1], e.p[2], e.lbl, e.e[0], e.e[1]}) {
            q = put_i(q, v);
            *q++ = '\t';
        }
        q = put_i(q, e.e[2]);
        if (!Aprev.empty()) {
            *q++ = '\t';
            q = put_g17(q, e.Jprev);
        }
        *q++ = '\n';
        return q;
    });
    if (!text_ok) {
        fclose(fp);
        warn("couldn't allocate the .ans text\n");
        return false;
    }
    fprintf(fp, "%i\n", (int)labellist.size());
    for (size_t k = 0; k < labellist.size(); k++) {
        int i = labellist[k].InCircuit;
        if (i < 0) fprintf(fp, "1\t0\t0\n");
        else {
            const CMCircuit &C = circproplist[i];
            if (C.Case == 0) fprintf(fp, "0\t%.17g\t%.17g\n", C.dV, C.dV_im);
            if (C.Case == 1) fprintf(fp, "1\t%.17g\t%.17g\n", C.J, C.J_im);
        }
    }
    fprintf(fp, "%i\n", NumPBCs);
    for (int k = 0; k < NumPBCs; k++) fprintf(fp, "%i  %i %i\n", pbclist[k].x, pbclist[k].y, pbclist[k].t);
    WriteAirGapElements(fp);
    fclose(fp);
    return true;
}

bool FSolver::runSolver(bool verbose)
{
    struct JoinRemovals {   // the mesh files are gone when runSolver returns, as in the reference
        FSolver *s;
        ~JoinRemovals() { s->join_removals(); }
    } join_at_exit{this};
    for (double &m : ms_phase) m = 0;
    auto t = std::chrono::steady_clock::now();
    // sharded (set_comm): every rank reads the same mesh files; they are
    // deleted by rank 0 once the collective solve has run (every rank has
    // read them by then)
    const bool delete_now = deleteMeshFiles && !comm;
    LoadMeshErr err = LoadMesh(delete_now);
    ms_phase[0] = ms_since(t);
    if (err != NOERROR) {
        warn(getErrorString(err));
        return false;
    }
    if (previousSolutionFile.empty()) {
        if (verbose) PrintMessage("renumbering nodes using Cuthill-McKee method\n");
        if (!Cuthill(delete_now)) {
            warn("problem renumbering node points\n");
            return false;
        }
    }
    ms_phase[1] = ms_since(t);
    if (!previousSolutionFile.empty()) {   // fsolver.cpp:1245-1320
        if (Frequency == 0 && PrevType != 0) {
            warn("Cannot handle incremental permeability problems with frequency 0.\n");
            return false;
        }
        if (Frequency != 0 && ProblemTypeV == AXISYMMETRIC) {
            warn("Cannot handle harmonic axisymmetric incremental problems.\n");
            return false;
        }
        if (Frequency != 0)
            warn("Harmonic planar incremental permeability problems are work in progress. RESULTS WON'T BE VALID!\n");
    }
    if (verbose) {
        PrintMessage("solving...\n");
        PrintMessage("Problem Statistics:\n%i nodes\n%i elements\nPrecision: %f\n", NumNodes, NumEls, Precision);
    }
    if (Frequency != 0) {   // Harmonic2D / HarmonicAxisymmetric, one .ans layout (fsolver.cpp:1312-1336)
        const bool solved = Harmonic2D();
        remove_mesh_files_after_collective_solve();
        if (!solved) {
            warn("Couldn't solve the problem\n");
            return false;
        }
        if (!writes_output()) return true;   // (sharded: rank 0 writes the .ans)
        if (verbose)
            PrintMessage(ProblemTypeV == AXISYMMETRIC ? "Harmonic axisymmetric problem solved\n"
                                                      : "Harmonic 2-D problem solved\n");
        t = std::chrono::steady_clock::now();
        if (!WriteHarmonic2D()) {
            warn("couldn't write results to disk\n");
            return false;
        }
        ms_phase[4] = ms_since(t);
        if (verbose) PrintMessage("results written to disk\n");
        return true;
    }
    const bool solved = Static2D();
    remove_mesh_files_after_collective_solve();
    if (!solved) {
        warn("Couldn't solve the problem\n");
        return false;
    }
    if (!writes_output()) return true;   // (sharded: rank 0 writes the .ans)
    if (verbose)
        PrintMessage(ProblemTypeV == AXISYMMETRIC ? "Static axisymmetric problem solved\n" : "Static 2-D problem solved\n");
    t = std::chrono::steady_clock::now();
    if (!WriteStatic2D()) {
        warn("couldn't write results to disk\n");
        return false;
    }
    ms_phase[4] = ms_since(t);
    if (verbose) PrintMessage("results written to disk\n");
    return true;
}

}  // namespace xfemm
