// Host driver + C-ABI of the MI355X fsolver hot path (include/xfemm_kernels.h).
//
// xfk_static2d() is FSolver::Static2D (cfemm/fsolver/static2d.cpp:53-1033) on
// the GPU.  Host work per problem is limited to O(boundary) preparation done
// once at creation: circuit totals (static2d.cpp:84-167, element order, so the
// circuit J/dV are bit-identical to the reference), the first/last Dirichlet
// value of every fixed node in the reference's SetValue call order
// (static2d.cpp:827-926), and the composition of the sequential
// Periodicity/AntiPeriodicity calls (spars.cpp:366-474) into one linear
// averaging map over CSR slots.  Everything else runs on the device.
#include <hipcub/hipcub.hpp>

#include "xfk_amg.h"
#include "xfk_spmv.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <iterator>
#include <set>
#include <type_traits>
#include <unordered_map>

#include "xfk_age.h"
#include "xfk_comm.h"
#include "xfk_kernels.h"
#include "xfk_magdir.h"
#include <cstdio>
#include <cstdlib>
#include "xfk_partition.h"

namespace {
// XFK_TRACE_CREATE=1: host milliseconds of each problem-creation stage on stderr
struct CreateTrace {
    bool on = std::getenv("XFK_TRACE_CREATE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char *what)
    {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[create] %-28s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};
}  // namespace

namespace xfk {

static thread_local std::string g_err;

// device allocation counters (xfk_alloc_stats)
namespace {
std::atomic<long long> g_nmalloc{0}, g_nfree{0}, g_nsmalloc{0}, g_nsfree{0};
long long now_ns()
{
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
}  // namespace

// Process-wide cache of device blocks.  A problem being destroyed (its main
// stream synchronised; every side-stream task was joined into it) returns its
// blocks here instead of to hipFree, and the next problem of the process --
// the next rotor angle, the next .fem of a session -- takes them back instead
// of calling hipMalloc (each call costs host time; each hipFree waits for the
// device).  Blocks are rounded up to size classes (powers of two up to 64 KiB,
// then sixteenth steps of the power of two: at most 6.25 % slack) and matched
// by class and device; at most kPoolCap bytes stay cached.  Any other free (a
// buffer that grows, a function's scratch) goes straight to hipFree: only the
// destroy path knows the device no longer reads the block.
namespace {
// cap: XFK_POOL_CAP_MB (default 64 GiB; 0 keeps nothing), read once
size_t env_mb(const char *name, size_t dflt)
{
    const char *v = std::getenv(name);
    if (!v || !*v) return dflt;
    return (size_t)std::strtoull(v, nullptr, 10) << 20;
}
const size_t kPoolCap = env_mb("XFK_POOL_CAP_MB", 64ull << 30);
struct BlockPool {
    std::mutex mu;
    std::map<std::pair<int, size_t>, std::vector<void *>> free;
    std::unordered_map<void *, std::pair<int, size_t>> live;   // block -> (device, class bytes)
    size_t cached = 0;
};
BlockPool &block_pool()
{
    static BlockPool *p = new BlockPool();   // (never destroyed: blocks outlive static destructors)
    return *p;
}
thread_local bool tl_pool_release = false;
thread_local DevArena *tl_arena = nullptr;
constexpr size_t kArenaChunk = 256ull << 20;
constexpr size_t kArenaAlign = 256;
std::atomic<long long> g_npool{0};
size_t size_class(size_t b)
{
    if (b <= 256) return 256;
    size_t p2 = 1;
    while (p2 < b) p2 <<= 1;
    if (p2 <= (64u << 10)) return p2;
    const size_t step = (p2 >> 1) >> 4;   // sixteenths of the lower power of two
    return ((b + step - 1) / step) * step;
}
}  // namespace

// blocks freed inside its scope go to the process cache (the caller has
// synchronised the device work that could read them)
struct PoolRelease {
    bool prev = tl_pool_release;
    PoolRelease() { tl_pool_release = true; }
    ~PoolRelease() { tl_pool_release = prev; }
};

ArenaScope::ArenaScope(DevArena *a) : prev(tl_arena) { tl_arena = a; }
ArenaScope::~ArenaScope() { tl_arena = prev; }

static hipError_t pool_malloc(void **p, size_t bytes);

hipError_t dev_malloc(void **p, size_t bytes)
{
    DevArena *a = tl_arena;
    if (!a) return pool_malloc(p, bytes);
    const size_t need = (bytes + kArenaAlign - 1) & ~(kArenaAlign - 1);
    // a block freed in an earlier solve of this problem, if one fits without
    // wasting more than its own size (a repeated solve asks for the same sizes)
    auto it = a->reuse.lower_bound(need);
    if (it != a->reuse.end() && it->first <= 2 * need + (64u << 10)) {
        char *q = it->second;
        a->carved[q] = it->first;
        a->reuse.erase(it);
        *p = q;
        std::lock_guard<std::mutex> g(block_pool().mu);
        block_pool().live[q] = {-1, 0};
        return hipSuccess;
    }
    size_t at = (a->off + kArenaAlign - 1) & ~(kArenaAlign - 1);
    if (a->chunks.empty() || at + need > a->chunks.back().second) {
        // (carving starts one alignment step in: no carved block has its chunk's address)
        const size_t csz = std::max(a->next_chunk, need + kArenaAlign);
        a->next_chunk = std::min(kArenaChunk, 2 * a->next_chunk);
        void *c = nullptr;
        tl_arena = nullptr;   // (the chunk itself comes from the process cache or hipMalloc)
        const hipError_t e = pool_malloc(&c, csz);
        tl_arena = a;
        if (e != hipSuccess) return e;
        a->chunks.push_back({static_cast<char *>(c), csz});
        at = kArenaAlign;
    }
    *p = a->chunks.back().first + at;
    a->off = at + need;
    a->carved[*p] = need;
    std::lock_guard<std::mutex> g(block_pool().mu);
    block_pool().live[*p] = {-1, 0};   // (carved: dev_free leaves it to the arena)
    return hipSuccess;
}

hipError_t DevArena::reserve(size_t bytes)
{
    const size_t at = (off + kArenaAlign - 1) & ~(kArenaAlign - 1);
    if (bytes == 0 || (!chunks.empty() && at + bytes <= chunks.back().second)) return hipSuccess;
    DevArena *cur = tl_arena;
    tl_arena = nullptr;   // (the chunk itself comes from the process cache or hipMalloc)
    void *c = nullptr;
    const size_t csz = ((bytes + kArenaAlign - 1) & ~(kArenaAlign - 1)) + kArenaAlign;
    const hipError_t e = pool_malloc(&c, csz);
    tl_arena = cur;
    if (e != hipSuccess) return e;
    chunks.push_back({static_cast<char *>(c), csz});
    off = kArenaAlign;   // (carving starts one alignment step in, as in dev_malloc)
    next_chunk = kArenaChunk;
    return hipSuccess;
}

bool DevArena::retire(void *p)
{
    auto it = carved.find(p);
    if (it == carved.end()) return false;
    pending.push_back({static_cast<char *>(p), it->second});
    carved.erase(it);
    std::lock_guard<std::mutex> g(block_pool().mu);
    block_pool().live.erase(p);
    return true;
}

bool arena_retire(void *p)
{
    return p && tl_arena && tl_arena->retire(p);
}

void DevArena::recycle()
{
    for (auto &b : pending) reuse.insert({b.second, b.first});
    pending.clear();
}

size_t DevArena::chunk_bytes() const
{
    size_t t = 0;
    for (auto &c : chunks) t += c.second;
    return t;
}

void DevArena::release()
{
    {
        std::lock_guard<std::mutex> g(block_pool().mu);
        for (auto &kv : carved) block_pool().live.erase(kv.first);
    }
    carved.clear();
    reuse.clear();
    pending.clear();
    for (auto &c : chunks) dev_free(c.first);
    chunks.clear();
    off = 0;
}

static hipError_t pool_malloc(void **p, size_t bytes)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    const size_t cls = size_class(bytes);
    BlockPool &bp = block_pool();
    {
        std::lock_guard<std::mutex> g(bp.mu);
        auto it = bp.free.find({dev, cls});
        if (it != bp.free.end() && !it->second.empty()) {
            *p = it->second.back();
            it->second.pop_back();
            bp.cached -= cls;
            bp.live[*p] = {dev, cls};
            ++g_npool;
            return hipSuccess;
        }
    }
    const long long t = now_ns();
    hipError_t e = hipMalloc(p, cls);
    g_nsmalloc += now_ns() - t;
    ++g_nmalloc;
    if (e != hipSuccess) {   // out of memory with blocks cached: return them and try once more
        std::vector<void *> drop;
        {
            std::lock_guard<std::mutex> g(bp.mu);
            for (auto &kv : bp.free)
                for (void *q : kv.second) drop.push_back(q);
            bp.free.clear();
            bp.cached = 0;
        }
        if (drop.empty()) return e;
        for (void *q : drop) (void)hipFree(q);
        (void)hipGetLastError();
        e = hipMalloc(p, cls);
    }
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> g(bp.mu);
        bp.live[*p] = {dev, cls};
    }
    return e;
}
void dev_free(void *p)
{
    if (arena_retire(p)) return;   // carved from the active arena: reusable after this solve
    BlockPool &bp = block_pool();
    {
        std::lock_guard<std::mutex> g(bp.mu);
        auto it = bp.live.find(p);
        if (it != bp.live.end()) {
            const auto key = it->second;
            bp.live.erase(it);
            if (key.second == 0) return;   // carved from an arena: freed with it
            if (tl_pool_release && bp.cached + key.second <= kPoolCap) {
                bp.free[key].push_back(p);
                bp.cached += key.second;
                return;
            }
        }
    }
    const long long t = now_ns();
    (void)hipFree(p);
    g_nsfree += now_ns() - t;
    ++g_nfree;
}
// Process-wide cache of pinned host buffers (each hipHostMalloc pins pages,
// tens of us; hipHostFree may wait for the device): a problem's host mirrors
// and its AMG's read-back / staging buffers go back here when the problem is
// destroyed, for the next problem of the process.  Size classes as above; at
// most kPinCap bytes stay cached.
namespace {
const size_t kPinCap = env_mb("XFK_PIN_CAP_MB", 1ull << 30);   // (XFK_PIN_CAP_MB, default 1 GiB)
struct PinPool {
    std::mutex mu;
    std::map<size_t, std::vector<void *>> free;
    std::unordered_map<void *, size_t> live;
    size_t cached = 0;
};
PinPool &pin_pool()
{
    static PinPool *p = new PinPool();   // (never destroyed, like the device cache)
    return *p;
}
}  // namespace

hipError_t pinned_malloc(void **p, size_t bytes)
{
    const size_t cls = size_class(bytes);
    PinPool &pp = pin_pool();
    {
        std::lock_guard<std::mutex> g(pp.mu);
        auto it = pp.free.find(cls);
        if (it != pp.free.end() && !it->second.empty()) {
            *p = it->second.back();
            it->second.pop_back();
            pp.cached -= cls;
            pp.live[*p] = cls;
            return hipSuccess;
        }
    }
    const hipError_t e = hipHostMalloc(p, cls);
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> g(pp.mu);
        pp.live[*p] = cls;
    }
    return e;
}
void pinned_free(void *p)
{
    if (!p) return;
    PinPool &pp = pin_pool();
    {
        std::lock_guard<std::mutex> g(pp.mu);
        auto it = pp.live.find(p);
        if (it != pp.live.end()) {
            const size_t cls = it->second;
            pp.live.erase(it);
            if (tl_pool_release && pp.cached + cls <= kPinCap) {
                pp.free[cls].push_back(p);
                pp.cached += cls;
                return;
            }
        }
    }
    (void)hipHostFree(p);
}

thread_local PhaseProf *g_prof = nullptr;
void set_error(const std::string &msg) { g_err = msg; }

// Symbolic composition of CBigLinProb::Periodicity / AntiPeriodicity
// (spars.cpp:366-474) applied in pbclist order (static2d.cpp:929-940).  Each
// touched matrix entry / RHS entry becomes a linear combination of the
// post-Dirichlet values; sets of rows k are structural supersets of the
// reference's value-based scan, which is exact because averaging zeros gives
// zero.
//
// Storage: every combination is an immutable run of (key, weight) terms in
// one pool (a handle = offset + length; entries that share a combination
// share the run), the current combination of each entry / RHS row sits in an
// open-addressing table, and the neighbour sets of the coupled nodes are
// indexed by a dense node -> slot array -- no allocation per entry (the
// per-entry vectors and node maps cost ~12 ms on the 2250 pairs of the
// refined TorqueBenchmark).
namespace {
using Term = std::pair<long long, double>;
struct TRun {
    unsigned off = 0, len = 0;
};
struct TermPool {
    std::vector<Term> t;
    // a x + b y of two runs sorted by key (every run is: a single term or
    // lin2's own output), merged -- a key in both gets a x + b y, in one a x
    // or b y, as the accumulation into a zeroed map gives; zeros dropped
    TRun lin2(double a, TRun x, double b, TRun y)
    {
        if (t.capacity() < t.size() + x.len + y.len) t.reserve(2 * (t.size() + x.len + y.len));
        const Term *xp = t.data() + x.off, *yp = t.data() + y.off;
        TRun out{(unsigned)t.size(), 0};
        unsigned i = 0, j = 0;
        while (i < x.len || j < y.len) {
            double v;
            long long k;
            if (j == y.len || (i < x.len && xp[i].first < yp[j].first)) {
                k = xp[i].first;
                v = a * xp[i++].second;
            } else if (i == x.len || yp[j].first < xp[i].first) {
                k = yp[j].first;
                v = b * yp[j++].second;
            } else {
                k = xp[i].first;
                v = a * xp[i++].second + b * yp[j++].second;
            }
            if (v != 0.0) t.push_back({k, v});   // (capacity reserved: xp, yp stay valid)
        }
        out.len = (unsigned)t.size() - out.off;
        return out;
    }
    TRun single(long long k)
    {
        t.push_back({k, 1.0});
        return TRun{(unsigned)t.size() - 1, 1};
    }
};
// key (>= 0) -> run, linear probing
struct RunMap {
    std::vector<long long> key;
    std::vector<TRun> val;
    size_t n = 0;
    int shift = 60;
    explicit RunMap(size_t expect)
    {
        size_t c = 16;
        while (c < 2 * expect) c <<= 1;
        alloc(c);
    }
    void alloc(size_t c)
    {
        key.assign(c, -1);
        val.assign(c, TRun{});
        shift = 64 - __builtin_ctzll(c);
    }
    size_t home(long long k) const { return (size_t)(((unsigned long long)k * 0x9E3779B97F4A7C15ULL) >> shift); }
    const TRun *find(long long k) const
    {
        const size_t m = key.size() - 1;
        for (size_t h = home(k);; h = (h + 1) & m) {
            if (key[h] == k) return &val[h];
            if (key[h] < 0) return nullptr;
        }
    }
    void put(long long k, TRun v)
    {
        if (2 * (n + 1) > key.size()) {
            std::vector<long long> ok;
            std::vector<TRun> ov;
            ok.swap(key);
            ov.swap(val);
            alloc(2 * ok.size());
            n = 0;
            for (size_t h = 0; h < ok.size(); ++h)
                if (ok[h] >= 0) put(ok[h], ov[h]);
        }
        const size_t m = key.size() - 1;
        for (size_t h = home(k);; h = (h + 1) & m) {
            if (key[h] == k) {
                val[h] = v;
                return;
            }
            if (key[h] < 0) {
                key[h] = k;
                val[h] = v;
                ++n;
                return;
            }
        }
    }
    // (key, run) pairs in ascending key order
    std::vector<std::pair<long long, TRun>> sorted() const
    {
        std::vector<std::pair<long long, TRun>> o;
        o.reserve(n);
        for (size_t h = 0; h < key.size(); ++h)
            if (key[h] >= 0) o.push_back({key[h], val[h]});
        std::sort(o.begin(), o.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        return o;
    }
};
}  // namespace

static inline long long ukey(int r, int c)
{
    if (c < r) std::swap(r, c);
    return ((long long)r << 32) | (unsigned)c;
}

static inline long long okey(int r, int c) { return ((long long)r << 32) | (unsigned)c; }

// small sorted neighbour sets (a node has ~6-20 neighbours): sorted vectors
using NbSet = std::vector<int>;
static inline void nb_insert(NbSet &v, int x)
{
    auto it = std::lower_bound(v.begin(), v.end(), x);
    if (it == v.end() || *it != x) v.insert(it, x);
}
static inline bool nb_has(const NbSet &v, int x) { return std::binary_search(v.begin(), v.end(), x); }

static int build_pbc_map(xfk_problem *P, bool aux)
{
    const int npbc = (int)P->hpbc.size() / 3;
    if (npbc == 0) return XFK_OK;
    CreateTrace tr;
    for (int q = 0; q < npbc; ++q) {
        const int i = P->hpbc[3 * q], j = P->hpbc[3 * q + 1], t = P->hpbc[3 * q + 2];
        if ((t == 0 || t == 1) && (i < 0 || j < 0 || i >= P->NL || j >= P->NL)) {
            set_error("pbc node index out of range");
            return XFK_ERR_ARG;
        }
    }
    // original neighbours of the coupled nodes (slot[v] >= 0), then the current ones
    std::vector<int> slot(std::max(1, P->NL), -1);
    std::vector<NbSet> N0;
    N0.reserve(2 * (size_t)npbc);
    for (int k = 0; k < npbc; ++k)
        for (int m = 0; m < 2; ++m) {
            const int v = P->hpbc[3 * k + m];
            if (v >= 0 && v < P->NL && slot[v] < 0) {
                slot[v] = (int)N0.size();
                N0.emplace_back();
            }
        }
    for (int e = 0; e < P->NE; ++e)
        for (int j = 0; j < 3; ++j) {
            const int v = P->hp[3 * e + j];
            if (v < 0 || v >= P->NL || slot[v] < 0) continue;
            NbSet &s = N0[slot[v]];
            for (int m = 0; m < 3; ++m)
                if (m != j) nb_insert(s, P->hp[3 * e + m]);
        }
    auto slot_of = [&](int v) { return (v >= 0 && v < P->NL) ? slot[v] : -1; };
    for (long long k : P->age_key) {   // air-gap couplings are entries of the matrix too
        const int r = (int)(k >> 32), c = (int)(k & 0xffffffff);
        if (r == c) continue;
        if (slot_of(r) >= 0) nb_insert(N0[slot_of(r)], c);
        if (slot_of(c) >= 0) nb_insert(N0[slot_of(c)], r);
    }
    tr.mark("    pbc neighbour sets");
    std::vector<NbSet> Ncur = N0;
    TermPool pool;
    pool.t.reserve(64 * (size_t)npbc);
    RunMap E(16 * (size_t)npbc), Eb(2 * (size_t)npbc);
    std::vector<long long> fill;
    auto is_orig = [&](int r, int c) -> bool {
        if (r == c) return true;
        int s = slot_of(r);
        if (s >= 0) return nb_has(N0[s], c);
        s = slot_of(c);
        if (s >= 0) return nb_has(N0[s], r);
        return false;
    };
    // the current combination of entry (r, c): the map's, else the entry itself
    // (an original one) or nothing
    auto get = [&](int r, int c) -> TRun {
        const long long k = ukey(r, c);
        if (const TRun *h = E.find(k)) return *h;
        if (is_orig(r, c)) return pool.single(k);
        return TRun{};
    };
    // auxiliary matrices of the Newton AC solver: ordered entries
    RunMap Ea(aux ? 32 * (size_t)npbc : 1);
    std::vector<long long> afill;
    auto geta = [&](int r, int c) -> TRun {
        const long long k = okey(r, c);
        if (const TRun *h = Ea.find(k)) return *h;
        if (is_orig(r, c)) return pool.single(k);
        return TRun{};
    };
    auto getb = [&](int i) -> TRun {
        if (const TRun *h = Eb.find(i)) return *h;
        return pool.single(i);
    };
    const TRun none{};
    NbSet K;
    for (int q = 0; q < npbc; ++q) {
        int i = P->hpbc[3 * q], j = P->hpbc[3 * q + 1], t = P->hpbc[3 * q + 2];
        if (t != 0 && t != 1) continue;  // static2d.cpp:932-939 only handles 0 and 1
        if (j < i) std::swap(i, j);
        const double sg = (t == 0) ? 1.0 : -1.0;
        NbSet &Ni = Ncur[slot[i]], &Nj = Ncur[slot[j]];
        K.clear();
        std::set_union(Ni.begin(), Ni.end(), Nj.begin(), Nj.end(), std::back_inserter(K));
        K.erase(std::remove_if(K.begin(), K.end(), [&](int x) { return x == i || x == j; }), K.end());
        for (int k : K) {
            const TRun c = pool.lin2(0.5, get(k, i), 0.5 * sg, get(k, j));
            E.put(ukey(k, j), sg > 0 ? c : pool.lin2(-1.0, c, 0.0, none));
            E.put(ukey(k, i), c);
            if (aux) {   // row k and, by the Hermitian / anti-Hermitian flip of Put, column k
                const TRun ca = pool.lin2(0.5, geta(k, i), 0.5 * sg, geta(k, j));
                const TRun ct = pool.lin2(0.5, geta(i, k), 0.5 * sg, geta(j, k));
                Ea.put(okey(k, i), ca);
                Ea.put(okey(k, j), pool.lin2(sg, ca, 0.0, none));
                Ea.put(okey(i, k), ct);
                Ea.put(okey(j, k), pool.lin2(sg, ct, 0.0, none));
            }
            for (int m : {i, j})
                if (!is_orig(k, m)) fill.push_back(ukey(k, m));
            nb_insert(Ni, k);
            nb_insert(Nj, k);
            const int sk = slot_of(k);
            if (sk >= 0) {
                nb_insert(Ncur[sk], i);
                nb_insert(Ncur[sk], j);
            }
        }
        const TRun d = pool.lin2(0.5, get(i, i), 0.5, get(j, j));
        E.put(ukey(i, i), d);
        E.put(ukey(j, j), d);
        if (aux) {   // auxiliary (i, j) block: c = (ii +- ij +- ji + jj) / 4 at ii, jj and +-c at ij, ji
            const TRun l1 = pool.lin2(1.0, geta(i, i), sg, geta(i, j));
            const TRun l2 = pool.lin2(sg, geta(j, i), 1.0, geta(j, j));
            const TRun da = pool.lin2(0.25, l1, 0.25, l2);
            Ea.put(okey(i, i), da);
            Ea.put(okey(j, j), da);
            Ea.put(okey(i, j), pool.lin2(sg, da, 0.0, none));
            Ea.put(okey(j, i), pool.lin2(sg, da, 0.0, none));
            if (!is_orig(i, j)) afill.push_back(ukey(i, j));   // (those in the fill-in are dropped below)
        }
        const TRun bi = getb(i), bj = getb(j);
        const TRun c = pool.lin2(0.5, bi, 0.5 * sg, bj);
        Eb.put(i, c);
        Eb.put(j, (sg > 0) ? c : pool.lin2(-1.0, c, 0.0, none));
    }
    tr.mark("    pbc composition");
    std::sort(fill.begin(), fill.end());
    fill.erase(std::unique(fill.begin(), fill.end()), fill.end());
    P->pbc_fill = fill;
    auto flatten = [&](const RunMap &M, std::vector<long long> &keys, std::vector<int> &ptr, std::vector<Term> &terms) {
        const auto o = M.sorted();
        keys.resize(o.size());
        ptr.assign(1, 0);
        ptr.reserve(o.size() + 1);
        terms.clear();
        for (size_t m = 0; m < o.size(); ++m) {
            keys[m] = o[m].first;
            terms.insert(terms.end(), pool.t.begin() + o[m].second.off,
                         pool.t.begin() + o[m].second.off + o[m].second.len);
            ptr.push_back((int)terms.size());
        }
    };
    flatten(E, P->pbc_entry_key, P->pbc_entry_ptr, P->pbc_entry_terms);
    if (aux) {
        flatten(Ea, P->pbca_entry_key, P->pbca_entry_ptr, P->pbca_entry_terms);
    } else {
        P->pbca_entry_key.clear();
        P->pbca_entry_ptr.assign(1, 0);
        P->pbca_entry_terms.clear();
    }
    std::sort(afill.begin(), afill.end());
    afill.erase(std::unique(afill.begin(), afill.end()), afill.end());
    P->pbca_fill.clear();
    for (long long k : afill)
        if (!std::binary_search(fill.begin(), fill.end(), k)) P->pbca_fill.push_back(k);
    {
        const auto o = Eb.sorted();
        P->pbc_b_key.resize(o.size());
        P->pbc_b_ptr.assign(1, 0);
        P->pbc_b_terms.clear();
        for (size_t m = 0; m < o.size(); ++m) {
            P->pbc_b_key[m] = (int)o[m].first;
            for (unsigned u = 0; u < o[m].second.len; ++u) {
                const Term &t = pool.t[o[m].second.off + u];
                P->pbc_b_terms.push_back({(int)t.first, t.second});
            }
            P->pbc_b_ptr.push_back((int)P->pbc_b_terms.size());
        }
    }
    tr.mark("    pbc sorted output");
    return XFK_OK;
}


// Air-gap couplings that no triangle provides join the CSR pattern through the
// fill-in list (merged with the periodic fill-in).
static void add_age_fill(xfk_problem *P)
{
    if (P->age_key.empty()) return;
    std::unordered_map<int, std::set<int>> adj;
    std::vector<char> isage(std::max(1, P->NL), 0);
    for (long long k : P->age_key) {
        const int r = (int)(k >> 32), c = (int)(k & 0xffffffff);
        if (r != c) {
            adj[r];
            adj[c];
            if (r >= 0 && r < P->NL) isage[r] = 1;
            if (c >= 0 && c < P->NL) isage[c] = 1;
        }
    }
    for (int e = 0; e < P->NE; ++e)
        for (int j = 0; j < 3; ++j) {
            const int v = P->hp[3 * e + j];
            if (v < 0 || v >= P->NL || !isage[v]) continue;
            auto it = adj.find(v);
            for (int m = 0; m < 3; ++m)
                if (m != j) it->second.insert(P->hp[3 * e + m]);
        }
    std::set<long long> fill(P->pbc_fill.begin(), P->pbc_fill.end());
    for (long long k : P->age_key) {
        const int r = (int)(k >> 32), c = (int)(k & 0xffffffff);
        if (r != c && !adj[r].count(c)) fill.insert(k);
    }
    P->pbc_fill.assign(fill.begin(), fill.end());
}

// device -> host read-back ordered on the problem's (non-blocking) stream
hipError_t d2h(void *dst, const void *src, size_t bytes, hipStream_t s)
{
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

// hipcub temporary storage, kept on the problem (no hipMalloc/hipFree per call)
static hipError_t cub_scratch(xfk_problem *P, size_t bytes, void **out)
{
    hipError_t e = P->cub_tmp.alloc(bytes ? bytes : 1);
    *out = P->cub_tmp.p;
    return e;
}

static hipError_t exclusive_scan(xfk_problem *P, const int *in, int *out, int n)
{
    // out has n+1 entries; out[n] = total
    hipStream_t s = P->stream;
    void *tmp = nullptr;
    size_t bytes = 0;
    hipError_t e = hipcub::DeviceScan::InclusiveSum(tmp, bytes, in, out + 1, n, s);
    if (e == hipSuccess) e = cub_scratch(P, bytes, &tmp);
    if (e == hipSuccess) e = hipMemsetAsync(out, 0, sizeof(int), s);
    if (e == hipSuccess) e = hipcub::DeviceScan::InclusiveSum(tmp, bytes, in, out + 1, n, s);
    return e;
}

static int alloc_cg(xfk_problem *P);

// Temporaries of the symbolic phase, carved from one persistent device buffer
// (P->sym_tmp) so that a rebuild performs no hipMalloc/hipFree.
struct SymTmp {
    static constexpr int kMaxRounds = 4096;
    static constexpr int kMaxColors = 128;
    // zero-initialised block (one memset)
    int *deg, *cursor, *cnt, *hist;
    // uninitialised
    int *rowcnt, *keys_out, *iota, *flag, *iperm, *rowtmp, *slot_val, *slot_key;
    unsigned char *active;
    unsigned long long *maxkey, *used;
    size_t zero_bytes = 0, bytes = 0;

    void carve(char *base, int N, int NE, int nfill)
    {
        size_t off = 0;
        auto take = [&](auto *&ptr, size_t n) {
            using T = std::remove_reference_t<decltype(*ptr)>;
            off = (off + 255) & ~size_t(255);
            ptr = base ? reinterpret_cast<T *>(base + off) : nullptr;
            off += (n ? n : 1) * sizeof(T);
        };
        take(deg, N);
        take(cursor, N);
        take(cnt, 4);
        take(hist, kMaxColors + 1);
        zero_bytes = off;
        take(rowcnt, N);
        take(active, N);
        take(keys_out, NE);
        take(iota, NE);
        take(flag, N);
        take(maxkey, N);
        take(used, 2 * (size_t)N);
        take(iperm, NE);
        take(slot_val, 3 * (size_t)NE);
        take(slot_key, 3 * (size_t)NE);
        take(rowtmp, (size_t)row_tmp_size(N, NE, nfill));
        bytes = off;
    }
};

// the CSR lengths of a deferred symbolic phase (build_symbolic), read once
int xfk_resolve_nnz(xfk_problem *P)
{
    if (!P->nnz_pending) return XFK_OK;
    XFK_CHECK(hipEventSynchronize(P->nnz_ev));
    P->nnz = P->hpin[0];
    P->nnz_own = P->hpin[1];
    P->row_max = P->hpin[5];
    P->nnz_pending = false;
    return XFK_OK;
}

int build_symbolic(xfk_problem *P)
{
    hipStream_t s = P->stream;
    P->ts.B = 0;   // the exchange-overlap tile split follows the pattern
    const int N = P->NR, NL = P->NL, NE = P->NE;   // assembled rows, local nodes, local elements
    SymTmp T;
    // periodic fill-in (+ the auxiliary matrices' (i, j) entries of the Newton AC solver)
    std::vector<long long> fillv = P->pbc_fill;
    if (P->harmonic && P->ac_solver == 1) fillv.insert(fillv.end(), P->pbca_fill.begin(), P->pbca_fill.end());
    const int nfill = 2 * (int)fillv.size();
    T.carve(nullptr, NL, NE, nfill);
    XFK_CHECK(P->sym_tmp.alloc(T.bytes));
    T.carve(P->sym_tmp.p, NL, NE, nfill);
    XFK_CHECK(hipMemsetAsync(P->sym_tmp.p, 0, T.zero_bytes, s));

    // node -> incident elements
    XFK_CHECK(P->n2e_ptr.alloc(NL + 1));
    XFK_CHECK(P->n2e.alloc(3 * (size_t)NE));
    // counts, scan, fill, per-node register sort (xfk_device.hip k_n2e_*):
    // each node's elements ascending (the reference's AddTo order);
    // XFK_N2E_RADIX=1: the stable radix sort of the element-major incidence
    // slots by node instead (same lists)
    static const bool n2e_radix = [] {
        const char *e = std::getenv("XFK_N2E_RADIX");
        return e && std::atoi(e) != 0;
    }();
    if (!n2e_radix) {
        launch_n2e_count(s, NE, P->p_raw.p, T.deg);
        XFK_CHECK(exclusive_scan(P, T.deg, P->n2e_ptr.p, NL));
        launch_n2e_fill(s, NE, P->p_raw.p, P->n2e_ptr.p, T.cursor, P->n2e.p);
        launch_n2e_sort(s, N, NL, P->n2e_ptr.p, P->n2e.p);   // rows < N: sorted by the row-length pass
    } else {
        launch_slot_elements(s, NE, T.slot_val);
        int bits = 1;
        while (bits < 31 && (1LL << bits) <= NL) ++bits;
        void *tmp = nullptr;
        size_t bytes = 0;
        const int n3 = 3 * NE;
        XFK_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, P->p_raw.p, T.slot_key, T.slot_val, P->n2e.p, n3, 0,
                                                     bits, s));
        XFK_CHECK(cub_scratch(P, bytes, &tmp));
        XFK_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, P->p_raw.p, T.slot_key, T.slot_val, P->n2e.p, n3, 0,
                                                     bits, s));
        launch_n2e_ptr(s, NL, T.slot_key, n3, P->n2e_ptr.p);
    }

    // periodic fill-in entries, CSR by row
    const int *fp = nullptr, *fc = nullptr;
    if (!fillv.empty()) {
        std::vector<std::vector<int>> rows(N);
        for (long long k : fillv) {
            int r = (int)(k >> 32), c = (int)(k & 0xffffffff);
            if (r < N) rows[r].push_back(c);   // rows beyond the assembled ones do not exist
            if (c < N) rows[c].push_back(r);
        }
        std::vector<int> hptr(N + 1, 0), hcol;
        for (int r = 0; r < N; ++r) {
            std::sort(rows[r].begin(), rows[r].end());
            hptr[r + 1] = hptr[r] + (int)rows[r].size();
            hcol.insert(hcol.end(), rows[r].begin(), rows[r].end());
        }
        XFK_CHECK(upload(P->fill_ptr, hptr.data(), hptr.size(), s));
        XFK_CHECK(upload(P->fill_col, hcol.data(), hcol.size(), s));
        XFK_CHECK(hipStreamSynchronize(s));
        fp = P->fill_ptr.p;
        fc = P->fill_col.p;
    }

    // CSR pattern
    XFK_CHECK(P->rowptr.alloc(N + 1));
    launch_row_build(s, N, P->p_raw.p, P->n2e_ptr.p, P->n2e.p, fp, fc, T.rowtmp, T.rowcnt, n2e_radix ? nullptr : P->n2e.p);
    XFK_CHECK(exclusive_scan(P, T.rowcnt, P->rowptr.p, N));
    XFK_CHECK(hipMemcpyAsync(P->hpin, P->rowptr.p + N, sizeof(int), hipMemcpyDeviceToHost, s));
    XFK_CHECK(hipMemcpyAsync(P->hpin + 1, P->rowptr.p + P->N, sizeof(int), hipMemcpyDeviceToHost, s));
    // the longest row, read with the lengths: a fresh AMG hierarchy sizes its
    // SpGEMM capacities from it (Amg::seed_hints) instead of measuring each
    // product list behind a host check
    P->hpin[5] = 0;
    if (!P->harmonic && N > 0 && P->amg && P->amg->cap_hint.empty()) {
        void *tmp = nullptr;
        size_t bytes = 0;
        XFK_CHECK(hipcub::DeviceReduce::Max(tmp, bytes, T.rowcnt, T.cnt + 3, N, s));
        XFK_CHECK(cub_scratch(P, bytes, &tmp));
        XFK_CHECK(hipcub::DeviceReduce::Max(tmp, bytes, T.rowcnt, T.cnt + 3, N, s));
        XFK_CHECK(hipMemcpyAsync(P->hpin + 5, T.cnt + 3, sizeof(int), hipMemcpyDeviceToHost, s));
    }
    // static problems without air gaps or periodic maps read
    // the lengths back later (xfk_resolve_nnz, at the preconditioner setup):
    // the pattern is filled and the matrix assembled into arrays sized for
    // the bound 6 NE + N + fill-in (a triangle adds at most six off-diagonal
    // entries), with no host check in between
    // (deferred only while the bound's col / val stay within 512 MB: on larger
    // meshes the one host check is negligible next to the memory the bound
    // would hold, ~0.7 GB on the configs[4] mesh)
    const long long bound_nnz = 6LL * NE + N + nfill;
    // (a sharded rank defers too: its halo plan was made at creation, and the
    // lengths are first needed by the AMG setup, after the assembly)
    const bool defer = !P->harmonic && P->age_key.empty() && P->pbc_entry_key.empty() &&
                       bound_nnz * 12 <= (512LL << 20);
    long long cap_nnz;
    if (defer) {
        if (!P->nnz_ev) XFK_CHECK(hipEventCreateWithFlags(&P->nnz_ev, hipEventDisableTiming));
        XFK_CHECK(hipEventRecord(P->nnz_ev, s));
        P->nnz_pending = true;
        cap_nnz = bound_nnz;
    } else {
        XFK_CHECK(hipStreamSynchronize(s));
        P->nnz = P->hpin[0];
        P->nnz_own = P->hpin[1];
        P->row_max = P->hpin[5];
        P->nnz_pending = false;
        cap_nnz = P->nnz;
    }
    XFK_CHECK(P->col.alloc(cap_nnz));
    XFK_CHECK(P->val.alloc(cap_nnz));
    XFK_CHECK(P->diag.alloc(N));
    launch_row_copy(s, N, P->p_raw.p, P->n2e_ptr.p, P->n2e.p, fp, fc, T.rowtmp, P->rowptr.p, P->col.p, P->diag.p);

    // The static path assembles by rows (k_assemble_rows): no colouring.  The
    // time-harmonic path still scatters by colour: Jones-Plassmann colouring
    // of elements (shared node = conflict) over full-array sweeps (kernels in
    // xfk_device.hip); the host checks for completion every kSyncRounds rounds.
    P->ncolors = 0;
    P->color_rounds = 0;
    if (P->harmonic) {
    XFK_CHECK(P->color.alloc(NE));
    XFK_CHECK(hipMemsetAsync(P->color.p, 0xff, sizeof(int) * NE, s));
    constexpr int kSyncRounds = 6;
    XFK_CHECK(hipMemsetAsync(T.active, 1, (size_t)NL, s));
    int round = 0, last = 0;
    for (;;) {
        XFK_REQUIRE(round < SymTmp::kMaxRounds, XFK_ERR_UNSUPPORTED, "element colouring did not terminate");
        for (int k = 0; k < kSyncRounds; ++k, ++round)
            launch_jp_round(s, NL, NE, round, T.active, T.cnt + 2, P->p_raw.p, P->n2e_ptr.p, P->n2e.p, P->color.p,
                            T.maxkey, T.used);
        XFK_CHECK(d2h(&last, T.cnt + 2, sizeof(int), s));
        if (last < round) break;       // the last round launched left nothing pending
    }
    round = last + 1;                  // rounds that coloured something
    P->color_rounds = round;
    const int maxc = SymTmp::kMaxColors;
    launch_color_hist(s, NE, P->color.p, T.hist, maxc);
    std::vector<int> hh(maxc + 1);
    XFK_CHECK(d2h(hh.data(), T.hist, sizeof(int) * (maxc + 1), s));
    XFK_REQUIRE(hh[maxc] == 0, XFK_ERR_UNSUPPORTED, "more than 128 element colours needed");
    int nc = 0;
    for (int c = 0; c < maxc; ++c)
        if (hh[c]) nc = c + 1;
    P->ncolors = nc;
    P->color_off.assign(nc + 1, 0);
    for (int c = 0; c < nc; ++c) P->color_off[c + 1] = P->color_off[c] + hh[c];

    // stable sort of elements by colour -> perm (colour order -> raw element)
    XFK_CHECK(P->perm.alloc(NE));
    launch_iota(s, NE, T.iota);
    {
        void *tmp = nullptr;
        size_t bytes = 0;
        XFK_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, P->color.p, T.keys_out, T.iota, P->perm.p, NE, 0,
                                                     8, s));
        XFK_CHECK(cub_scratch(P, bytes, &tmp));
        XFK_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, P->color.p, T.keys_out, T.iota, P->perm.p, NE, 0,
                                                     8, s));
    }
    XFK_CHECK(P->erec.alloc(NE));
    XFK_CHECK(P->ebits.alloc(NE));
    XFK_CHECK(P->slot.alloc(9 * (size_t)NE));
    launch_build_erec(s, NE, P->perm.p, P->p_raw.p, P->lbl_raw.p, P->ebits_raw.p, P->erec.p, P->ebits.p, T.iperm);
    launch_build_slots(s, NE, N, P->p_raw.p, T.iperm, P->rowptr.p, P->col.p, P->slot.p, T.cnt);
    }

    // rows adjacent to fixed nodes
    launch_mark_fix_adj(s, N, P->rowptr.p, P->col.p, P->fixed.p, T.flag);
    XFK_CHECK(P->fix_cols_row.alloc(N));
    launch_compact_flags(s, N, T.flag, T.cnt + 1, P->fix_cols_row.p);
    if (P->harmonic) {   // (its Dirichlet kernels and the slot check read the counts on the host)
        XFK_CHECK(hipMemcpyAsync(P->hpin + 2, T.cnt, sizeof(int) * 2, hipMemcpyDeviceToHost, s));
        XFK_CHECK(hipStreamSynchronize(s));
        const int hc[2] = {P->hpin[2], P->hpin[3]};
        XFK_REQUIRE(hc[0] == 0, XFK_ERR_HIP, "internal: element slot missing from the CSR pattern");
        P->nfix_cols = hc[1];
    } else {             // static paths: the count stays on the device (no host check)
        XFK_CHECK(P->nfix_dev.alloc(1));
        XFK_CHECK(hipMemcpyAsync(P->nfix_dev.p, T.cnt + 1, sizeof(int), hipMemcpyDeviceToDevice, s));
        P->nfix_cols = -1;
    }
    XFK_CHECK(P->mu1.alloc(NE));
    XFK_CHECK(P->mu2.alloc(NE));
    if (!P->harmonic) {
        XFK_CHECK(P->mu1b.alloc(NE));
        XFK_CHECK(P->mu2b.alloc(NE));
        if (P->any_nonlinear && !P->axi) {
            XFK_CHECK(P->dv_el.alloc(NE));
            XFK_CHECK(P->on_el.alloc(NE));
        }
        XFK_CHECK(P->asm_miss.alloc(1));
        XFK_CHECK(hipMemsetAsync(P->asm_miss.p, 0, sizeof(int), s));
        P->miss_checked = false;
    }

    // air-gap entries -> CSR slots (full storage: both triangles)
    P->age_n = 0;
    if (!P->age_key.empty()) {
        std::vector<int> rc;
        std::vector<double> v;
        for (size_t m = 0; m < P->age_key.size(); ++m) {
            const int r = (int)(P->age_key[m] >> 32), c = (int)(P->age_key[m] & 0xffffffff);
            rc.push_back(r); rc.push_back(c); v.push_back(P->age_val[m]);
            if (r != c) { rc.push_back(c); rc.push_back(r); v.push_back(P->age_val[m]); }
        }
        const int na = (int)v.size();
        DBuf<int> d_rc;
        XFK_CHECK(upload(d_rc, rc.data(), rc.size(), s));
        XFK_CHECK(upload(P->age_v, v.data(), v.size(), s));
        XFK_CHECK(P->age_slot.alloc(na));
        launch_lookup_slots(s, na, d_rc.p, P->rowptr.p, P->col.p, P->age_slot.p);
        std::vector<int> chk(na);
        XFK_CHECK(d2h(chk.data(), P->age_slot.p, sizeof(int) * na, s));
        for (int x : chk) XFK_REQUIRE(x >= 0, XFK_ERR_HIP, "internal: air-gap slot missing from the CSR pattern");
        P->age_n = na;
    }

    // periodic averaging maps -> CSR slots
    P->pm_n = 0;
    P->pb_n = 0;
    if (!P->pbc_entry_key.empty()) {
        std::vector<int> rc_dst, dst_owner, src_rc, ptr{0};
        std::vector<double> w;
        for (size_t m = 0; m < P->pbc_entry_key.size(); ++m) {
            long long k = P->pbc_entry_key[m];
            int r = (int)(k >> 32), c = (int)(k & 0xffffffff);
            const int t0 = P->pbc_entry_ptr[m], t1 = P->pbc_entry_ptr[m + 1];
            // one gather entry per destination slot (both triangles) in an
            // assembled row; a source (symmetric before the map) is read in
            // whichever orientation lies in an assembled row -- one of its
            // indices is always a coupled node (assembled on every rank)
            int ndst = (r == c) ? 1 : 2;
            for (int d = 0; d < ndst; ++d) {
                const int dr = d == 0 ? r : c, dc = d == 0 ? c : r;
                if (dr >= N) continue;
                rc_dst.push_back(dr);
                rc_dst.push_back(dc);
                for (int u = t0; u < t1; ++u) {
                    const auto &t = P->pbc_entry_terms[u];
                    const int a = (int)(t.first >> 32), b2 = (int)(t.first & 0xffffffff);
                    src_rc.push_back(a < N ? a : b2);
                    src_rc.push_back(a < N ? b2 : a);
                    w.push_back(t.second);
                }
                ptr.push_back((int)w.size());
            }
        }
        int nd = (int)rc_dst.size() / 2, ns = (int)w.size();
        DBuf<int> d_rc, s_rc;
        XFK_CHECK(upload(d_rc, rc_dst.data(), rc_dst.size(), s));
        XFK_CHECK(upload(s_rc, src_rc.data(), src_rc.size(), s));
        XFK_CHECK(P->pm_dst.alloc(nd));
        XFK_CHECK(P->pm_src.alloc(ns ? ns : 1));
        launch_lookup_slots(s, nd, d_rc.p, P->rowptr.p, P->col.p, P->pm_dst.p);
        launch_lookup_slots(s, ns, s_rc.p, P->rowptr.p, P->col.p, P->pm_src.p);
        XFK_CHECK(upload(P->pm_ptr, ptr.data(), ptr.size(), s));
        XFK_CHECK(upload(P->pm_w, w.data(), w.size(), s));
        XFK_CHECK(P->pm_tmp.alloc(nd));
        XFK_CHECK(hipStreamSynchronize(s));
        // every slot must exist
        std::vector<int> chk(nd), chk2(ns);
        XFK_CHECK(d2h(chk.data(), P->pm_dst.p, sizeof(int) * nd, s));
        if (ns) XFK_CHECK(d2h(chk2.data(), P->pm_src.p, sizeof(int) * ns, s));
        for (int v : chk) XFK_REQUIRE(v >= 0, XFK_ERR_HIP, "internal: periodic map slot missing");
        for (int v : chk2) XFK_REQUIRE(v >= 0, XFK_ERR_HIP, "internal: periodic map source slot missing");
        P->pm_n = nd;

        std::vector<int> bd, bsrc, bptr{0};
        std::vector<double> bw;
        for (size_t m = 0; m < P->pbc_b_key.size(); ++m) {
            bd.push_back(P->pbc_b_key[m]);
            for (int u = P->pbc_b_ptr[m]; u < P->pbc_b_ptr[m + 1]; ++u) {
                const auto &t = P->pbc_b_terms[u];
                bsrc.push_back(t.first);
                bw.push_back(t.second);
            }
            bptr.push_back((int)bw.size());
        }
        XFK_CHECK(upload(P->pb_dst, bd.data(), bd.size(), s));
        XFK_CHECK(upload(P->pb_src, bsrc.data(), bsrc.size(), s));
        XFK_CHECK(upload(P->pb_ptr, bptr.data(), bptr.size(), s));
        XFK_CHECK(upload(P->pb_w, bw.data(), bw.size(), s));
        XFK_CHECK(P->pb_tmp.alloc(bd.size()));
        XFK_CHECK(hipStreamSynchronize(s));
        P->pb_n = (int)bd.size();
    }

    // the auxiliary matrices' map (Newton AC solver): ordered entries, one gather per slot
    P->pa_n = 0;
    if (P->harmonic && P->ac_solver == 1 && !P->pbca_entry_key.empty()) {
        std::vector<int> rc_dst, src_rc, ptr{0};
        std::vector<double> w;
        for (size_t m = 0; m < P->pbca_entry_key.size(); ++m) {
            const long long k = P->pbca_entry_key[m];
            // (sharded: an entry of a row assembled elsewhere -- a neighbour of a
            // coupled node in the halo -- is that rank's; its terms lie in its own
            // row, the rows of the kept entries' terms are all assembled here)
            if ((int)(k >> 32) >= N) continue;
            rc_dst.push_back((int)(k >> 32));
            rc_dst.push_back((int)(k & 0xffffffff));
            for (int u = P->pbca_entry_ptr[m]; u < P->pbca_entry_ptr[m + 1]; ++u) {
                const auto &t = P->pbca_entry_terms[u];
                src_rc.push_back((int)(t.first >> 32));
                src_rc.push_back((int)(t.first & 0xffffffff));
                w.push_back(t.second);
            }
            ptr.push_back((int)w.size());
        }
        const int nd = (int)rc_dst.size() / 2, ns = (int)w.size();
        DBuf<int> d_rc, s_rc;
        XFK_CHECK(upload(d_rc, rc_dst.data(), rc_dst.size(), s));
        XFK_CHECK(upload(s_rc, src_rc.data(), src_rc.size(), s));
        XFK_CHECK(P->pa_dst.alloc(nd));
        XFK_CHECK(P->pa_src.alloc(ns ? ns : 1));
        launch_lookup_slots(s, nd, d_rc.p, P->rowptr.p, P->col.p, P->pa_dst.p);
        launch_lookup_slots(s, ns, s_rc.p, P->rowptr.p, P->col.p, P->pa_src.p);
        XFK_CHECK(upload(P->pa_ptr, ptr.data(), ptr.size(), s));
        XFK_CHECK(upload(P->pa_w, w.data(), w.size(), s));
        XFK_CHECK(P->pa_tmp.alloc(nd));
        std::vector<int> chk(nd), chk2(ns);
        XFK_CHECK(d2h(chk.data(), P->pa_dst.p, sizeof(int) * nd, s));
        if (ns) XFK_CHECK(d2h(chk2.data(), P->pa_src.p, sizeof(int) * ns, s));
        for (int v : chk) XFK_REQUIRE(v >= 0, XFK_ERR_HIP, "internal: auxiliary periodic map slot missing");
        for (int v : chk2) XFK_REQUIRE(v >= 0, XFK_ERR_HIP, "internal: auxiliary periodic map source slot missing");
        P->pa_n = nd;
    }

    // vectors and reduction scratch
    for (DBuf<double> *v : {&P->b, &P->P, &P->dinv}) XFK_CHECK(v->alloc(N));   // (N = assembled rows here)
    for (DBuf<double> *v : {&P->V, &P->Vold}) XFK_CHECK(v->alloc(NL));
    XFK_CHECK(P->partials.alloc(2 * kRedGrid));
    XFK_CHECK(P->counters.alloc(8));
    XFK_CHECK(hipMemsetAsync(P->counters.p, 0, sizeof(unsigned) * 8, s));
    XFK_CHECK(P->pcg.alloc(1));
    XFK_CHECK(P->nws.alloc(1));
    int rc2 = alloc_cg(P);
    if (rc2 != XFK_OK) return rc2;
    // (no host check: the host reads nothing more of this phase; host-side
    // staging vectors above were uploaded synchronously or checked already)
    P->symbolic_ready = true;
    return XFK_OK;
}

// numeric assembly + boundary conditions for Newton iteration `iter`
static int assemble(xfk_problem *P, int iter)
{
    hipStream_t s = P->stream;
    AssembleArgs A = {};
    A.erec = P->erec.p;
    A.ebits = P->ebits.p;
    A.slot = P->slot.p;
    A.x = P->x.p;
    A.y = P->y.p;
    A.labels = P->labels.p;
    A.blocks = P->blocks.p;
    A.lines = P->lines.p;
    A.circs = P->circs.p;
    A.bhB = P->bhB.p;
    A.bhH = P->bhH.p;
    A.bhS = P->bhS.p;
    A.mu1 = P->mu1.p;
    A.mu2 = P->mu2.p;
    A.V = P->V.p;
    A.val = P->val.p;
    A.b = P->b.p;
    A.iter = iter;
    A.axi = P->axi ? 1 : 0;
    A.ext_ro = P->ext_ro;
    A.ext_ri = P->ext_ri;
    A.ext_zo = P->ext_zo;
    A.p_raw = P->p_raw.p;
    A.lbl_raw = P->lbl_raw.p;
    A.ebits_raw = P->ebits_raw.p;
    A.n2e_ptr = P->n2e_ptr.p;
    A.n2e = P->n2e.p;
    A.rowptr = P->rowptr.p;
    A.col = P->col.p;
    // (a linear problem never reads the permeability state back)
    A.mu1_out = P->any_nonlinear ? P->mu1b.p : nullptr;
    A.mu2_out = P->any_nonlinear ? P->mu2b.p : nullptr;
    A.miss = P->asm_miss.p;
    // (XFK_ASM_STATE=0: the Newton state evaluated per row, as before -- measurement / the test)
    const char *st = std::getenv("XFK_ASM_STATE");
    const bool pre = P->any_nonlinear && !P->axi && P->dv_el.p && !(st && std::atoi(st) == 0);
    A.dv_el = pre ? P->dv_el.p : nullptr;
    A.on_el = pre ? P->on_el.p : nullptr;
    A.n_el = P->NE;
    launch_assemble_rows(s, P->NR, A);   // writes every entry of val and b (assembled rows)
    std::swap(P->mu1.p, P->mu1b.p);     // the state just written is read next iteration
    std::swap(P->mu1.n, P->mu1b.n);
    std::swap(P->mu2.p, P->mu2b.p);
    std::swap(P->mu2.n, P->mu2b.n);
    launch_add_at_slots(s, P->age_n, P->age_slot.p, P->age_v.p, P->val.p);   // air-gap elements
    launch_point_currents(s, P->npt, P->pt_nodes.p, P->pt_J.p, P->b.p);
    launch_dirichlet(s, P->nfix_rows, P->fix_rows.p, P->nfix_cols, P->nfix_dev.p, P->N, P->fix_cols_row.p,
                     P->rowptr.p, P->col.p, P->diag.p, P->fixed.p, P->fix_first.p, P->fix_last.p, P->val.p, P->b.p);
    launch_map(s, P->pm_n, P->pm_dst.p, P->pm_ptr.p, P->pm_src.p, P->pm_w.p, P->val.p, P->pm_tmp.p);
    launch_map(s, P->pb_n, P->pb_dst.p, P->pb_ptr.p, P->pb_src.p, P->pb_w.p, P->b.p, P->pb_tmp.p);
    XFK_CHECK(hipGetLastError());
    return XFK_OK;
}

// CBigLinProb::PCGSolve(flag) on the assembled system (Jacobi-preconditioned,
// two launches per iteration: xfk_pcg.hip).  Sharded: the halo of u is
// exchanged before every SpMV and the per-block partials are all-reduced
// (elementwise, so every rank then sums identical arrays in the same order and
// takes bit-identical alpha, beta and stopping decisions).
static int alloc_cg(xfk_problem *P)
{
    const int N = P->N, NL = P->NL;
    int G = std::max(cg_grid(N), cg_axpy_grid(N));
    if (P->comm)
        for (int q = 0; q < P->nranks; ++q) {
            const int nq = (int)(row_begin(P->N_global, q + 1, P->nranks) - row_begin(P->N_global, q, P->nranks));
            G = std::max(G, std::max(cg_grid(nq), cg_axpy_grid(nq)));
        }
    P->Gpart = G;
    XFK_CHECK(P->R2.alloc((size_t)N));            // r
    XFK_CHECK(P->W2.alloc((size_t)N));            // w = A u
    XFK_CHECK(P->Z2.alloc((size_t)N + NL));       // z (N), then u = M^-1 r (NL, halo last)
    XFK_CHECK(P->part_loc.alloc(4 * (size_t)G));
    if (P->comm) {
        XFK_CHECK(P->part_glob_buf.alloc(4 * (size_t)G));
        P->part_glob = P->part_glob_buf.p;
    } else {
        P->part_glob = P->part_loc.p;
    }
    return XFK_OK;
}

static CgAxpyArgs cg_args(xfk_problem *P, long long it)
{
    const int N = P->N;
    const size_t G = (size_t)P->Gpart;
    CgAxpyArgs A;
    A.W = P->W2.p;
    A.dinv = P->dinv.p;
    A.Z = P->Z2.p;
    A.U = P->Z2.p + N;
    A.P = P->P.p;
    A.V = P->V.p;
    A.R = P->R2.p;
    A.gam_in = P->part_glob + (size_t)(it & 1) * G;
    A.gam_out = P->part_loc.p + (size_t)((it + 1) & 1) * G;
    A.del_in = P->part_glob + 2 * G;
    A.reso = P->part_glob + 3 * G;
    A.amg = P->pc_used == XFK_PRECOND_AMG;
    if (P->comm) {
        A.Ggam = A.Gdel = (int)G;     // zero beyond this rank's grids
    } else {
        A.Ggam = (it == 0 || A.amg) ? cg_grid(N) : cg_axpy_grid(N);
        A.Gdel = cg_grid(N);
    }
    A.S = P->pcg.p;
    A.it = it;
    A.N = N;
    return A;
}

// sum of a host scalar over the ranks (setup-time decisions that must agree)
int allreduce_host(xfk_problem *P, double &v)
{
    if (!P->comm) return XFK_OK;
    hipStream_t s = P->stream;
    XFK_CHECK(P->nws_glob.alloc(4));
    XFK_CHECK(hipMemcpyAsync(P->nws_glob.p, &v, sizeof(double), hipMemcpyHostToDevice, s));
    int rc = P->comm->allreduce_sum(P->nws_glob.p, P->nws_glob.p + 2, 1, s);
    if (rc != XFK_OK) return rc;
    return d2h(&v, P->nws_glob.p + 2, sizeof(double), s) == hipSuccess ? XFK_OK : XFK_ERR_HIP;
}

int allreduce_host_n(xfk_problem *P, double *v, int n)
{
    if (!P->comm || n <= 0) return XFK_OK;
    hipStream_t s = P->stream;
    XFK_CHECK(P->nws_glob.alloc(2 * (size_t)std::max(n, 2)));
    XFK_CHECK(hipMemcpyAsync(P->nws_glob.p, v, sizeof(double) * n, hipMemcpyHostToDevice, s));
    int rc = P->comm->allreduce_sum(P->nws_glob.p, P->nws_glob.p + n, (size_t)n, s);
    if (rc != XFK_OK) return rc;
    return d2h(v, P->nws_glob.p + n, sizeof(double) * n, s) == hipSuccess ? XFK_OK : XFK_ERR_HIP;
}

static int exchange(xfk_problem *P, double *vec)
{
    return P->comm ? P->comm->exchange(P->halo, vec, P->stream) : XFK_OK;
}

static int allreduce_partials(xfk_problem *P, int narrays)
{
    if (!P->comm) return XFK_OK;
    return P->comm->allreduce_sum(P->part_loc.p, P->part_glob, (size_t)narrays * P->Gpart, P->stream);
}

static bool trace_newton() { return std::getenv("XFK_TRACE_NEWTON") != nullptr; }
// XFK_NEWTON_INEXACT=0 turns the inexact Newton passes off (XFK_OPT_NEWTON_INEXACT)
static bool newton_inexact_env()
{
    const char *e = std::getenv("XFK_NEWTON_INEXACT");
    return !(e && e[0] == '0');
}

// a Newton refresh re-forms level 0's P~ (~0.32 ms on configs[3]) when the
// last pass ran at least this many PCG iterations, else level 0 runs
// unfolded for the pass; configs[3] per step with 0 / 12 / 16 / 20 / never:
// 19.32-19.44 / 19.03-19.25 / 19.11-19.13 / 19.06-19.09 / 18.96-19.33 ms
// (profiles/r04_experiments/r04z4_*) -- within noise of each other
constexpr int kRefoldMinIters = 16;

// AMG hierarchy of the assembled matrix (owned block when sharded); falls
// back to Jacobi for this solve when the hierarchy cannot be built
static int amg_setup(xfk_problem *P)
{
    const bool was_amg = P->pc_used == XFK_PRECOND_AMG;
    P->pc_used = XFK_PRECOND_JACOBI;
    P->amg_fresh = false;
    if (P->precond != XFK_PRECOND_AMG) return XFK_OK;
    hipStream_t s = P->stream;
    // later Newton iterations: same pattern, new values -> keep the hierarchy
    // while the PCG stays within 2x the iterations of the last fresh build
    // (the decision reads iteration counts every rank shares)
    if (P->amg_reuse && P->amg_reusable && was_amg && P->amg &&
        P->amg_last_iters <= std::max(2 * P->amg_fresh_iters, P->amg_fresh_iters + 8)) {
        // level 0 stays folded when the pass is expected to run long enough to
        // repay re-forming P~ (k_refold_p): the last pass's count as the guess
        // (XFK_REFOLD_MIN: that threshold)
        const char *rm = std::getenv("XFK_REFOLD_MIN");   // (read per refresh: tests set it)
        const int refold_min = rm ? std::atoi(rm) : kRefoldMinIters;
        int rc = P->amg->refresh(s, P->amg_last_iters >= refold_min);
        if (rc != XFK_OK) return rc;
        P->pc_used = XFK_PRECOND_AMG;
        return XFK_OK;
    }
    P->amg_reusable = false;
    if (!P->amg) P->amg = new Amg();
    P->amg->theta = P->amg_theta;
    P->amg->sweeps = P->amg_sweeps;
    P->amg->omega = P->amg_omega;
    P->amg->rep_rows = P->amg_replicate;
    P->amg->dense_max = P->amg_dense;
    P->amg->fold_on = P->amg_fold;
    P->amg->col16 = P->amg_col16;
    P->amg->prec32 = P->amg_f32;
    P->amg->wlevel = P->amg_wlevel;
    P->amg->row_max0 = P->row_max;
    // setup time: an event pair per setup, read after the solve's final
    // synchronisation (no host check here); callers that never read them
    // recycle the pairs; a full pool (> 64 fresh builds in one solve) is
    // read out first, so no recorded pair is overwritten unread
    if (P->setup_used >= 64) {
        XFK_CHECK(hipStreamSynchronize(s));
        for (int k = 0; k < P->setup_used; ++k) {
            float m = 0;
            XFK_CHECK(hipEventElapsedTime(&m, P->setup_ev[2 * k], P->setup_ev[2 * k + 1]));
            P->setup_ms_pending += m;
        }
        P->setup_used = 0;
    }
    if (P->setup_ev.size() < 2 * (P->setup_used + 1)) {
        P->setup_ev.resize(2 * (P->setup_used + 1), nullptr);
        for (auto &e : P->setup_ev)
            if (!e) XFK_CHECK(hipEventCreate(&e));
    }
    hipEvent_t e0 = P->setup_ev[2 * P->setup_used], e1 = P->setup_ev[2 * P->setup_used + 1];
    XFK_CHECK(hipEventRecord(e0, s));
    // sharded: rank-local aggregation, global coarse levels (Amg::setup_dist)
    int rc = (P->comm && P->comm->size > 1)
                 ? P->amg->setup_dist(s, P->comm, P->halo, P->N, P->NL - P->N, P->rowptr.p, P->col.p, P->val.p,
                                      P->nnz_own)
                 : P->amg->setup(s, P->N, P->N, P->rowptr.p, P->col.p, P->val.p, P->nnz_own);
    XFK_CHECK(hipEventRecord(e1, s));
    ++P->setup_used;
    double ok = (rc == XFK_OK) ? 0.0 : 1.0;   // every rank must take the same preconditioner
    if (rc != XFK_OK && rc != XFK_ERR_UNSUPPORTED) return rc;
    if (rc != XFK_OK && trace_newton()) std::fprintf(stderr, "[newton] AMG setup declined: %s\n", xfk_last_error());
    int rc2 = allreduce_host(P, ok);
    if (rc2 != XFK_OK) return rc2;
    if (ok == 0.0) {
        P->pc_used = XFK_PRECOND_AMG;
        P->amg_fresh = true;
        P->amg_reusable = true;
        P->last.amg_levels = P->amg->stats.levels;
        P->last.amg_op_complexity = P->amg->stats.op_complexity;
    }
    return XFK_OK;
}

// the 16-bit tile columns of the operator (built with the AMG hierarchy on a
// single device: the SpMV reads A's pattern through them), or nulls
static void spmv_col16(const xfk_problem *P, const unsigned short *&c16, const int *&cbase)
{
    c16 = nullptr;
    cbase = nullptr;
    if (P->pc_used != XFK_PRECOND_AMG || !P->amg || P->amg->L.empty()) return;
    const AmgLevel &L0 = *P->amg->L[0];
    if (!L0.has16 || L0.rowptr != P->rowptr.p || L0.col != P->col.p) return;
    c16 = L0.a16.p;
    cbase = L0.a16b.p;
}

static int pcg_start(xfk_problem *P, int flag)
{
    hipStream_t s = P->stream;
    const int N = P->N;
    *P->pcg_host = CgState{};   // pinned: the upload does not stage through the host
    const double tol = P->pcg_tol > 0 ? P->pcg_tol : P->precision;
    P->pcg_host->tol = tol;
    P->pcg_host->tol_rel = P->pcg_tol_rel;
    launch_cg_state_init(s, P->pcg.p, tol, P->pcg_tol_rel);
    if (P->comm) XFK_CHECK(hipMemsetAsync(P->part_loc.p, 0, sizeof(double) * 4 * P->Gpart, s));
    launch_diag_inv(s, N, P->diag.p, P->val.p, P->dinv.p, P->pcg.p);
    int rc = XFK_OK;
    if (P->comm) {   // every rank must agree before the collective setup
        XFK_CHECK(hipMemcpyAsync(P->pcg_host, P->pcg.p, sizeof(CgState), hipMemcpyDeviceToHost, s));
        XFK_CHECK(hipStreamSynchronize(s));
        double singular = P->pcg_host->singular ? 1.0 : 0.0;
        rc = allreduce_host(P, singular);
        if (rc != XFK_OK) return rc;
        if (singular != 0.0) {
            set_error("singular flag tripped: zero diagonal entry in the assembled matrix");
            return XFK_ERR_SINGULAR;
        }
    }
    // (one device: the singular flag is read with the PCG's first poll)
    if ((rc = amg_setup(P)) != XFK_OK) return rc;
    const CgAxpyArgs A0 = cg_args(P, 0);
    const size_t G = (size_t)P->Gpart;
    if (flag && (rc = exchange(P, P->V.p)) != XFK_OK) return rc;
    launch_cg_init_r(s, N, flag, P->rowptr.p, P->col.p, P->val.p, P->b.p, P->V.p, A0.R, A0.U, A0.Z, A0.P, P->dinv.p,
                     P->part_loc.p + 3 * G, P->part_loc.p);
    if (P->pc_used == XFK_PRECOND_AMG) {
        // u0 = M^-1 r0; res_o = (M^-1 b).b (one more V-cycle when x0 != 0)
        if ((rc = P->amg->vcycle(s, A0.R, A0.U, nullptr)) != XFK_OK) return rc;
        if (flag) {
            if ((rc = P->amg->vcycle(s, P->b.p, P->W2.p, nullptr)) != XFK_OK) return rc;
            launch_cg_dot(s, N, P->b.p, P->W2.p, P->part_loc.p + 3 * G);
        } else {
            launch_cg_dot(s, N, P->b.p, A0.U, P->part_loc.p + 3 * G);
        }
        if ((rc = exchange(P, A0.U)) != XFK_OK) return rc;
        const unsigned short *c16;
        const int *cbase;
        spmv_col16(P, c16, cbase);
        launch_cg_spmv(s, N, P->rowptr.p, P->col.p, P->val.p, A0.U, P->W2.p, P->part_loc.p + 2 * G, nullptr, A0.R,
                       P->part_loc.p, nullptr, 0, c16, cbase);
        return allreduce_partials(P, 4);
    }
    if ((rc = exchange(P, A0.U)) != XFK_OK) return rc;
    launch_cg_spmv(s, N, P->rowptr.p, P->col.p, P->val.p, A0.U, P->W2.p, P->part_loc.p + 2 * G, nullptr);
    return allreduce_partials(P, 4);
}

// one PCG iteration: the streaming update then the SpMV (optionally bracketed
// by HIP events for the live roofline)
// the update of iteration it (k_cg_axpy: reductions, convergence test, the
// streaming update); algorithmic bytes: 10 vectors (AMG: w z p x r u read,
// z p x r written)
static void pcg_update(xfk_problem *P, long long it)
{
    hipStream_t s = P->stream;
    const CgAxpyArgs A = cg_args(P, it);
    XFK_PHASE("PCG update (Chronopoulos-Gear axpy)", 80.0 * (double)P->N, launch_cg_axpy(s, A));
}

// the rest of iteration it: u = M^-1 r (V-cycle) and w = A u with its partials
static int pcg_precond_spmv(xfk_problem *P, long long it, bool stamp)
{
    hipStream_t s = P->stream;
    const CgAxpyArgs A = cg_args(P, it);
    const size_t G = (size_t)P->Gpart;
    const double N = P->N;
    int rc;
    double *pgam = P->part_loc.p + (size_t)((it + 1) & 1) * G;
    if (A.amg && (rc = P->amg->vcycle(s, A.R, A.U, &P->pcg.p->done, pgam)) != XFK_OK) return rc;
    const bool gam = A.amg && !P->amg->gamma_done;   // the SpMV forms r.u itself (reads r)
    const double *Rg = A.amg && gam ? A.R : nullptr;
    double *pg = A.amg && gam ? pgam : nullptr;
    const CgState *St = P->pcg.p;
    if (P->comm && P->comm->size > 1 && overlap_enabled()) {
        // sharded: the halo of u travels on the side stream while the tiles
        // without halo columns multiply (bit-identical to the single launch)
        if (!P->ts.ready()) {
            if ((rc = P->side.init()) != XFK_OK) return rc;
            if ((rc = build_tile_split(s, P->N, kCgBlock, P->rowptr.p, P->col.p, P->ts)) != XFK_OK) return rc;
        }
        const unsigned short *c16;
        const int *cbase;
        spmv_col16(P, c16, cbase);   // (boundary tiles reach the halo ids: int columns, decided per tile)
        rc = exchange_overlapped(
            s, P->side, [&](hipStream_t cs) { return P->comm->exchange(P->halo, A.U, cs); },
            [&] {
                launch_cg_spmv(s, P->N, P->rowptr.p, P->col.p, P->val.p, A.U, P->W2.p, P->part_loc.p + 2 * G, St, Rg,
                               pg, P->ts.tiles.p, P->ts.n_in, c16, cbase);
            },
            [&] {
                launch_cg_spmv(s, P->N, P->rowptr.p, P->col.p, P->val.p, A.U, P->W2.p, P->part_loc.p + 2 * G, St, Rg,
                               pg, P->ts.tiles.p + P->ts.n_in, P->ts.n_bd, c16, cbase);
            });
        if (rc != XFK_OK) return rc;
        return allreduce_partials(P, 3);
    }
    rc = exchange(P, A.U);
    if (rc != XFK_OK) return rc;
    if (stamp) XFK_CHECK(hipEventRecord(P->spmv_ev[P->spmv_used], s));
    const unsigned short *c16;
    const int *cbase;
    spmv_col16(P, c16, cbase);
    const double spmv_bytes = (c16 ? 10.0 : 12.0) * (double)P->nnz_own + 4.0 * (N + 1) + (gam ? 24.0 : 16.0) * N;
    XFK_PHASE("PCG SpMV w = A u", spmv_bytes,
              launch_cg_spmv(s, P->N, P->rowptr.p, P->col.p, P->val.p, A.U, P->W2.p, P->part_loc.p + 2 * G, St, Rg,
                             pg, nullptr, 0, c16, cbase));
    if (stamp) {
        XFK_CHECK(hipEventRecord(P->spmv_ev[P->spmv_used + 1], s));
        P->spmv_used += 2;
    }
    return allreduce_partials(P, 3);
}

static int pcg_iteration(xfk_problem *P, long long it, bool stamp)
{
    pcg_update(P, it);
    return pcg_precond_spmv(P, it, stamp);
}

// the f32 parts of the preconditioner (level-0 transfers, coarsest inverse)
// are abandoned for f64 when the PCG stagnates: the iterate is not finite, or
// after this many iterations the residual ratio is still above 1e-4 (a
// V-cycle preconditioner reaches 1e-8 in 20-30 on the meshes measured)
constexpr int kF32Guard = 150;
constexpr int kRetryF64 = 1;   // (internal return codes of pcg_solve_once)
// a hierarchy kept from an earlier Newton pass is abandoned for a fresh one
// when this solve would take more than max(2x, +8) the iterations of the pass
// that built it (projected from the observed rate at each poll): the first
// nonlinear pass can change the permeabilities from their initial values
// enough to make the old hierarchy useless (the antiperiodic magnet machine:
// 767 iterations on the kept one, 31 on a fresh one)
constexpr int kRetryFresh = 2;

static int pcg_solve_once(xfk_problem *P, int flag, long long max_iters)
{
    hipStream_t s = P->stream;
    int rc = xfk_resolve_nnz(P);   // (the assembly is enqueued: no bubble)
    if (rc != XFK_OK) return rc;
    rc = alloc_cg(P);
    if (rc != XFK_OK) return rc;
    rc = pcg_start(P, flag);
    if (rc != XFK_OK) return rc;
    long long it = 0;
    // the first batch: the iterations the first pass of the last solve took
    // (same problem, same matrix family: one poll), else 8 / 16; an
    // iteration launched after convergence exits at once but still costs
    // its launches, so the hint is not padded
    int batch = P->pc_used == XFK_PRECOND_AMG ? 8 : 16;
    // (clamped like every later batch, and never past the iteration cap, so a
    // zero-diagonal matrix is still caught at the first poll)
    if (flag == 0 && P->pcg_hint0 > 0) batch = std::min(P->pcg_hint0, 512);
    // a warm start (a Newton pass from the last iterate; the restart after a
    // fresh hierarchy) needs anything from 1 to ~25 iterations: one
    // iteration, then a batch sized from the residual it left and the rate
    // of this problem's last solve (an iteration launched after convergence
    // still costs its ~14 launches: 8 of them in a 1-iteration pass ~0.5 ms)
    else if (flag != 0 && P->pc_used == XFK_PRECOND_AMG && P->pcg_rate < 0) batch = 1;
    // the speculative Newton residual goes with polls expected to be the last:
    // not with the one-iteration probe of a warm start
    bool expect_last = batch != 1 || flag == 0;
    long long it0 = -1;   // the first poll: iterations and er, for the observed rate
    double er0 = 0;
    // Every batch ends with an update, whose convergence test the poll reads:
    // the V-cycle and SpMV of that iteration open the next batch, so the
    // converged solve launches no iteration tail that would only exit
    // (one V-cycle + SpMV, ~14 launches, saved per solve)
    bool tail = false;   // iteration it - 1's V-cycle + SpMV not launched yet
    // (the bound is the reuse test of amg_setup: a solve that cannot stay
    // within it would not have kept the hierarchy had its count been known;
    // polled at least every 16 iterations while the hierarchy is a kept one)
    const long long stale = (P->pc_used == XFK_PRECOND_AMG && !P->amg_fresh && P->amg_fresh_iters > 0)
                                ? std::max<long long>(2LL * P->amg_fresh_iters, P->amg_fresh_iters + 8)
                                : -1;
    for (;;) {
        batch = (int)std::max<long long>(1, std::min<long long>(batch, max_iters - it));
        if (stale > 0 && it < stale) batch = (int)std::min<long long>({(long long)batch, stale - it, 16LL});
        for (int k = 0; k < batch; ++k, ++it) {
            if (tail) {
                const long long ip = it - 1;
                const bool stamp = P->time_spmv && (ip % 16 == 0) && P->spmv_used + 2 <= (int)P->spmv_ev.size();
                if ((rc = pcg_precond_spmv(P, ip, stamp)) != XFK_OK) return rc;
            }
            pcg_update(P, it);
            tail = true;
        }
        XFK_CHECK(hipGetLastError());
        XFK_CHECK(hipMemcpyAsync(P->pcg_host, P->pcg.p, sizeof(CgState), hipMemcpyDeviceToHost, s));
        if (P->nws_at_poll && expect_last) {   // speculative: the Newton residual of the iterate as it stands
            launch_newton_res(s, P->N, P->V.p, P->Vold.p, P->partials.p, P->counters.p + 3, P->nws.p);
            XFK_CHECK(hipMemcpyAsync(P->nws_host, P->nws.p, sizeof(NewtonScalars), hipMemcpyDeviceToHost, s));
        }
        const bool miss_read = !P->miss_checked && P->asm_miss.p;   // the assembly's slot check, first poll
        if (miss_read) XFK_CHECK(hipMemcpyAsync(P->hpin + 4, P->asm_miss.p, sizeof(int), hipMemcpyDeviceToHost, s));
        XFK_CHECK(hipStreamSynchronize(s));
        if (miss_read) {
            // (sharded: the flags summed over the ranks -- every rank takes the
            // same decision, none is left waiting in the next collective; every
            // rank reads its flag at the same poll, so the calls match)
            double miss = (double)P->hpin[4];
            if (P->comm && (rc = allreduce_host(P, miss)) != XFK_OK) return rc;
            XFK_REQUIRE(miss == 0, XFK_ERR_HIP, "internal: element entry missing from the CSR pattern");
            P->miss_checked = true;
        }
        const CgState &S = *P->pcg_host;
        if (S.singular) {
            set_error("singular flag tripped: zero diagonal entry in the assembled matrix");
            return XFK_ERR_SINGULAR;
        }
        if (S.done) {   // (iterations launched after the stop leave V as it is)
            P->nws_ready = P->nws_at_poll && expect_last;
            break;
        }
        expect_last = true;   // (every later batch is sized to reach the stop)
        if (it >= max_iters) {
            set_error("PCG did not converge within the iteration cap");
            return XFK_ERR_NOCONV;
        }
        // (S is the same on every rank: the decision is collective-safe)
        const bool force = std::getenv("XFK_TEST_F64_FALLBACK") != nullptr;   // test hook (read per poll)
        if (P->pc_used == XFK_PRECOND_AMG && P->amg && P->amg->f32_active() &&
            (force || !std::isfinite(S.er) || (S.iters >= kF32Guard && S.er > 1e-4)))
            return kRetryF64;
        // the stale-hierarchy projection: the rate from er = 1 at iteration 0
        double rate = (S.iters > 0 && S.er > 0 && S.er < 1) ? std::log(S.er) / (double)S.iters : 0.0;
        // (the stop level: Precision, or the inexact pass's fraction of er0)
        const double tol_eff = std::max(S.tol, S.tol_rel * S.er0);
        long long rem = rate < 0 ? (long long)std::ceil(std::log(tol_eff / S.er) / rate) : 2 * batch;
        // (S and the counts are the same on every rank: collective-safe)
        if (stale > 0 && (S.iters >= stale || S.iters + rem > stale)) return kRetryFresh;
        // the next batch: the iterations left at the rate observed since the
        // first poll (else the last solve's, else the one above), not padded --
        // one more poll (~25 us) costs less than an iteration launched past
        // convergence (~70 us)
        double r2 = 0.0;
        if (it0 >= 0 && S.iters > it0 && S.er > 0 && S.er < er0) r2 = std::log(S.er / er0) / (double)(S.iters - it0);
        else if (P->pcg_rate < 0) r2 = P->pcg_rate;
        else r2 = rate;
        if (it0 < 0 && S.er > 0) {
            it0 = S.iters;
            er0 = S.er;
        }
        const long long nb = r2 < 0 ? (long long)std::ceil(std::log(tol_eff / S.er) / r2) : 2 * batch;
        batch = (int)std::max<long long>(1, std::min<long long>(nb, 512));
        // (Jacobi: ~25 us iterations -- padded, at least 8 per poll)
        if (P->pc_used != XFK_PRECOND_AMG) batch = (int)std::max<long long>(8, std::min<long long>(rem + 2, 512));
    }
    {   // this solve's rate, for the next warm start's batches
        const CgState &S = *P->pcg_host;
        double r = 0.0;
        if (it0 >= 0 && S.iters > it0 && S.er > 0 && S.er < er0) r = std::log(S.er / er0) / (double)(S.iters - it0);
        else if (flag == 0 && S.iters > 0 && S.er > 0 && S.er < 1) r = std::log(S.er) / (double)S.iters;
        if (r < 0 && P->pc_used == XFK_PRECOND_AMG) P->pcg_rate = r;
    }
    if (flag == 0) P->pcg_hint0 = (int)P->pcg_host->iters + 1;   // iteration it = iters detected the stop
    return XFK_OK;
}

static int pcg_solve(xfk_problem *P, int flag, long long max_iters)
{
    P->pcg_discarded = 0;
    P->nws_ready = false;
    int rc = pcg_solve_once(P, flag, max_iters);
    if (rc == kRetryFresh) {   // a fresh hierarchy, the PCG restarted from the iterate
        P->pcg_discarded = P->pcg_host->iters;
        P->amg_reusable = false;
        // (the cap covers the whole solve: the discarded iterations count)
        rc = pcg_solve_once(P, 1, std::max<long long>(1, max_iters - P->pcg_discarded));
        if (rc == kRetryFresh) {
            set_error("internal: fresh hierarchy retried twice");
            return XFK_ERR_HIP;
        }
        if (rc != kRetryF64) {
            P->pcg_host->iters += P->pcg_discarded;
            return rc;
        }
    }
    if (rc != kRetryF64) return rc;
    // f64 transfers and coarsest inverse for the rest of this problem's life,
    // a fresh hierarchy, and the PCG restarted from the iterate (from zero if
    // it is not finite)
    const long long first = P->pcg_host->iters + P->pcg_discarded;
    P->pcg_discarded = first;
    P->amg_f32 = 0;
    P->f64_fallback = true;
    P->amg_reusable = false;
    int f2 = 1;
    if (!std::isfinite(P->pcg_host->er)) {
        XFK_CHECK(hipMemsetAsync(P->V.p, 0, sizeof(double) * P->NL, P->stream));
        f2 = 0;
    }
    rc = pcg_solve_once(P, f2, std::max<long long>(1, max_iters - first));
    if (rc == kRetryF64 || rc == kRetryFresh) {   // (cannot repeat: no f32 part is left, the hierarchy is fresh)
        set_error("internal: f64 fallback requested twice");
        return XFK_ERR_HIP;
    }
    P->pcg_host->iters += first;
    return rc;
}

}  // namespace xfk

using namespace xfk;

extern "C" {

const char *xfk_last_error(void) { return g_err.c_str(); }

int xfk_alloc_stats(double *out4, int reset)
{
    XFK_REQUIRE(out4, XFK_ERR_ARG, "null argument");
    out4[0] = (double)g_nmalloc.load();
    out4[1] = 1e-6 * (double)g_nsmalloc.load();
    out4[2] = (double)g_nfree.load();
    out4[3] = 1e-6 * (double)g_nsfree.load();
    if (reset) g_nmalloc = g_nfree = g_nsmalloc = g_nsfree = g_npool = 0;
    return XFK_OK;
}

int xfk_sort_elements(int n_elems, const unsigned *score, int device, int *perm)
{
    XFK_REQUIRE(n_elems >= 0 && (n_elems == 0 || (score && perm)), XFK_ERR_ARG, "xfk_sort_elements: bad arguments");
    if (n_elems <= 1) {
        if (n_elems == 1) perm[0] = 0;
        return XFK_OK;
    }
    XFK_CHECK(hipSetDevice(device));
    struct Scratch {   // device blocks back to the process cache once the stream is idle
        hipStream_t s = nullptr;
        std::vector<void *> blocks;
        ~Scratch()
        {
            if (s) (void)hipStreamSynchronize(s);
            PoolRelease pr;
            for (void *b : blocks) dev_free(b);
            if (s) stream_release(s);
        }
        void *get(size_t bytes)
        {
            void *q = nullptr;
            if (dev_malloc(&q, bytes) != hipSuccess) return nullptr;
            blocks.push_back(q);
            return q;
        }
    } sc;
    XFK_CHECK(stream_acquire(&sc.s));
    const size_t n = (size_t)n_elems, nred = 2 * n + 64;
    auto *key = static_cast<unsigned long long *>(sc.get(8 * n));
    auto *tmp = static_cast<unsigned long long *>(sc.get(8 * n));
    auto *red = static_cast<unsigned long long *>(sc.get(8 * nred));
    auto *cin = static_cast<unsigned long long *>(sc.get(8 * nred));
    auto *sd = static_cast<unsigned *>(sc.get(4 * n));
    auto *flag = static_cast<int *>(sc.get(2 * sizeof(int)));
    XFK_REQUIRE(key && tmp && red && cin && sd && flag, XFK_ERR_HIP, "xfk_sort_elements: device allocation failed");
    XFK_CHECK(hipMemcpyAsync(sd, score, 4 * n, hipMemcpyHostToDevice, sc.s));
    const int rc = sort_elements_device(sc.s, n_elems, sd, reinterpret_cast<int *>(sd), key, tmp, red, cin, flag,
                                        nullptr);
    if (rc != XFK_OK) return rc;
    XFK_CHECK(hipMemcpyAsync(perm, sd, 4 * n, hipMemcpyDeviceToHost, sc.s));
    XFK_CHECK(hipStreamSynchronize(sc.s));
    return XFK_OK;
}

int xfk_release_cache(void)
{
    std::vector<void *> dev, pin;
    {
        BlockPool &bp = block_pool();
        std::lock_guard<std::mutex> g(bp.mu);
        for (auto &kv : bp.free)
            for (void *q : kv.second) dev.push_back(q);
        bp.free.clear();
        bp.cached = 0;
    }
    {
        PinPool &pp = pin_pool();
        std::lock_guard<std::mutex> g(pp.mu);
        for (auto &kv : pp.free)
            for (void *q : kv.second) pin.push_back(q);
        pp.free.clear();
        pp.cached = 0;
    }
    int rc = XFK_OK;
    for (void *q : dev)
        if (hipFree(q) != hipSuccess) rc = XFK_ERR_HIP;
    for (void *q : pin)
        if (hipHostFree(q) != hipSuccess) rc = XFK_ERR_HIP;
    stream_pool_drain();
    if (rc != XFK_OK) set_error("xfk_release_cache: hipFree failed");
    return rc;
}

int xfk_cache_stats(long long *out3)
{
    XFK_REQUIRE(out3, XFK_ERR_ARG, "null output");
    {
        BlockPool &bp = block_pool();
        std::lock_guard<std::mutex> g(bp.mu);
        out3[0] = (long long)bp.cached;
    }
    {
        PinPool &pp = pin_pool();
        std::lock_guard<std::mutex> g(pp.mu);
        out3[1] = (long long)pp.cached;
    }
    out3[2] = stream_pool_idle();
    return XFK_OK;
}

int xfk_problem_memory(const xfk_problem *P, long long *out4)
{
    XFK_REQUIRE(P && out4, XFK_ERR_ARG, "null argument");
    const DevArena &a = P->arena;
    long long live = 0, reuse = 0;
    for (auto &kv : a.carved) live += (long long)kv.second;
    for (auto &kv : a.reuse) reuse += (long long)kv.first;
    for (auto &b : a.pending) reuse += (long long)b.second;
    out4[0] = (long long)a.chunk_bytes();
    out4[1] = (long long)a.chunks.size();
    out4[2] = live;
    out4[3] = reuse;
    return XFK_OK;
}

int xfk_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int xfk_device_init(int device)
{
    static std::mutex mu;
    static std::set<int> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count(device)) return XFK_OK;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        (void)hipGetLastError();
        set_error("xfk_device_init: no HIP device " + std::to_string(device));
        return XFK_ERR_HIP;
    }
    XFK_CHECK(hipSetDevice(device));
    XFK_CHECK(hipFree(nullptr));
    for (hipError_t (*w)() : {warm_module_device, warm_module_pcg, warm_module_amg, warm_module_harmonic,
                              warm_module_sort, warm_module_comm})
        XFK_CHECK(w());
    hipStream_t s[3] = {};   // a problem's solve stream, the AMG's side stream and the sort's
    for (hipStream_t &q : s) XFK_CHECK(stream_acquire(&q));
    for (hipStream_t q : s) stream_release(q);
    done.insert(device);
    return XFK_OK;
}

void xfk_problem_destroy(xfk_problem *P)
{
    if (!P) return;
    (void)hipSetDevice(P->device);
    if (P->stream) (void)hipStreamSynchronize(P->stream);
    for (auto &ev : P->pass_ev) (void)hipEventDestroy(ev);
    for (auto &ev : P->spmv_ev) (void)hipEventDestroy(ev);
    for (auto &ev : P->setup_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (P->nnz_ev) (void)hipEventDestroy(P->nnz_ev);
    hipStream_t s = P->stream;
    // every stream of the problem idle before its pinned buffers and device
    // blocks go to the process caches (a failed solve may have left side-stream
    // copies into them in flight)
    if (P->side.cs) (void)hipStreamSynchronize(P->side.cs);
    if (P->amg) P->amg->sync_streams();
    {
        PoolRelease pr;
        pinned_free(P->pcg_host);
        pinned_free(P->hpin);
        pinned_free(P->nws_host);
        pinned_free(P->hc_host);
        delete P->amg;
        P->amg = nullptr;
        DevArena arena = std::move(P->arena);
        delete P;   // device buffers free themselves (DBuf) into the process cache
        arena.release();   // (after every buffer carved from it)
    }
    stream_release(s);   // (synchronised above; pooled for the next problem)
}

}  // extern "C"

namespace xfk {

// ----------------------------------------------------------------------------
// problem creation: validation, global preparation, local (per-rank) build
// ----------------------------------------------------------------------------

bool edge_lines_used(const xfk_problem_desc *d, std::vector<char> &used);

int validate_desc(const xfk_problem_desc *d)
{
    XFK_REQUIRE(d->n_nodes > 0 && d->n_elems > 0, XFK_ERR_ARG, "empty mesh");
    XFK_REQUIRE(d->x && d->y && d->p && d->lbl, XFK_ERR_ARG, "missing mesh arrays");
    XFK_REQUIRE(d->n_blocks > 0 && d->blocks && d->n_labels > 0 && d->labels, XFK_ERR_ARG,
                "missing block or label tables");
    XFK_REQUIRE(d->n_lines == 0 || d->lines, XFK_ERR_ARG, "missing boundary table");
    XFK_REQUIRE(d->n_points == 0 || d->points, XFK_ERR_ARG, "missing point table");
    XFK_REQUIRE(d->n_circs == 0 || d->circs, XFK_ERR_ARG, "missing circuit table");
    XFK_REQUIRE(d->n_pbc == 0 || d->pbc, XFK_ERR_ARG, "missing pbc table");
    XFK_REQUIRE(d->n_ages >= 0 && (d->n_ages == 0 || d->ages), XFK_ERR_ARG, "missing air-gap element table");
    XFK_REQUIRE(d->length_units >= 0 && d->length_units < 6, XFK_ERR_ARG, "bad length units");
    XFK_REQUIRE(d->problem_type == XFK_PLANAR || d->problem_type == XFK_AXISYMMETRIC, XFK_ERR_ARG,
                "problem type must be planar or axisymmetric");
    const int N = d->n_nodes, NE = d->n_elems;
    // the per-element checks in parallel chunks; failures are reported in the
    // order of the checks
    std::atomic<int> bad{0};
    const int NL = d->n_labels;
    host_par_for(NE, 1 << 17, [&](long long a, long long b) {
        bool okp = true, okl = true;
        for (long long k = 3 * a; k < 3 * b; ++k) okp &= (unsigned)d->p[k] < (unsigned)N;
        for (long long i = a; i < b; ++i) okl &= (unsigned)d->lbl[i] < (unsigned)NL;
        if (!okp || !okl) bad |= (okp ? 0 : 1) | (okl ? 0 : 2);
    });
    XFK_REQUIRE(!(bad & 1), XFK_ERR_ARG, "element node index out of range");
    XFK_REQUIRE(!(bad & 2), XFK_ERR_ARG, "element label out of range");
    for (int k = 0; k < d->n_labels; ++k) {
        XFK_REQUIRE(d->labels[k].block >= 0 && d->labels[k].block < d->n_blocks, XFK_ERR_ARG,
                    "label block index out of range");
        XFK_REQUIRE(d->labels[k].in_circuit < d->n_circs, XFK_ERR_ARG, "label circuit index out of range");
        XFK_REQUIRE(!(d->problem_type == XFK_AXISYMMETRIC && d->labels[k].is_external) || d->ext_ro > 0, XFK_ERR_ARG,
                    "exterior region needs [extRo] > 0");
    }
    for (int k = 0; k < d->n_blocks; ++k) {
        const xfk_block_desc &b = d->blocks[k];
        XFK_REQUIRE(b.BHpoints == 0 || (b.BHpoints >= 2 && b.B && b.H && b.slope), XFK_ERR_ARG,
                    "B-H curve needs >= 2 points with slopes");
    }
    if (d->marker)
        for (int i = 0; i < N; ++i)
            XFK_REQUIRE(d->marker[i] < d->n_points, XFK_ERR_ARG, "node point-property index out of range");
    if (d->e) {
        // the device packs an element's three edge properties in 10-bit fields
        // of the properties the mesh uses (prepare_global compacts the table):
        // at most 1022 distinct ones on edges, any number defined
        std::vector<char> used;
        XFK_REQUIRE(edge_lines_used(d, used), XFK_ERR_ARG, "edge boundary-property index out of range");
        long long nused = 0;
        for (char u : used) nused += u;
        XFK_REQUIRE(nused <= 1022, XFK_ERR_UNSUPPORTED, "at most 1022 distinct boundary properties on element edges");
    }
    return XFK_OK;
}

// used[k] = 1 for the boundary properties some element edge carries; false
// when an edge index is >= n_lines
bool edge_lines_used(const xfk_problem_desc *d, std::vector<char> &used)
{
    const int nl = std::max(1, d->n_lines);
    const long long n3 = 3LL * d->n_elems;
    used.assign(nl, 0);
    if (!d->e) return true;
    std::mutex mu;
    std::atomic<bool> ok{true};
    host_par_for(n3, 1 << 18, [&](long long a, long long b) {
        std::vector<char> u(nl, 0);
        bool good = true;
        for (long long k = a; k < b; ++k) {
            const int e = d->e[k];
            good &= e < d->n_lines;
            if (e >= 0 && e < d->n_lines) u[e] = 1;
        }
        if (!good) ok = false;
        std::lock_guard<std::mutex> g(mu);
        for (int q = 0; q < nl; ++q) used[q] |= u[q];
    });
    return ok;
}

int check_device(int device)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("no HIP device available (the fsolver hot path has no CPU fallback)");
        return XFK_ERR_HIP;
    }
    XFK_REQUIRE(device >= 0 && device < ndev, XFK_ERR_ARG, "device index out of range");
    return XFK_OK;
}

int prepare_magdir(const xfk_problem_desc *d, GlobalPrep &G)
{
    // Functional magnetisation directions (static2d.cpp:509-583,
    // staticaxi.cpp:350-406): the reference runs the label's Lua chunk for
    // every element in every Newton pass, on one interpreter whose globals
    // persist from element to element.  The chunks run here once, in element
    // order on one native interpreter (xfk_magdir.cpp over xfk_lua.cpp, the
    // same angle to the bit); a nonlinear problem's later passes would give
    // the same angles unless a chunk changed state, which MagDir::repeatable
    // refuses.  Each element of such a label gets a label entry of its own
    // carrying cos / sin of its angle -- the device kernels are unchanged.
    bool any_fctn = false;
    for (int k = 0; k < d->n_labels; ++k) {
        const char *f = d->labels[k].mag_dir_fctn;
        any_fctn |= (f && *f);
    }
    if (!any_fctn) return XFK_OK;
    const int NE = d->n_elems;
    MagDir md(d->problem_type == XFK_AXISYMMETRIC);
    std::string err;
    bool any = false;
    std::vector<int> elab(d->lbl, d->lbl + NE);
    for (int i = 0; i < NE; ++i) {
        const int l = d->lbl[i];
        const char *f = d->labels[l].mag_dir_fctn;
        if (!f || !*f) continue;
        double X[3], Y[3], t = 0;
        for (int j = 0; j < 3; ++j) {
            X[j] = d->x[d->p[3LL * i + j]];
            Y[j] = d->y[d->p[3LL * i + j]];
        }
        XFK_REQUIRE(md.eval(f, X, Y, d->length_units, d->labels[l].mag_dir, &t, err), XFK_ERR_ARG, err.c_str());
        DevLabel v = G.lab[l];
        v.cos_m = cos(t * kPI / 180.);   // static2d.cpp:593-595
        v.sin_m = sin(t * kPI / 180.);
        elab[i] = (int)G.lab.size();
        G.lab.push_back(v);
        any = true;
    }
    if (!any) return XFK_OK;
    if (G.any_nonlinear) XFK_REQUIRE(md.repeatable(err), XFK_ERR_ARG, err.c_str());
    G.elab.swap(elab);
    return XFK_OK;
}

void prepare_global(const xfk_problem_desc *d, GlobalPrep &G)
{
    const int N = d->n_nodes, NE = d->n_elems;
    const double c = kC;
    const double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};

    // tables
    G.blk.resize(d->n_blocks);
    for (int k = 0; k < d->n_blocks; ++k) {
        const xfk_block_desc &b = d->blocks[k];
        DevBlock &o = G.blk[k];
        o.mu_x = b.mu_x; o.mu_y = b.mu_y; o.H_c = b.H_c; o.J_re = b.J_re; o.Cduct = b.Cduct;
        o.LamFill = b.LamFill; o.LamType = b.LamType; o.BHpoints = b.BHpoints;
        o.bh_off = (int)G.hB.size();
        // (XFK_BH_SCAN: the reference's knot scan for every table -- the test
        // that the bisection finds the same intervals)
        o.bh_sorted = std::getenv("XFK_BH_SCAN") ? 0 : 1;
        for (int i = 0; i < b.BHpoints; ++i) {
            if (i > 0 && !(b.B[i] >= b.B[i - 1])) o.bh_sorted = 0;
            G.hB.push_back(b.B[i]);
            G.hH.push_back(b.H[i]);
            G.hS.push_back(b.slope[i]);
        }
    }
    if (G.hB.empty()) { G.hB.push_back(0); G.hH.push_back(0); G.hS.push_back(0); }
    G.lab.resize(d->n_labels);
    for (int k = 0; k < d->n_labels; ++k) {
        const xfk_label_desc &l = d->labels[k];
        double t = l.mag_dir;
        G.lab[k].cos_m = cos(t * kPI / 180.);
        G.lab[k].sin_m = sin(t * kPI / 180.);
        G.lab[k].blk = l.block;
        G.lab[k].in_circuit = l.in_circuit;
        G.lab[k].is_wound = l.is_wound;
        G.lab[k].external = l.is_external;
    }
    // boundary properties used on element edges, compacted (the 10-bit edge
    // fields index this table; validate_desc bounds its size)
    // (ascending property index; validate_desc checked the indices)
    G.lmap.assign(std::max(1, d->n_lines), -1);
    G.lin_used.clear();
    if (d->e) {
        std::vector<char> used;
        edge_lines_used(d, used);
        for (int k = 0; k < (int)used.size(); ++k)
            if (used[k]) {
                G.lmap[k] = (int)G.lin_used.size();
                G.lin_used.push_back(k);
            }
    }
    G.lin.assign(std::max<size_t>(1, G.lin_used.size()), DevLine{});
    for (size_t m = 0; m < G.lin_used.size(); ++m) {
        const xfk_line_desc &l = d->lines[G.lin_used[m]];
        G.lin[m].c0 = l.c0;
        G.lin[m].c1 = l.c1;
        G.lin[m].format = l.format;
        G.lin[m].pad = 0;
    }
    G.axi = d->problem_type == XFK_AXISYMMETRIC;
    G.ext_ro = d->ext_ro * units[d->length_units];   // staticaxi.cpp:70-72
    G.ext_ri = d->ext_ri * units[d->length_units];
    G.ext_zo = d->ext_zo * units[d->length_units];
    // which elements are nonlinear -> LinearFlag (static2d.cpp:633-639)
    {
        std::vector<char> lnl(d->n_labels);
        bool any = false;
        for (int k = 0; k < d->n_labels; ++k) any |= (lnl[k] = G.blk[G.lab[k].blk].BHpoints != 0) != 0;
        std::atomic<bool> hit{false};
        if (any)
            host_par_for(NE, 1 << 18, [&](long long a, long long b) {
                for (long long i = a; i < b && !hit.load(std::memory_order_relaxed); ++i)
                    if (lnl[d->lbl[i]]) hit = true;
            });
        G.any_nonlinear = hit;
    }

    // circuits, element order (static2d.cpp:84-167)
    G.circ.assign(std::max(1, d->n_circs), DevCirc{});
    if (d->n_circs > 0) {
        std::vector<double> I1(d->n_circs, 0.0), I2(d->n_circs, 0.0), I3(d->n_circs, 0.0);
        for (int i = 0; i < NE; ++i) {
            const DevLabel &L = G.lab[d->lbl[i]];
            if (L.in_circuit == -1) continue;
            const int *n = d->p + 3LL * i;
            double p0 = d->y[n[1]] - d->y[n[2]], p1 = d->y[n[2]] - d->y[n[0]];
            double q0 = d->x[n[2]] - d->x[n[1]], q1 = d->x[n[0]] - d->x[n[2]];
            double a = (p0 * q1 - p1 * q0) / 2.;
            double Cduct = G.blk[L.blk].Cduct;
            if (L.is_wound) Cduct = 0;
            I1[L.in_circuit] += a;
            if (G.axi) I2[L.in_circuit] += 100. * a * Cduct / ((d->x[n[0]] + d->x[n[1]] + d->x[n[2]]) / 3.);
            else I2[L.in_circuit] += a * Cduct;   // staticaxi.cpp:96-104 / static2d.cpp:108-118
            I3[L.in_circuit] += G.blk[L.blk].J_re * a * 100.;
        }
        for (int k = 0; k < d->n_circs; ++k) {
            DevCirc &C = G.circ[k];
            C.amps_re = d->circs[k].amps_re;
            C.dvolts_re = d->circs[k].dvolts_re;
            C.type = d->circs[k].type;
            C.J = 0; C.dV = 0; C.ccase = 0;
            if (C.type == 0) {
                if (I2[k] == 0) {
                    C.ccase = 1;
                    C.J = (I1[k] == 0.) ? 0. : 0.01 * (C.amps_re - I3[k]) / I1[k];
                } else {
                    C.ccase = 0;
                    C.dV = -0.01 * (C.amps_re - I3[k]) / I2[k];
                }
            } else {
                C.ccase = 0;
                C.dV = C.dvolts_re;
            }
        }
    }

    // edges -> packed 3 x 10-bit boundary-property indices
    auto edge = [&](long long k) { return d->e ? d->e[k] : -1; };
    G.ebits.assign(NE, 0);
    // elements with a prescribed-A (format 0) edge, in element order (the
    // SetValue pass below visits only them)
    std::vector<int> dir_elems;
    if (d->e) {
        const int nch = 64;
        std::vector<std::vector<int>> part(nch);
        host_par_for(nch, 1, [&](long long a, long long b) {
            for (long long c = a; c < b; ++c)
                for (long long i = NE * c / nch; i < NE * (c + 1) / nch; ++i) {
                    unsigned bits = 0;
                    bool dir = false;
                    for (int j = 0; j < 3; ++j) {
                        const int ej = d->e[3 * i + j];
                        if (ej < 0) continue;
                        bits |= (unsigned)(G.lmap[ej] + 1) << (10 * j);
                        dir |= d->lines[ej].format == 0;
                    }
                    G.ebits[i] = (int)bits;
                    if (dir) part[c].push_back((int)i);
                }
        });
        for (auto &v : part) dir_elems.insert(dir_elems.end(), v.begin(), v.end());
    }

    // point currents and Dirichlet values in the reference's SetValue order
    G.fixed.assign(N, 0);
    G.first.assign(N, 0.0);
    G.last.assign(N, 0.0);
    auto set_value = [&](int i, double x) {
        if (!G.fixed[i]) G.first[i] = x;
        G.fixed[i] = 1;
        G.last[i] = x;
    };
    auto marker = [&](int i) { return d->marker ? d->marker[i] : -1; };
    for (int i = 0; i < N; ++i) {
        int m = marker(i);
        if (m >= 0 && d->points[m].J_re != 0.0) {
            G.pt_nodes.push_back(i);
            // axisymmetric: 0.01 J 2 r (staticaxi.cpp:644-650)
            G.pt_J.push_back(G.axi ? 0.01 * d->points[m].J_re * 2. * d->x[i] : 0.01 * d->points[m].J_re);
        }
    }
    for (int i = 0; i < N; ++i) {
        int m = marker(i);
        if (G.axi && fabs(d->x[i]) < units[d->length_units] * 1.e-06)
            set_value(i, 0.);   // A = 0 on the axis (staticaxi.cpp:652-659)
        else if (m >= 0 && d->points[m].J_re == 0 && d->points[m].J_im == 0)
            set_value(i, d->points[m].A_re / c);
    }
    for (int i : dir_elems)
        for (int j = 0; j < 3; ++j) {
            int k = (j + 1) % 3;
            int sgi = edge(3LL * i + j);
            if (sgi < 0 || d->lines[sgi].format != 0) continue;
            const xfk_line_desc &ln = d->lines[sgi];
            int nodes2[2] = {d->p[3LL * i + j], d->p[3LL * i + k]};
            for (int m = 0; m < 2; ++m) {
                double x = d->x[nodes2[m]], y = d->y[nodes2[m]], a;
                if (d->coords == 0) {
                    x /= units[d->length_units];
                    y /= units[d->length_units];
                    a = ln.A0 + x * ln.A1 + y * ln.A2;
                } else {
                    double r = sqrt(x * x + y * y), t;
                    if ((x == 0) && (y == 0)) t = 0;
                    else t = atan2(y, x) / kDEG;
                    r /= units[d->length_units];
                    a = ln.A0 + r * ln.A1 + t * ln.A2;
                }
                a *= cos(ln.phi * kDEG);
                if (!G.axi || x != 0) set_value(nodes2[m], a / c);   // staticaxi.cpp:681, 694, 712, 726
            }
        }
}

// Build the device problem of one rank (plan == nullptr: the whole mesh).
int build_local(const xfk_problem_desc *d, const GlobalPrep &G, const PartPlan *plan, int device,
                       xfk_comm *comm, xfk_problem **out)
{
    CreateTrace tr;
    xfk_problem *P = new xfk_problem();
    ArenaScope arena_scope(&P->arena);
    P->device = device;
    if (std::getenv("XFK_SPIN_WAIT")) {   // experiment: host waits spin instead of yielding
        hipError_t e = hipSetDevice(device);
        if (e == hipSuccess) e = hipSetDeviceFlags(hipDeviceScheduleSpin);
        std::fprintf(stderr, "[xfk] hipDeviceScheduleSpin: %s\n", hipGetErrorString(e));
    }
    if (hipSetDevice(device) != hipSuccess || stream_acquire(&P->stream) != hipSuccess) {
        set_error("cannot initialise the HIP device/stream");
        delete P;
        return XFK_ERR_HIP;
    }
    auto fail = [&](int code) {
        xfk_problem_destroy(P);
        return code;
    };
    tr.mark("  device + stream");
    const int Ng = d->n_nodes, NEg = d->n_elems;
    const int N = plan ? plan->n_own : Ng;                  // owned rows
    const int NR = plan ? plan->n_own + plan->n_extra : Ng; // assembled rows (+ coupled nodes owned elsewhere)
    const int NL = plan ? plan->n_own + plan->n_halo : Ng;  // local nodes
    const int NE = plan ? (int)plan->elems.size() : NEg;
    auto gnode = [&](int l) { return plan ? plan->l2g[l] : l; };
    auto gelem = [&](int l) { return plan ? plan->elems[l] : l; };
    P->N = N;
    P->NR = NR;
    P->NL = NL;
    P->NE = NE;
    P->N_global = Ng;
    P->precision = d->precision;
    P->relax = d->relax;
    P->length_units = d->length_units;
    P->coords = d->coords;
    P->axi = G.axi;
    if (G.axi) P->axi_x.assign(d->x, d->x + d->n_nodes);
    P->ext_ro = G.ext_ro;
    P->ext_ri = G.ext_ri;
    P->ext_zo = G.ext_zo;
    P->any_nonlinear = G.any_nonlinear;
    if (plan) {
        P->comm = comm;
        P->rank = plan->rank;
        P->nranks = plan->nranks;
        P->row0 = plan->row0;
        P->halo = plan->halo;
        P->l2g = plan->l2g;
    }

    // local mesh: a single device uploads the descriptor's (and the global
    // preparation's) own arrays -- no host copies; a rank gathers its part
    std::vector<double> xs, ys;
    std::vector<int> pls, lbls, ebs;
    const double *xp = d->x, *yp = d->y;
    const int *plp = d->p, *lblp = G.elab.empty() ? d->lbl : G.elab.data(), *ebp = G.ebits.data();
    // global -> local: owned, or inside a receive range
    std::unordered_map<int, int> g2l_halo;
    if (plan)
        for (const HaloRange &r : plan->halo.recv)
            for (int k = 0; k < r.len; ++k) g2l_halo[r.g0 + k] = r.off + k;
    auto g2l = [&](int g) -> int {
        if (!plan) return g;
        if (g >= plan->row0 && g < plan->row0 + plan->n_own) return g - plan->row0;
        auto it = g2l_halo.find(g);
        return it == g2l_halo.end() ? -1 : it->second;
    };
    if (plan) {
        xs.resize(NL);
        ys.resize(NL);
        for (int l = 0; l < NL; ++l) {
            xs[l] = d->x[gnode(l)];
            ys[l] = d->y[gnode(l)];
        }
        pls.resize(3LL * NE);
        lbls.resize(NE);
        ebs.resize(NE);
        for (int l = 0; l < NE; ++l) {
            const int e = gelem(l);
            for (int j = 0; j < 3; ++j) {
                const int v = g2l(d->p[3LL * e + j]);
                XFK_REQUIRE(v >= 0, fail(XFK_ERR_ARG), "internal: element node outside the local halo");
                pls[3LL * l + j] = v;
            }
            lbls[l] = lblp[e];
            ebs[l] = ebp[e];
        }
        xp = xs.data();
        yp = ys.data();
        plp = pls.data();
        lblp = lbls.data();
        ebp = ebs.data();
    }
    // the label table: with MagDirFctn labels it holds one entry per element of
    // such a label (prepare_magdir), so a rank uploads only the entries its
    // elements reference, renumbered
    std::vector<DevLabel> labs;
    const DevLabel *labp = G.lab.data();
    size_t nlab = G.lab.size();
    if (plan && !G.elab.empty()) {
        std::unordered_map<int, int> lmap;
        for (int l = 0; l < NE; ++l) {
            auto it = lmap.find(lbls[l]);
            if (it == lmap.end()) {
                it = lmap.emplace(lbls[l], (int)labs.size()).first;
                labs.push_back(G.lab[lbls[l]]);
            }
            lbls[l] = it->second;
        }
        if (labs.empty()) labs.push_back(G.lab[0]);
        labp = labs.data();
        nlab = labs.size();
    }
    // host element nodes: only the periodic / air-gap maps read them
    if (d->n_pbc || !G.age_key.empty()) P->hp.assign(plp, plp + 3LL * NE);
    if (d->n_pbc) {   // periodic pairs in local numbering (sharded: every coupled node is local)
        P->hpbc.assign(d->pbc, d->pbc + 3LL * d->n_pbc);
        for (int k = 0; k < d->n_pbc; ++k)
            for (int m = 0; m < 2; ++m) {
                const int g = d->pbc[3 * k + m];
                if (g < 0 || g >= Ng) continue;   // reported by build_pbc_map
                const int v = g2l(g);
                XFK_REQUIRE(v >= 0 && v < NR, fail(XFK_ERR_ARG), "internal: periodic node is not an assembled row");
                P->hpbc[3 * k + m] = v;
            }
    }

    // boundary data of the local nodes (global values), owned rows only for rows
    std::vector<unsigned char> fxs;
    std::vector<double> fsts, lsts;
    const unsigned char *fixed = G.fixed.data();
    const double *first = G.first.data(), *last = G.last.data();
    if (plan) {
        fxs.resize(NL);
        fsts.resize(NL);
        lsts.resize(NL);
        for (int l = 0; l < NL; ++l) {
            fxs[l] = G.fixed[gnode(l)];
            fsts[l] = G.first[gnode(l)];
            lsts[l] = G.last[gnode(l)];
        }
        fixed = fxs.data();
        first = fsts.data();
        last = lsts.data();
    }
    std::vector<int> pt_nodes, fix_rows;
    std::vector<double> pt_J;
    for (size_t k = 0; k < G.pt_nodes.size(); ++k) {
        const int l = g2l(G.pt_nodes[k]);
        if (l < 0 || l >= NR) continue;
        pt_nodes.push_back(l);
        pt_J.push_back(G.pt_J[k]);
    }
    for (int l = 0; l < NR; ++l)
        if (fixed[l]) fix_rows.push_back(l);
    P->npt = (int)pt_nodes.size();
    P->nfix_rows = (int)fix_rows.size();

    if (!plan) {
        P->age_key = G.age_key;
        P->age_val = G.age_val;
    } else {   // air-gap entries of the assembled rows, local numbering (r <= c kept as a key order)
        for (size_t m = 0; m < G.age_key.size(); ++m) {
            int r = g2l((int)(G.age_key[m] >> 32)), c = g2l((int)(G.age_key[m] & 0xffffffff));
            XFK_REQUIRE(r >= 0 && c >= 0 && r < NR && c < NR, fail(XFK_ERR_ARG),
                        "internal: air-gap node is not an assembled row");
            if (c < r) std::swap(r, c);
            P->age_key.push_back(((long long)r << 32) | (unsigned)c);
            P->age_val.push_back(G.age_val[m]);
        }
    }
    tr.mark("  local mesh + BC arrays");
    int rc = build_pbc_map(P, G.pbc_aux);
    if (rc != XFK_OK) return fail(rc);
    tr.mark("  periodic map");
    if (tr.on)
        std::fprintf(stderr, "[create]     %zu pairs, %zu entries (%zu terms), %zu fill, %zu age couplings\n",
                     P->hpbc.size() / 3, P->pbc_entry_key.size(), P->pbc_entry_terms.size(), P->pbc_fill.size(),
                     P->age_key.size());
    add_age_fill(P);
    tr.mark("  air-gap fill");

    hipStream_t s = P->stream;
    hipError_t e = hipSuccess;
#define UP(buf, ptr, n) if (e == hipSuccess) e = upload(buf, ptr, n, s)
    UP(P->x, xp, (size_t)NL);
    UP(P->y, yp, (size_t)NL);
    UP(P->p_raw, plp, 3 * (size_t)NE);
    UP(P->lbl_raw, lblp, (size_t)NE);
    UP(P->ebits_raw, ebp, (size_t)NE);
    UP(P->blocks, G.blk.data(), G.blk.size());
    UP(P->labels, labp, nlab);
    UP(P->lines, G.lin.data(), G.lin.size());
    UP(P->circs, G.circ.data(), G.circ.size());
    UP(P->bhB, G.hB.data(), G.hB.size());
    UP(P->bhH, G.hH.data(), G.hH.size());
    UP(P->bhS, G.hS.data(), G.hS.size());
    UP(P->pt_nodes, pt_nodes.data(), pt_nodes.size());
    UP(P->pt_J, pt_J.data(), pt_J.size());
    UP(P->fixed, fixed, (size_t)NL);
    UP(P->fix_first, first, (size_t)NL);
    UP(P->fix_last, last, (size_t)NL);
    UP(P->fix_rows, fix_rows.data(), fix_rows.size());
#undef UP
    tr.mark("  uploads enqueued");
    if (e == hipSuccess) e = pinned_malloc((void **)&P->pcg_host, sizeof(CgState));
    if (e == hipSuccess) e = pinned_malloc((void **)&P->hpin, 16 * sizeof(int));
    if (e == hipSuccess) e = pinned_malloc((void **)&P->nws_host, sizeof(NewtonScalars));
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    tr.mark("  pinned mirrors + sync");
    if (e != hipSuccess) {
        set_error(std::string("upload failed: ") + hipGetErrorString(e));
        return fail(XFK_ERR_HIP);
    }
    P->nblocks = d->n_blocks;
    P->nlabels = (int)nlab;
    P->nlines = d->n_lines;
    P->ncircs = d->n_circs;
    // the AMG object and its setup side stream are resources of the problem,
    // created with it (a stream's creation is not work of the first solve)
    P->amg = new Amg();
    if (P->amg->sw.init() != XFK_OK || P->amg->reserve_host() != XFK_OK) return fail(XFK_ERR_HIP);
    tr.mark("  AMG side stream");
    *out = P;
    return XFK_OK;
}

// The first solve's device footprint, reserved in the problem's arena at
// creation (outside any solve), so that the solve carves its buffers without a
// hipMalloc (16 calls, 0.34 ms of a configs[2] first solve): 4.32 GB of chunks
// at 1.0M rows (configs[2]), 0.50 GB at 103k rows (tools/lab/mem_probe.py,
// profiles/r05t_mem_probe.txt) -- ~4.4 kB per owned row.  A larger solve takes
// further chunks as before.  XFK_ARENA_RESERVE=0: no reservation.
// The reservation is only a speed-up: it is skipped when it would take more
// than half of the device's free memory, and a failed one is dropped (the
// HIP error cleared) -- creation never fails on it, so the ranks of a sharded
// problem cannot disagree about it.
static int reserve_first_solve(xfk_problem **out)
{
    xfk_problem *P = *out;
    static const long long per_row = [] {
        const char *e = std::getenv("XFK_ARENA_RESERVE");
        return e ? std::atoll(e) : 4400LL;
    }();
    if (!P || per_row <= 0) return XFK_OK;
    XFK_CHECK(hipSetDevice(P->device));
    const size_t bytes = (size_t)per_row * (size_t)std::max(0, P->N) + (64ull << 20);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return XFK_OK;
    }
    if (bytes > free_b / 2) return XFK_OK;
    if (P->arena.reserve(bytes) != hipSuccess) (void)hipGetLastError();
    return XFK_OK;
}

}  // namespace xfk

extern "C" {

int xfk_problem_create(const xfk_problem_desc *d, int device, xfk_problem **out)
{
    XFK_REQUIRE(d && out, XFK_ERR_ARG, "null argument");
    *out = nullptr;
    CreateTrace tr;
    int rc = validate_desc(d);
    if (rc == XFK_OK) rc = check_device(device);
    if (rc != XFK_OK) return rc;
    tr.mark("validate + device");
    GlobalPrep G;
    prepare_global(d, G);
    tr.mark("prepare_global");
    rc = prepare_magdir(d, G);
    if (rc != XFK_OK) return rc;
    rc = age_entries(d, 1.0, G.age_key, G.age_val);
    if (rc != XFK_OK) return rc;
    tr.mark("magdir + air gaps");
    rc = build_local(d, G, nullptr, device, nullptr, out);
    tr.mark("build_local");
    if (rc == XFK_OK) rc = reserve_first_solve(out);
    tr.mark("arena reserve");
    return rc;
}

int xfk_partition_plan(int n_nodes, int n_elems, const int *p, int rank, int nranks, xfk_dist_info *info,
                       int *l2g, int *elems, int *recv, int *send)
{
    return xfk_partition_plan_coupled(n_nodes, n_elems, p, rank, nranks, 0, nullptr, info, l2g, elems, recv, send);
}

int xfk_partition_plan_coupled(int n_nodes, int n_elems, const int *p, int rank, int nranks, int n_coupled,
                               const int *coupled, xfk_dist_info *info, int *l2g, int *elems, int *recv, int *send)
{
    XFK_REQUIRE(p && info && n_nodes > 0 && n_elems > 0, XFK_ERR_ARG, "null argument");
    XFK_REQUIRE(n_coupled == 0 || coupled, XFK_ERR_ARG, "null coupled-node list");
    std::vector<int> cpl(coupled, coupled + n_coupled);
    std::sort(cpl.begin(), cpl.end());
    cpl.erase(std::unique(cpl.begin(), cpl.end()), cpl.end());
    PartPlan plan;
    XFK_REQUIRE(plan_partition(n_nodes, n_elems, p, rank, nranks, plan, &cpl), XFK_ERR_ARG,
                "bad partition: rank / size out of range or fewer nodes than ranks");
    info->n_extra = plan.n_extra;
    info->rank = rank;
    info->nranks = nranks;
    info->n_global = n_nodes;
    info->row0 = plan.row0;
    info->n_own = plan.n_own;
    info->n_halo = plan.n_halo;
    info->n_elems = (int)plan.elems.size();
    info->n_send = (int)plan.halo.send.size();
    info->n_recv = (int)plan.halo.recv.size();
    if (l2g) std::copy(plan.l2g.begin(), plan.l2g.end(), l2g);
    if (elems) std::copy(plan.elems.begin(), plan.elems.end(), elems);
    auto put = [](const std::vector<HaloRange> &v, int *o) {
        for (size_t k = 0; k < v.size(); ++k) {
            o[4 * k] = v[k].peer;
            o[4 * k + 1] = v[k].off;
            o[4 * k + 2] = v[k].len;
            o[4 * k + 3] = v[k].g0;
        }
    };
    if (recv) put(plan.halo.recv, recv);
    if (send) put(plan.halo.send, send);
    return XFK_OK;
}

}  // extern "C"

namespace xfk {

// the row-block plan of this rank; coupled nodes (periodic pairs and air-gap
// quad nodes) are assembled on every rank
int plan_rank(const xfk_problem_desc *d, const GlobalPrep &G, xfk_comm *comm, PartPlan &plan)
{
    std::vector<int> coupled;
    for (int k = 0; k < d->n_pbc; ++k) {
        coupled.push_back(d->pbc[3 * k]);
        coupled.push_back(d->pbc[3 * k + 1]);
    }
    for (long long k : G.age_key) {
        coupled.push_back((int)(k >> 32));
        coupled.push_back((int)(k & 0xffffffff));
    }
    std::sort(coupled.begin(), coupled.end());
    coupled.erase(std::unique(coupled.begin(), coupled.end()), coupled.end());
    XFK_REQUIRE(plan_partition(d->n_nodes, d->n_elems, d->p, comm->rank, comm->size, plan, &coupled), XFK_ERR_ARG,
                "bad partition: fewer nodes than ranks");
    return XFK_OK;
}

}  // namespace xfk

extern "C" {

int xfk_problem_create_dist(const xfk_problem_desc *d, int device, xfk_comm *comm, xfk_problem **out)
{
    XFK_REQUIRE(d && out && comm, XFK_ERR_ARG, "null argument");
    *out = nullptr;
    int rc = validate_desc(d);
    if (rc == XFK_OK) rc = check_device(device);
    if (rc != XFK_OK) return rc;
    GlobalPrep G;
    prepare_global(d, G);
    rc = prepare_magdir(d, G);
    if (rc != XFK_OK) return rc;
    rc = age_entries(d, 1.0, G.age_key, G.age_val);
    if (rc != XFK_OK) return rc;
    PartPlan plan;
    if ((rc = plan_rank(d, G, comm, plan)) != XFK_OK) return rc;
    rc = build_local(d, G, &plan, device, comm, out);
    return rc == XFK_OK ? reserve_first_solve(out) : rc;
}

int xfk_dist_get_info(const xfk_problem *P, xfk_dist_info *info)
{
    XFK_REQUIRE(P && info, XFK_ERR_ARG, "null argument");
    info->rank = P->rank;
    info->nranks = P->nranks;
    info->n_global = P->N_global;
    info->row0 = P->row0;
    info->n_own = P->N;
    info->n_halo = P->NL - P->N;
    info->n_extra = P->NR - P->N;
    info->n_elems = P->NE;
    info->n_send = (int)P->halo.send.size();
    info->n_recv = (int)P->halo.recv.size();
    return XFK_OK;
}

}  // extern "C"

namespace xfk {
// End of a solve: every stream of the problem idle (the main stream, the
// exchange side stream, the AMG's overlap and setup streams), then the blocks
// the solve freed become reusable by the next one (DevArena::recycle).
void problem_recycle(xfk_problem *P)
{
    if (!P) return;
    (void)hipSetDevice(P->device);
    if (P->stream) (void)hipStreamSynchronize(P->stream);
    if (P->side.cs) (void)hipStreamSynchronize(P->side.cs);
    if (P->amg) P->amg->sync_streams();
    P->arena.recycle();
}
static int static2d_run(xfk_problem *P, int flags, xfk_result *res);
}  // namespace xfk

extern "C" {

int xfk_static2d(xfk_problem *P, int flags, xfk_result *res)
{
    ArenaScope arena_scope(P ? &P->arena : nullptr);
    const int rc = static2d_run(P, flags, res);
    problem_recycle(P);
    return rc;
}

}  // extern "C"

namespace xfk {
static int static2d_run(xfk_problem *P, int flags, xfk_result *res)
{
    ArenaScope arena_scope(P ? &P->arena : nullptr);
    XFK_REQUIRE(P, XFK_ERR_ARG, "null problem");
    XFK_REQUIRE(!P->harmonic, XFK_ERR_ARG, "harmonic problem: use xfk_harmonic2d");
    XFK_CHECK(hipSetDevice(P->device));
    hipStream_t s = P->stream;
    ScopedEvents<5> ev;
    XFK_CHECK(ev.create());
    hipEvent_t e0 = ev[0], e1 = ev[1], e2 = ev[2], es0 = ev[3], es1 = ev[4];
    xfk_result R{};
    int rc = XFK_OK;
    float ms = 0;
    if (P->comm && (rc = P->comm->solve_boundary()) != XFK_OK) return rc;
    P->pcg_tol = 0;
    P->pcg_tol_rel = 0;
    P->time_spmv = (flags & XFK_TIME_SPMV) != 0;
    P->spmv_used = 0;
    if (P->amg) {
        P->amg->time_tail = (flags & XFK_TIME_TAIL) != 0 && P->comm;
        P->amg->tail_used = 0;
    }
    if (P->time_spmv && P->spmv_ev.empty()) {
        P->spmv_ev.resize(2 * 512);
        for (auto &ev : P->spmv_ev) XFK_CHECK(hipEventCreate(&ev));
    }
    P->last.ms_amg_setup = 0;
    P->last.amg_levels = 0;
    P->last.amg_op_complexity = 0;
    P->setup_used = 0;
    P->setup_ms_pending = 0;
    XFK_CHECK(hipEventRecord(es0, s));
    if (!P->symbolic_ready || (flags & XFK_REBUILD_SYMBOLIC)) {
        P->symbolic_ready = false;
        rc = build_symbolic(P);
        if (rc != XFK_OK) return rc;
    }
    XFK_CHECK(hipEventRecord(es1, s));   // (read after the solve: no host check here)

    const int N = P->N;
    XFK_CHECK(hipMemsetAsync(P->V.p, 0, sizeof(double) * P->NL, s));   // CBigLinProb::Create: V = 0
    double Relax = P->relax, resn = 0, lastres = 0;
    int Iter = 0;
    bool LinearFlag = !P->any_nonlinear;
    const long long cap = std::max<long long>(100000, 20LL * N);
    P->amg_reusable = false;   // a hierarchy is reused only inside one solve
    P->pc_used = XFK_PRECOND_JACOBI;
    // inexact Newton (XFK_OPT_NEWTON_INEXACT): the pass's PCG tolerance from
    // the last Newton change (Eisenstat-Walker forcing term eta |dV|/|V|);
    // the first pass of a nonlinear problem at 1e-4 (its answer moves by
    // O(1) in the next); a pass solved looser than Precision never ends the
    // loop -- the next one runs at Precision
    const bool inexact = !LinearFlag && (P->newton_inexact >= 0 ? P->newton_inexact == 1 : newton_inexact_env());
    // pass 0 (from V = 0, the initial permeabilities): to kTolFirst of |b|;
    // later passes while the Newton change is above kExactBelow: until the
    // linear residual fell by kEta from its start (Eisenstat-Walker's
    // ||r|| <= eta ||F(x_k)||, the warm start's residual being F(x_k));
    // then every pass to Precision
    constexpr double kEta = 0.05, kTolFirst = 1e-4, kExactBelow = 1e-3;
    double pass_tol = P->precision, pass_rel = 0.0;
    for (;;) {
        if (inexact) {
            pass_tol = P->precision;
            pass_rel = 0.0;
            if (Iter == 0) pass_tol = std::max(kTolFirst, P->precision);
            else if (resn >= kExactBelow) pass_rel = kEta;
        }
        P->pcg_tol = pass_tol;
        P->pcg_tol_rel = pass_rel;
        // per-pass events, read once after the loop (no host wait per pass)
        while ((int)P->pass_ev.size() < 3 * (Iter + 1)) {
            hipEvent_t ev_new = nullptr;
            XFK_CHECK(hipEventCreate(&ev_new));
            P->pass_ev.push_back(ev_new);
        }
        e0 = P->pass_ev[3 * Iter];
        e1 = P->pass_ev[3 * Iter + 1];
        e2 = P->pass_ev[3 * Iter + 2];
        XFK_CHECK(hipEventRecord(e0, s));
        if (Iter > 0 && (rc = exchange(P, P->V.p)) != XFK_OK) return rc;   // halo of V for the element B
        rc = assemble(P, Iter);
        if (rc != XFK_OK) return rc;
        // (the Newton residual and the relaxation read Vold; a linear problem
        // has neither)
        if (!LinearFlag) XFK_CHECK(hipMemcpyAsync(P->Vold.p, P->V.p, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
        XFK_CHECK(hipEventRecord(e1, s));
        static const bool nws_poll = !std::getenv("XFK_NWS_AT_POLL") || std::atoi(std::getenv("XFK_NWS_AT_POLL")) != 0;
        P->nws_at_poll = nws_poll && !LinearFlag && !P->comm;
        rc = pcg_solve(P, Iter, cap);
        P->nws_at_poll = false;
        if (rc != XFK_OK) return rc;
        XFK_CHECK(hipEventRecord(e2, s));
        R.cg_iters += P->pcg_host->iters;
        R.final_er = P->pcg_host->er;
        P->amg_last_iters = P->pcg_host->iters - P->pcg_discarded;
        if (P->amg_fresh) P->amg_fresh_iters = P->pcg_host->iters - P->pcg_discarded;

        if (!LinearFlag) {
            if (!P->nws_ready) {   // (else read with the PCG's final poll)
                launch_newton_res(s, N, P->V.p, P->Vold.p, P->partials.p, P->counters.p + 3, P->nws.p);
                const double *nws_src = reinterpret_cast<const double *>(P->nws.p);
                if (P->comm) {
                    XFK_CHECK(P->nws_glob.alloc(4));
                    rc = P->comm->allreduce_sum(nws_src, P->nws_glob.p, 2, s);
                    if (rc != XFK_OK) return rc;
                    nws_src = P->nws_glob.p;
                }
                XFK_CHECK(hipMemcpyAsync(P->nws_host, nws_src, sizeof(NewtonScalars), hipMemcpyDeviceToHost, s));
                XFK_CHECK(hipStreamSynchronize(s));
            }
            P->nws_ready = false;
            const double x = P->nws_host->dx2, y = P->nws_host->v2;
            if (y == 0) LinearFlag = true;
            else {
                lastres = resn;
                resn = sqrt(x / y);
            }
            if (Iter > 5) {
                if ((resn > lastres) && (Relax > 0.125)) Relax /= 2.;
                else Relax += 0.1 * (1. - Relax);
                launch_relax(s, N, Relax, P->V.p, P->Vold.p);
            }
        }
        if ((resn < 100. * P->precision) && (Iter > 0) && pass_tol <= P->precision && pass_rel == 0.0) LinearFlag = true;
        if (trace_newton())   // lab: one line per Newton pass
            std::fprintf(stderr, "[newton] pass %d (tol %.1e rel %.2g): pcg %lld (%lld before a restart; %s%s, levels %d) res %.3e relax %.3f\n",
                         Iter, pass_tol, pass_rel, (long long)P->pcg_host->iters, P->pcg_discarded,
                         P->pc_used == XFK_PRECOND_AMG ? "amg" : "jacobi",
                         P->pc_used == XFK_PRECOND_AMG ? (P->amg_fresh ? " fresh" : " reused") : "",
                         (P->pc_used == XFK_PRECOND_AMG && P->amg) ? P->amg->stats.levels : 0, resn, Relax);
        Iter++;
        if (LinearFlag) break;
        if (Iter > 10000) {
            set_error("nonlinear iteration did not converge");
            return XFK_ERR_NOCONV;
        }
    }
    P->pcg_tol = 0;
    P->pcg_tol_rel = 0;
    XFK_CHECK(hipStreamSynchronize(s));
    XFK_CHECK(hipEventElapsedTime(&ms, es0, es1));
    R.ms_symbolic = ms;
    for (int k = 0; k < Iter; ++k) {
        XFK_CHECK(hipEventElapsedTime(&ms, P->pass_ev[3 * k], P->pass_ev[3 * k + 1]));
        R.ms_assemble += ms;
        XFK_CHECK(hipEventElapsedTime(&ms, P->pass_ev[3 * k + 1], P->pass_ev[3 * k + 2]));
        R.ms_solve += ms;
    }
    for (int k = 0; k < P->setup_used; ++k) {
        float m = 0;
        XFK_CHECK(hipEventElapsedTime(&m, P->setup_ev[2 * k], P->setup_ev[2 * k + 1]));
        P->last.ms_amg_setup += m;
    }
    P->last.ms_amg_setup += P->setup_ms_pending;
    P->setup_used = 0;
    P->setup_ms_pending = 0;
    if (P->time_spmv && P->spmv_used > 0) {
        double sum = 0;
        for (int k = 0; k < P->spmv_used; k += 2) {
            float m = 0;
            XFK_CHECK(hipEventElapsedTime(&m, P->spmv_ev[k], P->spmv_ev[k + 1]));
            sum += m;
        }
        R.spmv_samples = P->spmv_used / 2;
        R.spmv_ms_avg = sum / R.spmv_samples;
    }
    if (P->amg && P->amg->time_tail) {
        if ((rc = P->amg->tail_read(R.ms_rep_cycle, R.rep_cycles, R.ms_rep_setup)) != XFK_OK) return rc;
        P->amg->time_tail = false;
    }
    R.prec_fallback = P->f64_fallback ? 1 : 0;
    R.newton_iters = Iter;
    R.last_res = resn;
    R.nnz = P->nnz_own;
    R.ncolors = P->ncolors;
    R.color_rounds = P->color_rounds;
    R.precond = P->pc_used;
    R.amg_levels = P->last.amg_levels;
    R.amg_op_complexity = P->last.amg_op_complexity;
    R.ms_amg_setup = P->last.ms_amg_setup;
    P->last = R;
    if (res) *res = R;
    return XFK_OK;
}
}  // namespace xfk

extern "C" {

int xfk_get_solution(xfk_problem *P, double *A)
{
    XFK_REQUIRE(P && A, XFK_ERR_ARG, "null argument");
    XFK_REQUIRE(P->symbolic_ready, XFK_ERR_ARG, "no solution yet");
    XFK_CHECK(hipSetDevice(P->device));
    hipStream_t s = P->stream;
    if (!P->comm) {
        XFK_CHECK(d2h(A, P->V.p, sizeof(double) * P->N, s));
        for (int i = 0; i < P->N; ++i) A[i] = A[i] * kC;   // L.b[i] = L.V[i]*c (static2d.cpp:1018-1021)
        if (P->axi)   // flux 2 pi r A, Webers (staticaxi.cpp:774-779)
            for (int i = 0; i < P->N; ++i) A[i] *= (P->axi_x[i] * 0.01 * 2 * kPI);
        return XFK_OK;
    }
    // sharded: all-gather the owned rows (padded to the largest block)
    const int R = P->nranks;
    size_t maxn = 0;
    for (int q = 0; q < R; ++q)
        maxn = std::max<size_t>(maxn, row_begin(P->N_global, q + 1, R) - row_begin(P->N_global, q, R));
    XFK_CHECK(P->gather_buf.alloc(maxn * (1 + R)));
    double *send = P->gather_buf.p, *recv = P->gather_buf.p + maxn;
    XFK_CHECK(hipMemsetAsync(send, 0, sizeof(double) * maxn, s));
    XFK_CHECK(hipMemcpyAsync(send, P->V.p, sizeof(double) * P->N, hipMemcpyDeviceToDevice, s));
    int rc = P->comm->allgather(send, recv, maxn, s);
    if (rc != XFK_OK) return rc;
    std::vector<double> h(maxn * R);
    XFK_CHECK(d2h(h.data(), recv, sizeof(double) * h.size(), s));
    for (int q = 0; q < R; ++q) {
        const long long r0 = row_begin(P->N_global, q, R), r1 = row_begin(P->N_global, q + 1, R);
        for (long long i = r0; i < r1; ++i) A[i] = h[(size_t)q * maxn + (i - r0)] * kC;
    }
    if (P->axi)
        for (int i = 0; i < P->N_global; ++i) A[i] *= (P->axi_x[i] * 0.01 * 2 * kPI);
    return XFK_OK;
}

int xfk_get_circuits(xfk_problem *P, int *ccase, double *J, double *dV)
{
    XFK_REQUIRE(P, XFK_ERR_ARG, "null problem");
    if (P->ncircs == 0) return XFK_OK;
    std::vector<DevCirc> h(P->ncircs);
    XFK_CHECK(d2h(h.data(), P->circs.p, sizeof(DevCirc) * P->ncircs, P->stream));
    for (int k = 0; k < P->ncircs; ++k) {
        if (ccase) ccase[k] = h[k].ccase;
        if (J) J[k] = h[k].J;
        if (dV) dV[k] = h[k].dV;
    }
    return XFK_OK;
}

long long xfk_get_nnz(xfk_problem *P) { return P && xfk_resolve_nnz(P) == XFK_OK ? P->nnz_own : -1; }

double xfk_spmv_col_bytes(xfk_problem *P)
{
    if (!P || xfk_resolve_nnz(P) != XFK_OK) return -1.0;
    const unsigned short *c16;
    const int *cbase;
    spmv_col16(P, c16, cbase);
    if (!c16 || P->nnz_own <= 0) return 4.0;
    const int N = P->N, nt = (N + kCgBlock - 1) / kCgBlock;
    std::vector<int> base(nt), rp(N + 1);
    if (d2h(base.data(), cbase, sizeof(int) * nt, P->stream) != hipSuccess ||
        d2h(rp.data(), P->rowptr.p, sizeof(int) * (N + 1), P->stream) != hipSuccess)
        return -1.0;
    long long wide = 0;
    for (int t = 0; t < nt; ++t)
        if (base[t] == kNoColBase) wide += rp[std::min(N, (t + 1) * kCgBlock)] - rp[t * kCgBlock];
    return (2.0 * (double)P->nnz_own + 2.0 * (double)wide) / (double)P->nnz_own;
}

int xfk_get_csr(xfk_problem *P, int *rowptr, int *col, double *val, double *b)
{
    XFK_REQUIRE(P && P->symbolic_ready, XFK_ERR_ARG, "no assembled system");
    XFK_CHECK(hipSetDevice(P->device));
    XFK_CHECK(hipStreamSynchronize(P->stream));
    if (xfk_resolve_nnz(P) != XFK_OK) return XFK_ERR_HIP;
    if (rowptr) XFK_CHECK(d2h(rowptr, P->rowptr.p, sizeof(int) * (P->N + 1), P->stream));
    if (col) XFK_CHECK(d2h(col, P->col.p, sizeof(int) * P->nnz_own, P->stream));
    if (val) XFK_CHECK(d2h(val, P->val.p, sizeof(double) * P->nnz_own, P->stream));
    if (b) XFK_CHECK(d2h(b, P->b.p, sizeof(double) * P->N, P->stream));
    return XFK_OK;
}

int xfk_get_stream(xfk_problem *P, void **st)
{
    XFK_REQUIRE(P && st, XFK_ERR_ARG, "null argument");
    *st = (void *)P->stream;
    return XFK_OK;
}

int xfk_pcg_solve_csr(int n, const int *rowptr, const int *col, const double *val, const double *b, double *V,
                      int flag, double precision, int device, long long *iters, double *er)
{
    return xfk_pcg_solve_csr_pc(n, rowptr, col, val, b, V, flag, precision, device, XFK_PRECOND_JACOBI, iters, er);
}

int xfk_set_option(xfk_problem *P, int option, double value)
{
    XFK_REQUIRE(P, XFK_ERR_ARG, "null problem");
    switch (option) {
    case XFK_OPT_PRECOND:
        XFK_REQUIRE(value == XFK_PRECOND_JACOBI || value == XFK_PRECOND_AMG, XFK_ERR_ARG, "unknown preconditioner");
        P->precond = (int)value;
        return XFK_OK;
    case XFK_OPT_AMG_SWEEPS:
        XFK_REQUIRE(value >= 1 && value <= 8 && value == (int)value, XFK_ERR_ARG, "AMG sweeps must be 1..8");
        P->amg_sweeps = (int)value;
        return XFK_OK;
    case XFK_OPT_AMG_THETA:
        XFK_REQUIRE(value >= 0.0 && value < 1.0, XFK_ERR_ARG, "AMG strength threshold must be in [0, 1)");
        P->amg_theta = value;
        return XFK_OK;
    case XFK_OPT_AMG_OMEGA:
        XFK_REQUIRE(value > 0.0 && value < 2.0, XFK_ERR_ARG, "AMG Jacobi weight factor must be in (0, 2)");
        P->amg_omega = value;
        return XFK_OK;
    case XFK_OPT_AMG_REPLICATE:
        XFK_REQUIRE(value >= 0 && value <= 2e9 && value == (int)value, XFK_ERR_ARG,
                    "AMG replication threshold must be a row count");
        P->amg_replicate = (int)value;
        return XFK_OK;
    case XFK_OPT_AMG_REUSE:
        XFK_REQUIRE(value == 0 || value == 1, XFK_ERR_ARG, "AMG reuse is 0 or 1");
        P->amg_reuse = (int)value;
        return XFK_OK;
    case XFK_OPT_AMG_DENSE:
        XFK_REQUIRE(value >= 16 && value <= kAmgDenseMax && value == (int)value, XFK_ERR_ARG,
                    "AMG dense coarsest size must be 16..2048 rows");
        P->amg_dense = (int)value;
        return XFK_OK;
    case XFK_OPT_AMG_FOLD:
        XFK_REQUIRE(value == 0 || value == 1, XFK_ERR_ARG, "AMG fold is 0 or 1");
        P->amg_fold = (int)value;
        return XFK_OK;
    case XFK_OPT_AMG_COL16:
        XFK_REQUIRE(value == 0 || value == 1, XFK_ERR_ARG, "AMG 16-bit columns is 0 or 1");
        P->amg_col16 = (int)value;
        return XFK_OK;
    case XFK_OPT_AMG_F32:
        XFK_REQUIRE(value == 0 || value == 1, XFK_ERR_ARG, "AMG f32 level-0 operators is 0 or 1");
        P->amg_f32 = (int)value;
        return XFK_OK;
    case XFK_OPT_NEWTON_INEXACT:
        XFK_REQUIRE(value == 0 || value == 1, XFK_ERR_ARG, "inexact Newton is 0 or 1");
        P->newton_inexact = (int)value;
        return XFK_OK;
    case XFK_OPT_AMG_WLEVEL:
        XFK_REQUIRE(value >= -2 && value < kAmgMaxLevels && value == (int)value, XFK_ERR_ARG,
                    "AMG W-cycle level must be -2, -1 or a level index");
        P->amg_wlevel = (int)value;
        return XFK_OK;
    default:
        set_error("unknown option");
        return XFK_ERR_ARG;
    }
}

int xfk_pcg_solve_csr_pc(int n, const int *rowptr, const int *col, const double *val, const double *b, double *V,
                         int flag, double precision, int device, int precond, long long *iters, double *er)
{
    XFK_REQUIRE(precond == XFK_PRECOND_JACOBI || precond == XFK_PRECOND_AMG, XFK_ERR_ARG, "unknown preconditioner");
    XFK_REQUIRE(n > 0 && rowptr && col && val && b && V, XFK_ERR_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("no HIP device available (the fsolver hot path has no CPU fallback)");
        return XFK_ERR_HIP;
    }
    XFK_CHECK(hipSetDevice(device));
    xfk_problem *P = new xfk_problem();
    P->device = device;
    P->N = n;
    P->NL = n;
    P->nnz = rowptr[n];
    P->nnz_own = P->nnz;
    P->NR = n;
    P->precision = precision;
    P->precond = precond;
    int rc = XFK_OK;
    hipError_t e = stream_acquire(&P->stream);
    // diagonal positions
    std::vector<int> diag(n, -1);
    for (int i = 0; i < n; ++i)
        for (int k = rowptr[i]; k < rowptr[i + 1]; ++k)
            if (col[k] == i) diag[i] = k;
    for (int i = 0; i < n && rc == XFK_OK; ++i)
        if (diag[i] < 0) {
            set_error("row without a diagonal entry");
            rc = XFK_ERR_SINGULAR;
        }
    hipStream_t s = P->stream;
    if (e == hipSuccess) e = upload(P->rowptr, rowptr, (size_t)n + 1, s);
    if (e == hipSuccess) e = upload(P->col, col, (size_t)P->nnz, s);
    if (e == hipSuccess) e = upload(P->val, val, (size_t)P->nnz, s);
    if (e == hipSuccess) e = upload(P->b, b, (size_t)n, s);
    if (e == hipSuccess) e = upload(P->V, V, (size_t)n, s);
    if (e == hipSuccess) e = upload(P->diag, diag.data(), (size_t)n, s);
    for (DBuf<double> *v : {&P->P, &P->dinv})
        if (e == hipSuccess) e = v->alloc(n);
    if (e == hipSuccess) e = P->partials.alloc(2 * kRedGrid);
    if (e == hipSuccess) e = P->counters.alloc(8);
    if (e == hipSuccess) e = hipMemsetAsync(P->counters.p, 0, sizeof(unsigned) * 8, s);
    if (e == hipSuccess) e = P->pcg.alloc(1);
    if (e == hipSuccess) e = pinned_malloc((void **)&P->pcg_host, sizeof(CgState));
    if (e == hipSuccess) e = pinned_malloc((void **)&P->hpin, 16 * sizeof(int));
    if (e != hipSuccess) {
        set_error(std::string("pcg setup failed: ") + hipGetErrorString(e));
        rc = XFK_ERR_HIP;
    }
    if (rc == XFK_OK) rc = pcg_solve(P, flag, std::max<long long>(100000, 20LL * n));
    if (rc == XFK_OK || rc == XFK_ERR_NOCONV) {
        if (d2h(V, P->V.p, sizeof(double) * n, P->stream) != hipSuccess) rc = XFK_ERR_HIP;
        if (iters) *iters = P->pcg_host->iters;
        if (er) *er = P->pcg_host->er;
    }
    xfk_problem_destroy(P);
    return rc;
}

int xfk_phase_profile(xfk_problem *P, int iters, int flags, xfk_phase *out, int cap, int *count)
{
    XFK_REQUIRE(P && P->symbolic_ready && iters > 0 && out && count, XFK_ERR_ARG, "no assembled system");
    XFK_REQUIRE(!P->harmonic && !P->comm, XFK_ERR_UNSUPPORTED, "phase profile: single-device static problems only");
    XFK_REQUIRE(P->amg && P->pc_used == XFK_PRECOND_AMG, XFK_ERR_ARG, "phase profile: solve with the AMG first");
    XFK_CHECK(hipSetDevice(P->device));
    hipStream_t s = P->stream;
    PhaseProf prof;
    prof.s = s;
    g_prof = &prof;
    int rc = XFK_OK;
    // always a fresh hierarchy built inside pcg_start (as in a solve's first
    // pass), never a Newton refresh of the last one: a refresh runs level 0
    // unfolded, which is not the cycle a solve's first pass times.  Without
    // XFK_PROFILE_SETUP the setup's own phases are dropped from the table.
    P->amg_reusable = false;
    if (rc == XFK_OK) {
        const double tol = P->precision;
        P->precision = 0.0;   // never converges: fixed iteration count
        rc = pcg_start(P, 1);
        P->precision = tol;
        for (int k = 0; rc == XFK_OK && k < iters; ++k) rc = pcg_iteration(P, k, false);
    }
    g_prof = nullptr;
    if (rc != XFK_OK) return rc;
    XFK_CHECK(hipStreamSynchronize(s));
    std::vector<std::string> order;
    std::map<std::string, xfk_phase> agg;
    for (const auto &r : prof.recs) {
        if (r.ev0 < 0 || r.ev1 < 0) continue;
        if (!(flags & XFK_PROFILE_SETUP) && r.name.compare(0, 5, "setup") == 0) continue;
        float ms = 0;
        XFK_CHECK(hipEventElapsedTime(&ms, prof.ev[r.ev0], prof.ev[r.ev1]));
        auto it = agg.find(r.name);
        if (it == agg.end()) {
            xfk_phase ph{};
            std::snprintf(ph.name, sizeof ph.name, "%s", r.name.c_str());
            it = agg.emplace(r.name, ph).first;
            order.push_back(r.name);
        }
        xfk_phase &ph = it->second;
        ph.bytes_per_call = (ph.bytes_per_call * ph.calls + r.bytes) / (ph.calls + 1);
        ph.calls += 1;
        ph.ms_total += ms;
    }
    int k = 0;
    for (const auto &nm : order) {
        if (k >= cap) break;
        out[k++] = agg[nm];
    }
    *count = k;
    return XFK_OK;
}

int xfk_pcg_time(xfk_problem *P, int iters, double *ms_spmv, double *ms_iter)
{
    XFK_REQUIRE(P && P->symbolic_ready && iters > 0, XFK_ERR_ARG, "no assembled system");
    XFK_CHECK(hipSetDevice(P->device));
    hipStream_t s = P->stream;
    const double tol = P->precision;
    P->precision = 0.0;   // never converges: fixed iteration count
    int rc = pcg_start(P, 1);
    P->precision = tol;
    if (rc != XFK_OK) return rc;
    if ((int)P->spmv_ev.size() < 2 * iters) {
        for (auto &ev : P->spmv_ev) (void)hipEventDestroy(ev);
        P->spmv_ev.resize(2 * iters);
        for (auto &ev : P->spmv_ev) XFK_CHECK(hipEventCreate(&ev));
    }
    ScopedEvents<2> ev;
    XFK_CHECK(ev.create());
    hipEvent_t t0 = ev[0], t1 = ev[1];
    if (const char *ge = std::getenv("XFK_PCG_GRAPH")) {
        // lab: the same iterations launched one by one vs replayed from a
        // hipGraph of K captured iterations (no events inside); ms_spmv gets
        // the stream time per iteration, ms_iter the graph time per iteration
        const int K = std::max(2, std::atoi(ge) & ~1);
        for (int k = 0; k < 2; ++k)
            if ((rc = pcg_iteration(P, k, false)) != XFK_OK) return rc;
        XFK_CHECK(hipEventRecord(t0, s));
        for (int k = 2; k < 2 + iters; ++k)
            if ((rc = pcg_iteration(P, k, false)) != XFK_OK) return rc;
        XFK_CHECK(hipEventRecord(t1, s));
        XFK_CHECK(hipEventSynchronize(t1));
        float ts = 0;
        XFK_CHECK(hipEventElapsedTime(&ts, t0, t1));
        hipGraph_t g = nullptr;
        hipGraphExec_t ge2 = nullptr;
        XFK_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int k = 2; k < 2 + K; ++k)
            if ((rc = pcg_iteration(P, k, false)) != XFK_OK) {
                (void)hipStreamEndCapture(s, &g);
                return rc;
            }
        XFK_CHECK(hipStreamEndCapture(s, &g));
        XFK_CHECK(hipGraphInstantiate(&ge2, g, nullptr, nullptr, 0));
        XFK_CHECK(hipGraphLaunch(ge2, s));   // warm
        const int R = std::max(1, iters / K);
        XFK_CHECK(hipEventRecord(t0, s));
        for (int q = 0; q < R; ++q) XFK_CHECK(hipGraphLaunch(ge2, s));
        XFK_CHECK(hipEventRecord(t1, s));
        XFK_CHECK(hipEventSynchronize(t1));
        float tg = 0;
        XFK_CHECK(hipEventElapsedTime(&tg, t0, t1));
        (void)hipGraphExecDestroy(ge2);
        (void)hipGraphDestroy(g);
        if (ms_spmv) *ms_spmv = ts / iters;
        if (ms_iter) *ms_iter = tg / (R * K);
        return XFK_OK;
    }
    P->spmv_used = 0;
    XFK_CHECK(hipEventRecord(t0, s));
    for (int k = 0; k < iters; ++k) {
        rc = pcg_iteration(P, k, true);
        if (rc != XFK_OK) return rc;
    }
    XFK_CHECK(hipEventRecord(t1, s));
    XFK_CHECK(hipEventSynchronize(t1));
    double sum = 0;
    for (int k = 0; k < P->spmv_used; k += 2) {
        float m = 0;
        XFK_CHECK(hipEventElapsedTime(&m, P->spmv_ev[k], P->spmv_ev[k + 1]));
        sum += m;
    }
    float tot = 0;
    XFK_CHECK(hipEventElapsedTime(&tot, t0, t1));
    if (ms_spmv) *ms_spmv = sum / (P->spmv_used / 2);
    if (ms_iter) *ms_iter = tot / iters;
    P->spmv_used = 0;
    return XFK_OK;
}

}  // extern "C"
