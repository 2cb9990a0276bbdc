// Row-block partition planning (see xfk_partition.h).  Host code only.
#include "xfk_partition.h"

#include <algorithm>
#include <climits>

namespace xfk {

namespace {

// sorted unique nodes -> runs [g0, g0 + len)
void to_runs(const std::vector<int> &v, std::vector<std::pair<int, int>> &out)
{
    out.clear();
    for (size_t k = 0; k < v.size();) {
        size_t e = k + 1;
        while (e < v.size() && v[e] == v[e - 1] + 1) ++e;
        out.push_back({v[k], (int)(e - k)});
        k = e;
    }
}

}  // namespace

bool plan_partition(int n_nodes, int n_elems, const int *p, int rank, int nranks, PartPlan &out,
                    const std::vector<int> *coupled)
{
    out = PartPlan();
    if (nranks < 1 || rank < 0 || rank >= nranks || n_nodes < nranks) return false;
    out.rank = rank;
    out.nranks = nranks;
    out.n_global = n_nodes;
    std::vector<int> start(nranks + 1);
    for (int q = 0; q <= nranks; ++q) start[q] = (int)row_begin(n_nodes, q, nranks);
    auto owner = [&](int g) {
        return (int)(std::upper_bound(start.begin(), start.end(), g) - start.begin()) - 1;
    };
    out.row0 = start[rank];
    out.n_own = start[rank + 1] - start[rank];

    // coupled nodes and the elements touching them (held by every rank)
    std::vector<char> isx(coupled && !coupled->empty() ? n_nodes : 0, 0);
    for (int g : coupled ? *coupled : std::vector<int>())
        if (g >= 0 && g < n_nodes) isx[g] = 1;
    auto touches_x = [&](const int *n) { return !isx.empty() && (isx[n[0]] || isx[n[1]] || isx[n[2]]); };
    std::vector<char> ring(isx.empty() ? 0 : n_nodes, 0);   // nodes of those elements

    // lo/hi[q * nranks + a]: span of the rows owned by a that rank q needs
    // for its ordinary (owned-row) elements
    const size_t R2 = (size_t)nranks * nranks;
    std::vector<int> lo(R2, INT_MAX), hi(R2, -1);
    for (int e = 0; e < n_elems; ++e) {
        const int *n = p + 3LL * e;
        const bool tx = touches_x(n);
        if (tx)
            for (int j = 0; j < 3; ++j) ring[n[j]] = 1;
        int o[3] = {owner(n[0]), owner(n[1]), owner(n[2])};
        if (o[0] == o[1] && o[1] == o[2]) {
            if (o[0] == rank || tx) out.elems.push_back(e);
            continue;
        }
        if (o[0] == rank || o[1] == rank || o[2] == rank || tx) out.elems.push_back(e);
        for (int j = 0; j < 3; ++j) {
            const int q = o[j];
            if ((j == 1 && q == o[0]) || (j == 2 && (q == o[0] || q == o[1]))) continue;   // each q once
            for (int k = 0; k < 3; ++k) {
                if (o[k] == q) continue;
                const size_t ix = (size_t)q * nranks + o[k];
                lo[ix] = std::min(lo[ix], n[k]);
                hi[ix] = std::max(hi[ix], n[k]);
            }
        }
    }

    // what rank q receives from peer a: the coupled nodes of a (every rank
    // needs them all), then the span plus the ring of the coupled elements,
    // without the coupled nodes
    std::vector<std::pair<int, int>> runs;
    auto xruns = [&](int a, std::vector<std::pair<int, int>> &r) {
        std::vector<int> v;
        for (int g = start[a]; g < start[a + 1] && !isx.empty(); ++g)
            if (isx[g]) v.push_back(g);
        to_runs(v, r);
    };
    auto oruns = [&](int q, int a, std::vector<std::pair<int, int>> &r) {
        const size_t ix = (size_t)q * nranks + a;
        std::vector<int> v;
        if (isx.empty()) {
            r.clear();
            if (hi[ix] >= 0) r.push_back({lo[ix], hi[ix] - lo[ix] + 1});
            return;
        }
        for (int g = start[a]; g < start[a + 1]; ++g) {
            const bool in_span = hi[ix] >= 0 && g >= lo[ix] && g <= hi[ix];
            if ((in_span || ring[g]) && !isx[g]) v.push_back(g);
        }
        to_runs(v, r);
    };

    out.l2g.resize(out.n_own);
    for (int i = 0; i < out.n_own; ++i) out.l2g[i] = out.row0 + i;
    int off = out.n_own;
    for (int pass = 0; pass < 2; ++pass)
        for (int a = 0; a < nranks; ++a) {
            if (a == rank) continue;
            if (pass == 0) xruns(a, runs);
            else oruns(rank, a, runs);
            for (auto &rr : runs) {
                HaloRange r{a, off, rr.second, rr.first};
                out.halo.recv.push_back(r);
                for (int g = r.g0; g < r.g0 + r.len; ++g) out.l2g.push_back(g);
                off += r.len;
            }
            if (pass == 0) out.n_extra = off - out.n_own;
        }
    out.n_halo = off - out.n_own;
    // sends: per peer q the same ranges q receives from this rank, in q's order
    std::vector<std::pair<int, int>> xr;
    xruns(rank, xr);
    for (int q = 0; q < nranks; ++q) {
        if (q == rank) continue;
        for (auto &rr : xr) out.halo.send.push_back(HaloRange{q, rr.first - out.row0, rr.second, rr.first});
        oruns(q, rank, runs);
        for (auto &rr : runs) out.halo.send.push_back(HaloRange{q, rr.first - out.row0, rr.second, rr.first});
    }
    return true;
}

}  // namespace xfk
