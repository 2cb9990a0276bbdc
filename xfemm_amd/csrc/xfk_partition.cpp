// Row-block partition planning (see xfk_partition.h).  Host code only.
#include "xfk_partition.h"

#include <algorithm>
#include <climits>

namespace xfk {

bool plan_partition(int n_nodes, int n_elems, const int *p, int rank, int nranks, PartPlan &out)
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

    // lo/hi[q * nranks + a]: span of the rows owned by a that rank q needs
    const size_t R2 = (size_t)nranks * nranks;
    std::vector<int> lo(R2, INT_MAX), hi(R2, -1);
    for (int e = 0; e < n_elems; ++e) {
        const int *n = p + 3LL * e;
        int o[3] = {owner(n[0]), owner(n[1]), owner(n[2])};
        if (o[0] == o[1] && o[1] == o[2]) {
            if (o[0] == rank) out.elems.push_back(e);
            continue;
        }
        if (o[0] == rank || o[1] == rank || o[2] == rank) out.elems.push_back(e);
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

    out.l2g.resize(out.n_own);
    for (int i = 0; i < out.n_own; ++i) out.l2g[i] = out.row0 + i;
    int off = out.n_own;
    for (int a = 0; a < nranks; ++a) {
        const size_t ix = (size_t)rank * nranks + a;
        if (a == rank || hi[ix] < 0) continue;
        HaloRange r{a, off, hi[ix] - lo[ix] + 1, lo[ix]};
        out.halo.recv.push_back(r);
        for (int g = r.g0; g < r.g0 + r.len; ++g) out.l2g.push_back(g);
        off += r.len;
    }
    out.n_halo = off - out.n_own;
    for (int q = 0; q < nranks; ++q) {
        const size_t ix = (size_t)q * nranks + rank;
        if (q == rank || hi[ix] < 0) continue;
        out.halo.send.push_back(HaloRange{q, lo[ix] - out.row0, hi[ix] - lo[ix] + 1, lo[ix]});
    }
    return true;
}

}  // namespace xfk
