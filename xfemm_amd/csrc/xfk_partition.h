// Row-block partition of the fsolver mesh for the sharded solve (host only).
//
// Rank q owns the contiguous global rows [row_begin(q), row_begin(q+1)) of the
// node numbering it is given (the reference renumbers nodes with
// Cuthill-McKee, FSolver::Cuthill, cfemm/libfemm/feasolver.cpp, so row blocks
// of a banded matrix touch few neighbours).  Its local problem holds every
// element with at least one owned node ("ghost" elements are replicated, so
// assembly needs no communication), and the nodes of those elements it does
// not own form the halo.  The halo nodes owned by one peer are received as ONE
// contiguous global range [g0, g0 + len) of that peer's rows -- the span of
// what is needed, so a send or receive is a plain slice of the vector and no
// pack/unpack kernel runs per exchange.
//
// Local numbering: owned rows first (local = global - row0), then the receive
// ranges in ascending peer order.
//
// Coupled nodes (periodic / antiperiodic pairs and air-gap quad nodes, whose
// rows the reference's Periodicity / AntiPeriodicity mix with their partners'
// and whose air-gap couplings reach across the machine): every rank holds
// every element touching one of them and assembles their rows itself -- the
// "extra" rows, local ids n_own .. n_own + n_extra - 1 (the first receive
// ranges, before the ordinary halo) -- so the periodic averaging map of its
// owned rows finds every pre-map entry locally.  Only the owned rows enter
// the solve.  A peer may then send several ranges to one rank: the coupled
// nodes first, then the ordinary span, in the same order on both sides.
#pragma once

#include <vector>

namespace xfk {

struct HaloRange {
    int peer;   // the other rank
    int off;    // local offset in the vector (owned part for sends, halo part for receives)
    int len;    // entries
    int g0;     // first global row of the range
};

struct HaloPlan {
    std::vector<HaloRange> send, recv;   // ascending peer order
};

struct PartPlan {
    int rank = 0, nranks = 1;
    int n_global = 0;
    int row0 = 0, n_own = 0, n_halo = 0;
    int n_extra = 0;         // coupled nodes owned elsewhere: assembled here too (local n_own ..)
    std::vector<int> l2g;    // local node -> global node, n_own + n_halo
    std::vector<int> elems;  // global ids of the local elements, ascending
    HaloPlan halo;
};

inline long long row_begin(long long n, int q, int nranks) { return n * q / nranks; }

// Plan rank `rank` of `nranks` for a mesh of n_nodes nodes and n_elems
// triangles p (3 per element).  Every rank computes the same global picture
// (who needs which range from whom) from the same mesh, so no exchange of
// lists is needed.  Returns false if a rank would own no rows.
bool plan_partition(int n_nodes, int n_elems, const int *p, int rank, int nranks, PartPlan &out,
                    const std::vector<int> *coupled = nullptr);

}  // namespace xfk
