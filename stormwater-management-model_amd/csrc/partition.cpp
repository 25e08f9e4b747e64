// partition.cpp -- owner assignment, ghost links, neighbour lists and the
// local node -> link incidence (see partition.h).
#include "partition.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <numeric>
#include <string>
#include <unordered_map>

namespace swx {

namespace {

// smallest-index root union-find (deferred-node groups)
int findRoot(std::vector<int>& up, int a)
{
    while (up[a] != a) {
        up[a] = up[up[a]];
        a = up[a];
    }
    return a;
}

}  // namespace

int buildPartition(const Network& net, Partition& part, std::string* msg)
{
    const int nN = net.nNodes(), nL = net.nLinks(), R = part.nranks;
    if (R < 1 || part.rank < 0 || part.rank >= R) {
        if (msg) *msg = "invalid rank / number of ranks";
        return 500;
    }
    const int me = part.rank;
    // nodes: contiguous blocks of the node index; or (SWMM5_PART_BLOCK = B > 0)
    // blocks of B nodes dealt to the ranks in turn, so that a hot region (the
    // synthetic grids' surcharged corner next to the outlet: a 2-rank strip
    // split gives the last strip 3x the first one's sparse iterations) is
    // shared by every rank, at the price of more cut links
    part.nodeOwner.assign(nN, 0);
    long long block = 0;
    if (const char* b = getenv("SWMM5_PART_BLOCK")) block = atoll(b);
    const bool weighted = block <= 0 && (int)part.weight.size() == nN && nN > 0;
    // the nodes of `idx` (ascending node order) cut into nb contiguous blocks
    // of equal weight (node i to the block whose share holds the midpoint of
    // its weight interval); block b goes to rank rankOf(b)
    auto equalWeightBlocks = [&](const std::vector<int>& idx, int nb, auto rankOf) {
        double total = 0.0;
        for (int i : idx) total += std::max(part.weight[i], 0.0);
        double run = 0.0;
        const long long m = (long long)idx.size();
        for (long long q = 0; q < m; q++) {
            const double w = std::max(part.weight[idx[q]], 0.0);
            const double mid = run + 0.5 * w;
            run += w;
            int b = total > 0.0 ? (int)(mid * nb / total) : (int)(q * nb / m);
            part.nodeOwner[idx[q]] = rankOf(std::min(std::max(b, 0), nb - 1));
        }
    };
    auto same = [](int b) { return b; };
    if (weighted && part.mode == PART_TWO_REGION) {
        double lo = part.weight[0], hi = part.weight[0];
        for (int i = 0; i < nN; i++) {
            lo = std::min(lo, part.weight[i]);
            hi = std::max(hi, part.weight[i]);
        }
        const double cut = lo + 0.25 * (hi - lo);
        std::vector<int> hot, cold;
        for (int i = 0; i < nN; i++) (hi > lo && part.weight[i] >= cut ? hot : cold).push_back(i);
        // the hot region in 2R blocks dealt 0, 1, .., R-1, R-1, .., 1, 0: a
        // trend of the work across the region (the surcharge front at its
        // upstream edge) cancels between each rank's two blocks
        equalWeightBlocks(hot, 2 * R, [R](int b) { return b < R ? b : 2 * R - 1 - b; });
        equalWeightBlocks(cold, R, same);
    } else if (weighted) {
        std::vector<int> all(nN);
        std::iota(all.begin(), all.end(), 0);
        equalWeightBlocks(all, R, same);
    } else {
        for (int i = 0; i < nN; i++)
            part.nodeOwner[i] = block > 0 ? (int)((i / block) % R) : (int)((long long)i * R / nN);
    }
    // pumps / regulators: their end nodes ("deferred": updated by k_nc from
    // running link-order totals) and every link touching one stay on one rank,
    // the owner of the group's smallest node
    std::vector<char> deferred(nN, 0);
    for (int j = 0; j < nL; j++)
        if (!net.isTrueConduit(j)) deferred[net.node1[j]] = deferred[net.node2[j]] = 1;
    {
        std::vector<int> up(nN);
        std::iota(up.begin(), up.end(), 0);
        for (int j = 0; j < nL; j++) {
            int a = net.node1[j], b = net.node2[j];
            if (!deferred[a] || !deferred[b]) continue;
            a = findRoot(up, a);
            b = findRoot(up, b);
            if (a != b) up[std::max(a, b)] = std::min(a, b);
        }
        for (int i = 0; i < nN; i++)
            if (deferred[i]) part.nodeOwner[i] = part.nodeOwner[findRoot(up, i)];
    }
    // conduits: owner of node1 (of the deferred end, if one end is deferred);
    // outfalls: owner of their conduit
    part.linkOwner.assign(nL, 0);
    for (int j = 0; j < nL; j++) {
        int n1 = net.node1[j], n2 = net.node2[j];
        part.linkOwner[j] = part.nodeOwner[(deferred[n2] && !deferred[n1]) ? n2 : n1];
    }
    for (int j = 0; j < nL; j++) {
        int n1 = net.node1[j], n2 = net.node2[j];
        if (net.nodeType[n2] == OUTFALL) part.nodeOwner[n2] = part.linkOwner[j];
        else if (net.nodeType[n1] == OUTFALL) part.nodeOwner[n1] = part.linkOwner[j];
    }
    // holders of each node: its owner and the owners of the links touching it
    // (a rank holds a node it owns or that one of its links touches); the
    // nodes with more than one holder are few (strip boundaries)
    std::unordered_map<int, std::vector<int>> extra;
    auto addHolder = [&](int n, int r) {
        if (r == part.nodeOwner[n]) return;
        std::vector<int>& v = extra[n];
        if (std::find(v.begin(), v.end(), r) == v.end()) v.push_back(r);
    };
    for (int j = 0; j < nL; j++) {
        addHolder(net.node1[j], part.linkOwner[j]);
        addHolder(net.node2[j], part.linkOwner[j]);
    }
    auto holds = [&](int n, int r) {
        if (part.nodeOwner[n] == r) return true;
        auto it = extra.find(n);
        return it != extra.end() && std::find(it->second.begin(), it->second.end(), r) != it->second.end();
    };
    // a link is a ghost on every rank other than its owner that holds one of
    // its end nodes; deferred nodes must not be held by two ranks (k_nc runs
    // on one rank)
    for (const auto& kv : extra)
        if (deferred[kv.first]) {
            if (msg) *msg = "a pump / regulator end node is shared between ranks";
            return 500;
        }
    // ghost sets: (receiver, sender, link); global slots: links that are a
    // ghost anywhere
    struct G { int to, from, link; };
    std::vector<G> ghosts;
    std::vector<int> slotLinks;
    for (int j = 0; j < nL; j++) {
        const int s = part.linkOwner[j];
        int rs[8], nr = 0;
        for (int n : {net.node1[j], net.node2[j]}) {
            auto add = [&](int r) {
                if (r == s) return;
                for (int q = 0; q < nr; q++) if (rs[q] == r) return;
                if (nr < 8) rs[nr++] = r;
            };
            add(part.nodeOwner[n]);
            auto it = extra.find(n);
            if (it != extra.end()) for (int r : it->second) add(r);
        }
        if (nr == 0) continue;
        slotLinks.push_back(j);
        for (int q = 0; q < nr; q++) ghosts.push_back({rs[q], s, j});
    }
    part.nSlotGlobal = (int)slotLinks.size();
    std::unordered_map<int, int> slotOf;
    slotOf.reserve(slotLinks.size() * 2 + 1);
    for (size_t k = 0; k < slotLinks.size(); k++) slotOf[slotLinks[k]] = (int)k;

    // ---- this rank's held nodes and owned links --------------------------
    part.lnode.clear();
    part.gnode.assign(nN, -1);
    for (int i = 0; i < nN; i++)
        if (holds(i, me)) {
            part.gnode[i] = (int)part.lnode.size();
            part.lnode.push_back(i);
        }
    part.llink.clear();
    part.glink.assign(nL, -1);
    for (int j = 0; j < nL; j++)
        if (part.linkOwner[j] == me) {
            part.glink[j] = (int)part.llink.size();
            part.llink.push_back(j);
        }
    const int n = (int)part.lnode.size();
    part.owned.assign(n, 0);
    for (int k = 0; k < n; k++) part.owned[k] = part.nodeOwner[part.lnode[k]] == me;

    // ---- ghosts received (sender ascending, link ascending) and links sent
    std::vector<G> in, out;
    for (const G& g : ghosts) {
        if (g.to == me) in.push_back(g);
        if (g.from == me) out.push_back(g);
    }
    auto bySender = [](const G& a, const G& b) { return a.from != b.from ? a.from < b.from : a.link < b.link; };
    auto byReceiver = [](const G& a, const G& b) { return a.to != b.to ? a.to < b.to : a.link < b.link; };
    std::sort(in.begin(), in.end(), bySender);
    std::sort(out.begin(), out.end(), byReceiver);
    part.lghost.clear();
    part.recvSlot.clear();
    for (const G& g : in) {
        part.lghost.push_back(g.link);
        part.recvSlot.push_back(slotOf[g.link]);
    }
    part.sendLink.clear();
    part.sendSlot.clear();
    for (const G& g : out) {
        part.sendLink.push_back(part.glink[g.link]);
        part.sendSlot.push_back(slotOf[g.link]);
    }
    part.nbr.clear();
    for (const G& g : in) part.nbr.push_back(g.from);
    for (const G& g : out) part.nbr.push_back(g.to);
    std::sort(part.nbr.begin(), part.nbr.end());
    part.nbr.erase(std::unique(part.nbr.begin(), part.nbr.end()), part.nbr.end());
    const int nb = (int)part.nbr.size();
    part.sendOff.assign(nb + 1, 0);
    part.recvOff.assign(nb + 1, 0);
    for (int k = 0; k < nb; k++) {
        const int r = part.nbr[k];
        part.sendOff[k + 1] = part.sendOff[k] + (int)std::count_if(out.begin(), out.end(),
                                                                   [r](const G& g) { return g.to == r; });
        part.recvOff[k + 1] = part.recvOff[k] + (int)std::count_if(in.begin(), in.end(),
                                                                   [r](const G& g) { return g.from == r; });
    }
    // held nodes touched by a ghost link: their sums include received values
    // (never reused across iterations, never frozen: see k_node)
    part.hasGhost.assign(n, 0);
    for (int g : part.lghost)
        for (int e : {net.node1[g], net.node2[g]})
            if (part.gnode[e] >= 0) part.hasGhost[part.gnode[e]] = 1;
    return 0;
}

void buildLocalCsr(const Network& net, const Partition& part, bool conduitsOnly, std::vector<int>& rowptr,
                   std::vector<int>& csr)
{
    const int n = (int)part.lnode.size();
    const int nOwned = (int)part.llink.size();
    const int nLoc = nOwned + (int)part.lghost.size();
    auto global = [&](int l) { return l < nOwned ? part.llink[l] : part.lghost[l - nOwned]; };
    rowptr.assign(n + 1, 0);
    for (int l = 0; l < nLoc; l++) {
        const int g = global(l);
        if (conduitsOnly && !net.isTrueConduit(g)) continue;
        for (int e : {net.node1[g], net.node2[g]})
            if (part.gnode[e] >= 0) rowptr[part.gnode[e] + 1]++;
    }
    for (int i = 0; i < n; i++) rowptr[i + 1] += rowptr[i];
    csr.assign(rowptr[n], 0);
    std::vector<int> fill(rowptr.begin(), rowptr.end() - 1);
    for (int l = 0; l < nLoc; l++) {
        const int g = global(l);
        if (conduitsOnly && !net.isTrueConduit(g)) continue;
        const int a = part.gnode[net.node1[g]], b = part.gnode[net.node2[g]];
        if (a >= 0) csr[fill[a]++] = l;
        if (b >= 0) csr[fill[b]++] = (int)((unsigned)l | 0x80000000u);
    }
    // ascending global link index within each row (owned links come first in
    // local order, so a row that mixes in ghosts needs sorting)
    for (int i = 0; i < n; i++) {
        auto key = [&](int ent) { return global(ent & 0x7FFFFFFF); };
        std::stable_sort(csr.begin() + rowptr[i], csr.begin() + rowptr[i + 1],
                         [&](int x, int y) { return key(x) < key(y); });
    }
}

}  // namespace swx
