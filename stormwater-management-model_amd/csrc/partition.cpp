// partition.cpp -- owner assignment and local index maps (see partition.h).
#include "partition.h"

#include <string>

namespace swx {

int buildPartition(const Network& net, Partition& part, std::string* msg)
{
    const int nN = net.nNodes(), nL = net.nLinks(), R = part.nranks;
    if (R < 1 || part.rank < 0 || part.rank >= R) {
        if (msg) *msg = "invalid rank / number of ranks";
        return 500;
    }
    // nodes: contiguous blocks of the node index
    part.nodeOwner.assign(nN, 0);
    for (int i = 0; i < nN; i++) part.nodeOwner[i] = (int)((long long)i * R / nN);
    // conduits: owner of node1; outfalls: owner of their conduit
    part.linkOwner.assign(nL, 0);
    for (int j = 0; j < nL; j++) part.linkOwner[j] = part.nodeOwner[net.node1[j]];
    for (int j = 0; j < nL; j++) {
        int n1 = net.node1[j], n2 = net.node2[j];
        if (net.nodeType[n2] == OUTFALL) part.nodeOwner[n2] = part.linkOwner[j];
        else if (net.nodeType[n1] == OUTFALL) part.nodeOwner[n1] = part.linkOwner[j];
    }
    // ranks touching each node: its owner and the owners of its conduits.
    // A node is shared when that set has more than one rank.
    std::vector<int> firstRank(nN), shared(nN, 0);
    for (int i = 0; i < nN; i++) firstRank[i] = part.nodeOwner[i];
    for (int j = 0; j < nL; j++) {
        int r = part.linkOwner[j];
        for (int n : {net.node1[j], net.node2[j]})
            if (r != firstRank[n]) shared[n] = 1;
    }
    // present on this rank: owned nodes and both ends of owned conduits
    std::vector<char> here(nN, 0);
    for (int i = 0; i < nN; i++)
        if (part.nodeOwner[i] == part.rank) here[i] = 1;
    for (int j = 0; j < nL; j++)
        if (part.linkOwner[j] == part.rank) here[net.node1[j]] = here[net.node2[j]] = 1;

    part.lnode.clear();
    part.gnode.assign(nN, -1);
    std::vector<int> slotOf(nN, -1);
    int slot = 0;
    for (int i = 0; i < nN; i++) {
        if (shared[i]) slotOf[i] = slot++;
        if (here[i]) {
            part.gnode[i] = (int)part.lnode.size();
            part.lnode.push_back(i);
        }
    }
    part.nSharedGlobal = slot;
    part.llink.clear();
    part.glink.assign(nL, -1);
    for (int j = 0; j < nL; j++)
        if (part.linkOwner[j] == part.rank) {
            part.glink[j] = (int)part.llink.size();
            part.llink.push_back(j);
        }
    const int n = (int)part.lnode.size();
    part.sharedSlot.assign(n, -1);
    part.owned.assign(n, 0);
    for (int k = 0; k < n; k++) {
        int g = part.lnode[k];
        part.sharedSlot[k] = slotOf[g];
        part.owned[k] = part.nodeOwner[g] == part.rank;
    }
    return 0;
}

}  // namespace swx
