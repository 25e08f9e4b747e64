// partition.h -- link-partitioned multi-GPU layout.
//
// One process per GPU.  Nodes are split into contiguous blocks of the
// reference's node index (row strips for the row-major synthetic grids); a
// conduit belongs to the rank that owns its node1, an outfall to the rank that
// owns its (single) conduit.  Pumps and regulators (routed by k_nc, whose node
// sums need the running totals of their end nodes) keep their end nodes and
// every link touching those nodes on one rank.
//
// A rank holds its *owned* links and every node they touch (owned nodes plus
// replicas of nodes owned elsewhere).  For every held node it also needs the
// contributions of the links of other ranks that touch the node: those are
// its *ghost* links.  Each Picard iteration the owner of a ghost link sends
// its {flow, surface areas, dq/dh (, evaporation, seepage)} to the ranks that
// hold it as a ghost (strip neighbours for the grids), and every held node is
// then summed over all its links in global link order -- the reference's
// serial scatter order (dynwave.c:398-411, 528-589).  Every replica of a node
// therefore computes exactly the single-GPU update: the partitioned run is
// bitwise equal to one GPU.  A small all-reduce (max) of the per-iteration
// "some node did not converge" flag keeps the ranks' Picard loops in step.
#pragma once

#include <string>
#include <vector>

#include "model.h"

namespace swx {

// Host exchange used instead of RCCL by the test transport: in-place reduction
// of n doubles across the ranks (op 0 = sum, 1 = min).  Returns 0 on success.
typedef int (*ExchangeFn)(double* buf, long n, int op, void* user);

// Transports of the per-iteration exchange: RCCL (ncclSend / ncclRecv and
// ncclAllReduce captured in the step graph), HOST (the callback below; tests:
// several ranks on one GPU), IPC (device-initiated stores into the peers'
// memory, mapped with hipIpcOpenMemHandle; no collective library inside a
// step; bootstrapped over the host callback when one is set, else over RCCL).
enum { XCHG_RCCL = 0, XCHG_HOST = 1, XCHG_IPC = 2 };
enum { PART_CONTIGUOUS = 0, PART_TWO_REGION = 1 };

struct Partition {
    int rank = 0, nranks = 1;
    int transport = XCHG_RCCL;
    std::vector<unsigned char> ncclId;     // 128-byte ncclUniqueId (RCCL transport / bootstrap)
    ExchangeFn xchg = nullptr;             // host callback (HOST transport; IPC bootstrap)
    void* xuser = nullptr;
    // optional per-node work weights (global node order; empty: every node
    // weighs 1): the contiguous node blocks then carry equal weight instead
    // of equal node counts (swmmx_setPartitionWeights; e.g. 1 + the node's
    // measured sparse-iteration updates times their relative cost)
    std::vector<double> weight;
    // PART_CONTIGUOUS: one contiguous block of equal weight per rank;
    // PART_TWO_REGION (needs weights): the "hot" nodes -- weight excess over
    // the lightest node at least a quarter of the largest excess (the surcharged band
    // whose nodes run every sparse iteration) -- are cut into 2 nranks
    // contiguous blocks of equal weight dealt 0, 1, .., R-1, R-1, .., 0 (a
    // trend across the band cancels between a rank's two blocks), the other
    // nodes into nranks blocks, rank r taking block r: every rank gets an
    // equal share of the sparse work and of the full passes, at the price of
    // a few more cut rows
    int mode = 0;

    // ---- derived by buildPartition (identical on every rank) -------------
    std::vector<int> nodeOwner, linkOwner;  // global object -> rank
    std::vector<int> lnode, llink;          // local -> global, ascending global index (llink: owned)
    std::vector<int> gnode, glink;          // global -> local, -1 when not held (glink: owned only)
    std::vector<char> owned;                // per local node: this rank owns it
    std::vector<char> hasGhost;             // per local node: a ghost link touches it
    // ghost links: local link index nOwned + g holds global link lghost[g];
    // grouped by the sending rank (ascending), ascending global index within
    std::vector<int> lghost;
    // neighbour exchange: nbr[k] = k-th rank this one exchanges with
    // (ascending); the links sent to it are sendLink[sendOff[k] .. sendOff[k+1])
    // (local owned indices, in the receiver's ghost order); the ghosts received
    // from it are lghost[recvOff[k] .. recvOff[k+1])
    std::vector<int> nbr, sendOff, sendLink, recvOff;
    // host transport: one global slot per link that is a ghost anywhere
    // (ascending global index); sendSlot / recvSlot per send / ghost entry
    std::vector<int> sendSlot, recvSlot;
    int nSlotGlobal = 0;

    bool forced = false;                    // partitioned code path with one rank (tests)
    bool active() const { return nranks > 1 || forced; }
    int nOwnedLinks() const { return (int)llink.size(); }
};

// Fills the derived fields of `part` for `net`.  Returns 0, or an error code
// (and message) when the network cannot be partitioned.
int buildPartition(const Network& net, Partition& part, std::string* msg);

// Node -> link incidence of this rank's held nodes over its owned and ghost
// links, each row in ascending GLOBAL link index (the reference's summation
// order).  Entries are local link indices (ghosts: nOwned + g) with bit 31 set
// when the node is the link's node2.  conduitsOnly drops pumps and regulators
// from the rows (their flows join the node sums after all conduits, in k_nc).
void buildLocalCsr(const Network& net, const Partition& part, bool conduitsOnly,
                   std::vector<int>& rowptr, std::vector<int>& csr);

}  // namespace swx
