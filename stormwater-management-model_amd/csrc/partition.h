// partition.h -- link-partitioned multi-GPU layout.
//
// One process per GPU.  Nodes are split into contiguous blocks of the
// reference's node index (row strips for the row-major synthetic grids); a
// conduit belongs to the rank that owns its node1, an outfall to the rank that
// owns its (single) conduit.  A node is *shared* when the conduits touching it
// belong to more than one rank, or to a rank other than the node's owner.
// Every rank touching a shared node keeps a replica of it.  Each Picard
// iteration, every rank sums the contributions of its own conduits (plus, on
// the owner, the node's own inflow and ponded area) for its shared nodes and
// one all-reduce adds the partial sums; every replica then applies the same
// depth update to the same sums, so the replicas stay identical without a
// second exchange.  Interior nodes and all conduits are computed exactly as on
// one GPU (same arithmetic, same summation order); only a shared node's sums
// are reassociated (partial sums per rank).
#pragma once

#include <vector>

#include "model.h"

namespace swx {

// Host exchange used instead of RCCL by the test transport: in-place reduction
// of n doubles across the ranks (op 0 = sum, 1 = min).  Returns 0 on success.
typedef int (*ExchangeFn)(double* buf, long n, int op, void* user);

enum { XCHG_RCCL = 0, XCHG_HOST = 1 };

struct Partition {
    int rank = 0, nranks = 1;
    int transport = XCHG_RCCL;
    std::vector<unsigned char> ncclId;     // 128-byte ncclUniqueId (RCCL transport)
    ExchangeFn xchg = nullptr;
    void* xuser = nullptr;

    // ---- derived by buildPartition (identical on every rank) -------------
    std::vector<int> nodeOwner, linkOwner;  // global object -> rank
    std::vector<int> lnode, llink;          // local -> global, ascending global index
    std::vector<int> gnode, glink;          // global -> local, -1 when not present here
    std::vector<int> sharedSlot;            // per local node: global shared slot or -1
    std::vector<char> owned;                // per local node: this rank owns it
    int nSharedGlobal = 0;

    bool forced = false;                    // partitioned code path with one rank (tests)
    bool active() const { return nranks > 1 || forced; }
};

// Fills the derived fields of `part` for `net`.  Returns 0, or an error code
// (and message) when the network cannot be partitioned.
int buildPartition(const Network& net, Partition& part, std::string* msg);

}  // namespace swx
