// The one collective of a sharded server step: the all-reduce (sum, fp32) of each
// rank's partial [S_t | losses] over RCCL, for a caller that does not go through
// torch.distributed (include/flsim.h flsim_comm_*, flsim_allreduce_sum).  The reference has no
// collective at all: its workers run sequentially in one process (main.py:137), and their
// gradients meet in rule() (main.py:184); sharded, the partial sums meet here first.
//
// RCCL is bound at run time (dlopen), not linked: under torch the process already holds torch's
// own librccl.so.1 (torch/lib), and a second copy of the library in one process would keep its
// own state, so the copy already loaded is used when there is one (RTLD_NOLOAD), else
// $FLSIM_RCCL_LIB, else the system librccl.so.1 (/opt/rocm/lib).  A one-rank communicator made
// without a unique id never touches RCCL: its all-reduce is the identity (the world = 1 path).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

#include "common.h"
#include "flsim.h"

namespace flsim {
namespace {

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t,
                               ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    bool ok = false;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

template <class F>
bool bind(void* h, const char* name, F* out) {
    *out = reinterpret_cast<F>(dlsym(h, name));
    return *out != nullptr;
}

// the process's RCCL, bound on first use (nullptr + flsim_last_error when it cannot be found)
const Rccl* rccl() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl.ok) return &g_rccl;
    void* h = nullptr;
    for (const char* n : {"librccl.so.1", "librccl.so"})
        if (!h) h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    if (!h) {
        if (const char* e = getenv("FLSIM_RCCL_LIB")) h = dlopen(e, RTLD_NOW | RTLD_LOCAL);
    }
    for (const char* n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
        if (!h) h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        set_error("RCCL not found (librccl.so.1; set FLSIM_RCCL_LIB): %s", dlerror());
        return nullptr;
    }
    Rccl r;
    if (!bind(h, "ncclGetUniqueId", &r.get_unique_id) ||
        !bind(h, "ncclCommInitRank", &r.init_rank) || !bind(h, "ncclAllReduce", &r.all_reduce) ||
        !bind(h, "ncclCommDestroy", &r.destroy) || !bind(h, "ncclGetErrorString", &r.error_string)) {
        set_error("librccl.so lacks an NCCL entry point: %s", dlerror());
        return nullptr;
    }
    r.ok = true;
    g_rccl = r;
    return &g_rccl;
}

int nccl_check(const Rccl* r, ncclResult_t e, const char* what) {
    if (e == ncclSuccess) return 0;
    set_error("%s failed: %s", what, r->error_string ? r->error_string(e) : "?");
    return 2;
}

}  // namespace
}  // namespace flsim

struct flsim_comm {
    int nranks;
    int rank;
    ncclComm_t nccl;       // nullptr: the local one-rank communicator (no RCCL)
};

using namespace flsim;

extern "C" {

static_assert(sizeof(ncclUniqueId) == FLSIM_COMM_ID_BYTES, "ncclUniqueId size");

int flsim_comm_unique_id(unsigned char* id) {
    FLSIM_REQUIRE(id, "null pointer");
    const Rccl* r = rccl();
    if (!r) return 2;
    ncclUniqueId u;
    RC(nccl_check(r, r->get_unique_id(&u), "ncclGetUniqueId"));
    memcpy(id, &u, sizeof(u));
    return 0;
}

int flsim_comm_create(int nranks, int rank, const unsigned char* id, flsim_comm** out) {
    FLSIM_REQUIRE(out, "null pointer");
    *out = nullptr;
    FLSIM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "rank %d of %d", rank, nranks);
    FLSIM_REQUIRE(id || nranks == 1, "a communicator of %d ranks needs the unique id", nranks);
    ncclComm_t c = nullptr;
    if (id) {
        const Rccl* r = rccl();
        if (!r) return 2;
        ncclUniqueId u;
        memcpy(&u, id, sizeof(u));
        RC(nccl_check(r, r->init_rank(&c, nranks, u, rank), "ncclCommInitRank"));
    }
    *out = new flsim_comm{nranks, rank, c};
    return 0;
}

int flsim_comm_size(const flsim_comm* comm) { return comm ? comm->nranks : -1; }

int flsim_comm_rank(const flsim_comm* comm) { return comm ? comm->rank : -1; }

int flsim_allreduce_sum(flsim_comm* comm, float* buf, size_t count, flsim_stream_t stream) {
    FLSIM_REQUIRE(comm, "null communicator");
    if (count == 0) return 0;
    FLSIM_REQUIRE(buf, "null pointer");
    if (!comm->nccl) return 0;            // one rank, no RCCL: the sum of one partial is itself
    const Rccl* r = rccl();
    if (!r) return 2;
    return nccl_check(r, r->all_reduce(buf, buf, count, ncclFloat32, ncclSum, comm->nccl,
                                       reinterpret_cast<hipStream_t>(stream)),
                      "ncclAllReduce");
}

int flsim_comm_destroy(flsim_comm* comm) {
    if (!comm) return 0;
    int rc = 0;
    if (comm->nccl) {
        const Rccl* r = rccl();
        rc = r ? nccl_check(r, r->destroy(comm->nccl), "ncclCommDestroy") : 2;
    }
    delete comm;
    return rc;
}

}  // extern "C"
