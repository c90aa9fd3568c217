// zr_rccl.h — the runtime's RCCL binding (host only).
//
// RCCL is resolved at run time: the copy the process already loaded (PyTorch
// ships one) is preferred, so the runtime's communicators and the caller's use
// one library instance; otherwise librccl.so from the ROCm install.  Only the
// point-to-point subset is used (grouped ncclSend / ncclRecv on a HIP stream).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>

namespace zr {

constexpr size_t kRcclIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES

// Loads the library once; false + message when it is unavailable.
bool rccl_load(std::string& err);
bool rccl_unique_id(void* out, std::string& err);
// Creates a communicator of `nranks` with this process as `rank` (blocking until
// every rank joined).  *comm is an opaque ncclComm_t.
bool rccl_comm_init(void** comm, const void* unique_id, int nranks, int rank, std::string& err);
void rccl_comm_destroy(void* comm);
bool rccl_group_start(std::string& err);
bool rccl_group_end(std::string& err);
bool rccl_send(const void* buf, size_t bytes, int peer, void* comm, hipStream_t s, std::string& err);
bool rccl_recv(void* buf, size_t bytes, int peer, void* comm, hipStream_t s, std::string& err);
// One grouped batch of point-to-point calls: ncclGroupStart, every op (a send of
// `buf` when `send`, else a receive into it) until the first failure, then
// ncclGroupEnd -- only when the start succeeded, and always then, whatever the
// sends returned (an unbalanced start or end is an RCCL error of its own and
// would hide the first one's message).  Both collectives go through it
// (zr_runtime.cpp); tests/test_rccl_group.py drives it against a fake RCCL.
struct P2POp {
    void* buf;
    size_t bytes;
    int peer;
    bool send;
};
bool rccl_grouped(const P2POp* ops, size_t n, void* comm, hipStream_t s, std::string& err);
// RCCL's ncclAllToAll extension (one call instead of a group of 2 * nranks
// point-to-point calls); absent from plain NCCL-API builds.
bool rccl_has_all_to_all();
bool rccl_all_to_all(const void* send, void* recv, size_t bytes_per_rank, void* comm, hipStream_t s, std::string& err);

}  // namespace zr
