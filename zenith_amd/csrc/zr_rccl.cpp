// zr_rccl.cpp — run-time binding of RCCL's point-to-point API (zr_rccl.h).
#include "zr_rccl.h"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace zr {
namespace {

struct UniqueId {
    char internal[kRcclIdBytes];
};
using Result = int;             // ncclResult_t (0 = ncclSuccess)
constexpr int kUint8 = 1;       // ncclUint8 (rccl.h ncclDataType_t)

struct Api {
    void* lib = nullptr;
    Result (*get_unique_id)(UniqueId*) = nullptr;
    Result (*comm_init_rank)(void**, int, UniqueId, int) = nullptr;
    Result (*comm_destroy)(void*) = nullptr;
    Result (*group_start)() = nullptr;
    Result (*group_end)() = nullptr;
    Result (*send)(const void*, size_t, int, int, void*, hipStream_t) = nullptr;
    Result (*recv)(void*, size_t, int, int, void*, hipStream_t) = nullptr;
    Result (*all_to_all)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;  // RCCL extension
    const char* (*error_string)(Result) = nullptr;
    std::string load_error;
};

Api g_api;
std::once_flag g_once;

template <typename F>
bool bind(void* lib, const char* name, F& fn) {
    fn = reinterpret_cast<F>(dlsym(lib, name));
    return fn != nullptr;
}

void load_once() {
    void* lib = nullptr;
    if (const char* p = getenv("ZR_RCCL_LIB")) lib = dlopen(p, RTLD_NOW | RTLD_LOCAL);
    // the instance the process already has (PyTorch's), then the ROCm install's
    for (const char* name : {"librccl.so", "librccl.so.1"})
        if (!lib) lib = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    for (const char* name : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so"})
        if (!lib) lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
    if (!lib) {
        g_api.load_error = std::string("RCCL not found: ") + dlerror();
        return;
    }
    Api a;
    a.lib = lib;
    const bool ok = bind(lib, "ncclGetUniqueId", a.get_unique_id) && bind(lib, "ncclCommInitRank", a.comm_init_rank) &&
                    bind(lib, "ncclCommDestroy", a.comm_destroy) && bind(lib, "ncclGroupStart", a.group_start) &&
                    bind(lib, "ncclGroupEnd", a.group_end) && bind(lib, "ncclSend", a.send) &&
                    bind(lib, "ncclRecv", a.recv) && bind(lib, "ncclGetErrorString", a.error_string);
    if (!ok) {
        g_api.load_error = "RCCL library lacks the point-to-point API";
        return;
    }
    if (!getenv("ZR_RCCL_NO_ALLTOALL")) bind(lib, "ncclAllToAll", a.all_to_all);  // optional
    g_api = a;
}

bool check(Result r, const char* what, std::string& err) {
    if (r == 0) return true;
    err = std::string(what) + ": " + (g_api.error_string ? g_api.error_string(r) : "RCCL error");
    return false;
}

}  // namespace

bool rccl_load(std::string& err) {
    std::call_once(g_once, load_once);
    if (!g_api.lib) err = g_api.load_error;
    return g_api.lib != nullptr;
}

bool rccl_unique_id(void* out, std::string& err) {
    if (!rccl_load(err)) return false;
    UniqueId id;
    if (!check(g_api.get_unique_id(&id), "ncclGetUniqueId", err)) return false;
    memcpy(out, id.internal, kRcclIdBytes);
    return true;
}

bool rccl_comm_init(void** comm, const void* unique_id, int nranks, int rank, std::string& err) {
    if (!rccl_load(err)) return false;
    UniqueId id;
    memcpy(id.internal, unique_id, kRcclIdBytes);
    return check(g_api.comm_init_rank(comm, nranks, id, rank), "ncclCommInitRank", err);
}

void rccl_comm_destroy(void* comm) {
    if (comm && g_api.comm_destroy) (void)g_api.comm_destroy(comm);
}

bool rccl_group_start(std::string& err) { return check(g_api.group_start(), "ncclGroupStart", err); }
bool rccl_group_end(std::string& err) { return check(g_api.group_end(), "ncclGroupEnd", err); }

bool rccl_send(const void* buf, size_t bytes, int peer, void* comm, hipStream_t s, std::string& err) {
    return check(g_api.send(buf, bytes, kUint8, peer, comm, s), "ncclSend", err);
}

bool rccl_recv(void* buf, size_t bytes, int peer, void* comm, hipStream_t s, std::string& err) {
    return check(g_api.recv(buf, bytes, kUint8, peer, comm, s), "ncclRecv", err);
}

bool rccl_grouped(const P2POp* ops, size_t n, void* comm, hipStream_t s, std::string& err) {
    if (!rccl_load(err) || !rccl_group_start(err)) return false;
    bool ok = true;
    for (size_t i = 0; ok && i < n; ++i)
        ok = ops[i].send ? rccl_send(ops[i].buf, ops[i].bytes, ops[i].peer, comm, s, err)
                         : rccl_recv(ops[i].buf, ops[i].bytes, ops[i].peer, comm, s, err);
    std::string end_err;
    const bool ended = rccl_group_end(end_err);
    if (ok && !ended) err = end_err;  // (a failed op's message is the one to report)
    return ok && ended;
}

bool rccl_has_all_to_all() { return g_api.all_to_all != nullptr; }

bool rccl_all_to_all(const void* send, void* recv, size_t bytes_per_rank, void* comm, hipStream_t s, std::string& err) {
    return check(g_api.all_to_all(send, recv, bytes_per_rank, kUint8, comm, s), "ncclAllToAll", err);
}

}  // namespace zr
