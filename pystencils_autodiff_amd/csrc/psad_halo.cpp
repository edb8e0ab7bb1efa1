// RCCL halo exchange of the z-slab decomposition, part of libpsad_hip.so.
//
// The reference has no multi-GPU path; its pystencils GPU kernels run on one device. Here each rank
// owns a z-slab of every field and, once per sweep, swaps its RZ boundary planes with ranks k-1 / k+1:
// one ncclGroupStart / ncclSend+ncclRecv per neighbour and field / ncclGroupEnd on the caller's
// stream, nothing else — no torch.distributed work objects, watchdog events or Python per call
// (torch's batch_isend_irecv costs ~80 us of host time per exchange, scripts/probes/p2p_host_cost.py).
//
// librccl is opened at run time (dlopen of the path the caller names — torch's own copy, so one RCCL
// instance serves both torch's process group and this communicator); no RCCL headers are needed: the
// few entry points used have the stable NCCL 2.x C signatures declared below.
#include "psad.h"

#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <cstring>

namespace {

struct UniqueId { char internal[128]; };   // ncclUniqueId
typedef void* Comm;                          // ncclComm_t
typedef int Result;                          // ncclResult_t, 0 = ncclSuccess
constexpr int kInt8 = 0;                     // ncclInt8

struct Rccl {
    void* handle = nullptr;
    Result (*get_unique_id)(UniqueId*) = nullptr;
    Result (*comm_init_rank)(Comm*, int, UniqueId, int) = nullptr;
    Result (*comm_destroy)(Comm) = nullptr;
    Result (*group_start)() = nullptr;
    Result (*group_end)() = nullptr;
    Result (*send)(const void*, size_t, int, int, Comm, hipStream_t) = nullptr;
    Result (*recv)(void*, size_t, int, int, Comm, hipStream_t) = nullptr;
    const char* (*error_string)(Result) = nullptr;
} g_rccl;

constexpr int kNotLoaded = 100;   // PSAD_RCCL_ERROR_BASE + kNotLoaded: library / symbol missing

int rc(Result r) { return r == 0 ? 0 : PSAD_RCCL_ERROR_BASE + r; }

template <typename F>
bool sym(F& f, const char* name) {
    f = reinterpret_cast<F>(dlsym(g_rccl.handle, name));
    return f != nullptr;
}

}  // namespace

extern "C" {

int psad_rccl_open(const char* library_path) {
    if (g_rccl.handle != nullptr) return 0;
    void* h = dlopen(library_path, RTLD_NOW | RTLD_LOCAL);
    if (h == nullptr) return PSAD_RCCL_ERROR_BASE + kNotLoaded;
    g_rccl.handle = h;
    bool ok = sym(g_rccl.get_unique_id, "ncclGetUniqueId") && sym(g_rccl.comm_init_rank, "ncclCommInitRank") &&
              sym(g_rccl.comm_destroy, "ncclCommDestroy") && sym(g_rccl.group_start, "ncclGroupStart") &&
              sym(g_rccl.group_end, "ncclGroupEnd") && sym(g_rccl.send, "ncclSend") &&
              sym(g_rccl.recv, "ncclRecv") && sym(g_rccl.error_string, "ncclGetErrorString");
    if (!ok) {
        dlclose(h);
        g_rccl = Rccl{};
        return PSAD_RCCL_ERROR_BASE + kNotLoaded;
    }
    return 0;
}

int psad_rccl_unique_id(void* id) {
    if (g_rccl.handle == nullptr) return PSAD_RCCL_ERROR_BASE + kNotLoaded;
    UniqueId u;
    int e = rc(g_rccl.get_unique_id(&u));
    if (e == 0) std::memcpy(id, u.internal, sizeof(u.internal));
    return e;
}

int psad_rccl_comm_init(const void* id, int nranks, int rank, void** comm) {
    if (g_rccl.handle == nullptr) return PSAD_RCCL_ERROR_BASE + kNotLoaded;
    UniqueId u;
    std::memcpy(u.internal, id, sizeof(u.internal));
    Comm c = nullptr;
    int e = rc(g_rccl.comm_init_rank(&c, nranks, u, rank));
    *comm = e == 0 ? c : nullptr;
    return e;
}

int psad_rccl_comm_destroy(void* comm) {
    if (g_rccl.handle == nullptr) return PSAD_RCCL_ERROR_BASE + kNotLoaded;
    return comm == nullptr ? 0 : rc(g_rccl.comm_destroy(static_cast<Comm>(comm)));
}

int psad_halo_exchange(void* comm, int n_fields, const void* const* send_lo, void* const* recv_lo,
                       const void* const* send_hi, void* const* recv_hi, const size_t* bytes, int peer_lo,
                       int peer_hi, void* stream) {
    if (g_rccl.handle == nullptr) return PSAD_RCCL_ERROR_BASE + kNotLoaded;
    Comm c = static_cast<Comm>(comm);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int e = rc(g_rccl.group_start());
    if (e != 0) return e;
    for (int i = 0; i < n_fields && e == 0; ++i) {
        if (peer_lo >= 0) {
            e = rc(g_rccl.send(send_lo[i], bytes[i], kInt8, peer_lo, c, s));
            if (e == 0) e = rc(g_rccl.recv(recv_lo[i], bytes[i], kInt8, peer_lo, c, s));
        }
        if (e == 0 && peer_hi >= 0) {
            e = rc(g_rccl.send(send_hi[i], bytes[i], kInt8, peer_hi, c, s));
            if (e == 0) e = rc(g_rccl.recv(recv_hi[i], bytes[i], kInt8, peer_hi, c, s));
        }
    }
    int e2 = rc(g_rccl.group_end());   // always close the group
    return e != 0 ? e : e2;
}

const char* psad_rccl_error_string(int code) {
    if (code == PSAD_RCCL_ERROR_BASE + kNotLoaded) return "RCCL library not loaded (psad_rccl_open) or symbol missing";
    if (g_rccl.error_string == nullptr) return "RCCL error (library not loaded)";
    return g_rccl.error_string(static_cast<Result>(code - PSAD_RCCL_ERROR_BASE));
}

}  // extern "C"
