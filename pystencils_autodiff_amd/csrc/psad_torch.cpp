// psad_torch.cpp — native autograd node for the torch_native op (_psad_torch extension module).
//
// The reference's op is a Python torch.autograd.Function (backends/_torch_native.py:10-142) whose backward
// torch's autograd engine runs on its per-device thread: the Python backward needs the GIL on that thread,
// and for a small field the engine's thread hand-off plus the Python body is longer than the kernels
// (2-D 4096² 5-point: 44 µs of kernels, 115-166 µs per apply+backward step,
// scripts/probes/autograd_handoff.py). Here the same forward/backward launches are a C++
// torch::autograd::Function: the forward allocates, patches the tensor pointers into a launch-argument
// template and launches through the C ABI (psad_launch, include/psad.h) on the current stream; the
// backward does the same for the adjoint kernel on the engine's thread without touching Python.
//
// A plan (both launches, resolved once by the Python op for one input signature — shapes, dtypes, device —
// by HipStencilKernel.prepare) holds: the function handle, grid and block, the packed argument template
// whose first n_ptr 8-byte slots are the field pointers (hip_kernel._Plan.pack), for each slot the index of
// the tensor in the call's table, and the byte offsets of the scalar parameters, patched per call from the
// op's class_kwargs (a coefficient that changes every step reuses the plan). Forward table: inputs ++ outputs; backward table:
// saved forward tensors ++ output gradients ++ adjoint outputs. apply() returns None when a call does not
// match its plan (device, dtype, shape, contiguity, 32-byte alignment): the Python op then takes the
// general path.
#include <torch/extension.h>

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "psad.h"

namespace {

struct Launch {
    void* fn = nullptr;
    unsigned grid = 0, block = 0;
    std::string args;          // packed template; pointer i at byte 8*i
    std::vector<int64_t> slot; // pointer i <- table[slot[i]]
    std::vector<int64_t> s_off, s_f64, s_idx;   // scalar j at byte s_off[j] (f64 or f32) <- scalars[s_idx[j]]
    int64_t sig_ptr_off = -1, sig_val_off = -1; // start signal (hip_emitter SIG): word pointer and value, or -1
    int64_t hw_ptr_off = -1, hw_val_off = -1;   // halo wait (hip_emitter HWAIT): word pointer and value, or -1
};

struct Alloc {
    std::vector<int64_t> shape;
    at::ScalarType dtype;
    bool zero;                 // torch.zeros (outputs the kernel reads or writes only in part)
};

struct Plan {
    int device = 0;
    // forward
    std::vector<std::vector<int64_t>> in_shape;
    std::vector<at::ScalarType> in_dtype;
    std::vector<Alloc> fwd_out;
    Launch fwd;
    std::vector<int64_t> saved;      // forward-table indices kept for the backward
    // backward
    std::vector<Alloc> bwd_out;
    Launch bwd;
    std::vector<int64_t> grad_of_input;   // per forward input: backward-table index or -1
    int64_t n_scalars = 0;
    std::string name;
};

std::mutex g_mutex;
std::vector<std::unique_ptr<Plan>> g_plans;   // plans live as long as the process (graphs may outlive ops)
std::atomic<bool> g_poison{false};             // tests: fill uninitialised outputs with NaN

const Plan& plan_at(int64_t id) {
    std::lock_guard<std::mutex> lock(g_mutex);
    TORCH_CHECK(id >= 0 && id < static_cast<int64_t>(g_plans.size()), "psad: unknown plan ", id);
    return *g_plans[id];
}

at::Tensor allocate(const Alloc& a, int device) {
    auto opt = at::TensorOptions().dtype(a.dtype).device(at::kCUDA, device);
    if (a.zero) return at::zeros(a.shape, opt);
    at::Tensor t = at::empty(a.shape, opt);
    if (g_poison.load(std::memory_order_relaxed)) t.fill_(std::numeric_limits<double>::quiet_NaN());
    return t;
}

bool aligned(const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 31u) == 0; }

void launch_on(const Launch& l, const std::vector<at::Tensor>& table, const std::vector<double>& scalars,
               hipStream_t stream, uint32_t* sig = nullptr, uint32_t sig_value = 0, const uint32_t* hw = nullptr,
               uint32_t hw_value = 0);

void launch(const Launch& l, const std::vector<at::Tensor>& table, const std::vector<double>& scalars,
            int device) {
    // the function handle belongs to the module loaded on the plan's device: launch with it current
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
    launch_on(l, table, scalars, c10::hip::getCurrentHIPStream(device).stream());
}

void launch_on(const Launch& l, const std::vector<at::Tensor>& table, const std::vector<double>& scalars,
               hipStream_t stream, uint32_t* sig, uint32_t sig_value, const uint32_t* hw, uint32_t hw_value) {
    std::string args = l.args;
    if (sig != nullptr) {       // the launch stores sig_value to *sig when it starts (its template holds nullptr)
        TORCH_CHECK(l.sig_ptr_off >= 0 && l.sig_val_off >= 0, "psad: launch without a start-signal slot");
        std::memcpy(&args[l.sig_ptr_off], &sig, sizeof(sig));
        std::memcpy(&args[l.sig_val_off], &sig_value, sizeof(sig_value));
    }
    if (hw != nullptr) {        // the launch's loader waits for *hw >= hw_value (its template holds nullptr)
        TORCH_CHECK(l.hw_ptr_off >= 0 && l.hw_val_off >= 0, "psad: launch without a halo-wait slot");
        std::memcpy(&args[l.hw_ptr_off], &hw, sizeof(hw));
        std::memcpy(&args[l.hw_val_off], &hw_value, sizeof(hw_value));
    }
    for (size_t i = 0; i < l.slot.size(); ++i) {
        void* p = table[l.slot[i]].data_ptr();
        std::memcpy(&args[8 * i], &p, sizeof(p));
    }
    for (size_t j = 0; j < l.s_off.size(); ++j) {
        const double v = scalars[l.s_idx[j]];
        if (l.s_f64[j]) {
            std::memcpy(&args[l.s_off[j]], &v, sizeof(v));
        } else {
            const float f = static_cast<float>(v);
            std::memcpy(&args[l.s_off[j]], &f, sizeof(f));
        }
    }
    int rc = psad_launch(l.fn, l.grid, 1, 1, l.block, 1, 1, 0, stream, args.data(), args.size());
    TORCH_CHECK(rc == 0, "psad: hipModuleLaunchKernel failed: ", psad_error_string(rc), " (code ", rc, ")");
}

struct StencilFunction : public torch::autograd::Function<StencilFunction> {
    static torch::autograd::variable_list forward(torch::autograd::AutogradContext* ctx, int64_t id,
                                                  at::TensorList inputs, std::vector<double> scalars) {
        const Plan& p = plan_at(id);
        std::vector<at::Tensor> table(inputs.begin(), inputs.end());
        std::vector<at::Tensor> outs;
        for (const auto& a : p.fwd_out) {
            outs.push_back(allocate(a, p.device));
            table.push_back(outs.back());
        }
        launch(p.fwd, table, scalars, p.device);
        std::vector<at::Tensor> saved;
        for (auto i : p.saved) saved.push_back(table[i]);
        ctx->save_for_backward(saved);
        ctx->saved_data["plan"] = id;
        ctx->saved_data["scalars"] = scalars;          // the forward's values, as the Python op's ctx.scalars
        return outs;
    }

    static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx,
                                                   torch::autograd::variable_list grads) {
        const Plan& p = plan_at(ctx->saved_data["plan"].toInt());
        std::vector<at::Tensor> table = ctx->get_saved_variables();
        for (auto& g : grads) {
            // undefined gradients arrive as zeros (materialize_grads); the adjoint kernel reads dense,
            // 32-byte-aligned fields like the ones its plan was made for
            at::Tensor t = g.is_contiguous() ? g : g.contiguous();
            if (!aligned(t)) t = t.clone();
            table.push_back(t);
        }
        std::vector<at::Tensor> outs;
        for (const auto& a : p.bwd_out) {
            outs.push_back(allocate(a, p.device));
            table.push_back(outs.back());
        }
        launch(p.bwd, table, ctx->saved_data["scalars"].toDoubleVector(), p.device);
        // one slot per forward argument, in order: plan id, each input of the list, the scalars
        torch::autograd::variable_list result(2 + p.grad_of_input.size());
        for (size_t i = 0; i < p.grad_of_input.size(); ++i)
            if (p.grad_of_input[i] >= 0) result[1 + i] = table[p.grad_of_input[i]];
        return result;
    }
};

// ---- z-slab sweeps (zslab.py): the RCCL face exchange and the interior / face launches of one rank ----------
//
// ZSlabOp's sweep in Python issues, per sweep: an event on the compute stream and a wait for it on the halo
// stream, one RCCL group (psad_halo_exchange) on the halo stream, the interior launch on the compute stream, an
// event on the halo stream and a wait for it on the compute stream, then the face launch(es). For small slabs
// (the 8-GPU 96×768² fp16 27-point slab computes a sweep in ~50 µs) the Python argument preparation around
// those calls was what the GPU waited on. A slab plan resolves all of it once per input signature: the
// launches' argument templates (field pointers patched per call, the receive buffers' halo pointers baked in),
// the exchange's receive buffers, byte counts and peers; a sweep is then these HIP / RCCL calls and nothing else.
// The send side needs no record_stream: the compute stream waits for the halo stream before the face launch,
// so any later reuse of an input's memory is ordered after the exchange has read it.

struct Exchange {
    void* comm = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev_faces = nullptr, ev_halos = nullptr;
    std::vector<int64_t> slot;            // table index of each exchanged field
    std::vector<int64_t> last_off;        // byte offset of its last RZ planes
    std::vector<void*> recv_lo, recv_hi;  // receive buffers (nullptr: no neighbour on that side)
    std::vector<size_t> bytes;
    int peer_lo = -1, peer_hi = -1;
    bool loopback = false;                // one-rank communicator: both faces to itself (periodic z)
    // the two cross-stream orderings as stream memory operations (hipStreamWriteValue32 / hipStreamWaitValue32 on a
    // signal-memory word with a sweep counter; PSAD_SLAB_SYNC=event: event record + wait instead)
    // one HSA signal per ordering (signal memory is allocated 8 bytes at a time)
    uint32_t* sig = nullptr;              // faces final (compute -> halo stream)
    uint32_t* sig_halo = nullptr;         // halos landed (halo -> compute)
    // under g_sweep_mutex: the sweep counter, and the one compute stream whose sweeps order through the signals. A
    // wait for "sig >= seq" is a point in THAT stream only while every write to sig comes from it, in counter order;
    // a sweep enqueued on another compute stream (torch.cuda.stream(s2), a second Python thread) would let the halo
    // stream pass early, so such sweeps take the event record + wait path instead
    mutable uint32_t seq = 0;
    mutable hipStream_t sig_stream = nullptr;   // (torch's default stream IS nullptr: sig_bound says whether it is set)
    mutable bool sig_bound = false;
    // compute -> halo by event record + wait (a marker packet on the compute queue) and halo -> compute by the
    // stream memory operation (PSAD_SLAB_SYNC=mixed): the compute queue then carries one ROCclr stream-op kernel per
    // sweep instead of two
    bool faces_by_event = false;
    // the interior launch writes the compute -> halo signal itself (default; PSAD_SLAB_START_SIG=0: a
    // hipStreamWriteValue32 on the compute stream)
    bool start_sig = true;
    // the face launches on the compute stream, waiting in their loaders (PSAD_SLAB_FACE_WAIT=1; default: see sweep_from)
    bool faces_wait = false;
};

std::mutex g_sweep_mutex;               // serialises the enqueue of exchanging sweeps (counter order = stream order)
std::atomic<int64_t> g_event_sweeps{0};  // exchanging sweeps ordered by events (tests)
std::atomic<int64_t> g_start_sig_sweeps{0};   // exchanging sweeps whose interior launch wrote the signal (tests)
std::atomic<int64_t> g_face_wait_sweeps{0};   // ... whose face launches waited in-kernel on the compute stream (tests)

struct Sweep {
    Exchange ex;
    bool has_inner = false;
    Launch inner;
    std::vector<Launch> faces;
    bool faces_on_halo = false;           // face launch(es) on the halo stream right behind the exchange
};

struct SlabPlan {
    int device = 0;
    std::vector<std::vector<int64_t>> in_shape;
    std::vector<at::ScalarType> in_dtype;
    std::vector<Alloc> fwd_out, bwd_out;
    Sweep fwd, bwd;
    std::vector<int64_t> saved, grad_of_input;
    int64_t n_scalars = 0;
    std::string name;
};

std::vector<std::unique_ptr<SlabPlan>> g_slab_plans;

const SlabPlan& slab_plan_at(int64_t id) {
    std::lock_guard<std::mutex> lock(g_mutex);
    TORCH_CHECK(id >= 0 && id < static_cast<int64_t>(g_slab_plans.size()), "psad: unknown slab plan ", id);
    return *g_slab_plans[id];
}

void hip_ok(hipError_t e, const char* what) {
    TORCH_CHECK(e == hipSuccess, "psad: ", what, " failed: ", hipGetErrorString(e));
}

void run_sweep(const Sweep& w, const std::vector<at::Tensor>& table, const std::vector<double>& scalars, int device) {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
    hipStream_t cur = c10::hip::getCurrentHIPStream(device).stream();
    const Exchange& ex = w.ex;
    const size_t n = ex.slot.size();
    std::unique_lock<std::mutex> lock(g_sweep_mutex, std::defer_lock);
    if (n) lock.lock();
    const bool sig = n && ex.sig && (!ex.sig_bound || ex.sig_stream == cur);
    uint32_t seq = 0;
    if (sig) {
        ex.sig_stream = cur;
        ex.sig_bound = true;
        seq = ++ex.seq;
    }
    // the interior launch stores seq to the signal word when it starts (every earlier launch of the compute stream
    // has completed then): the compute queue carries no stream-memory write kernel for this ordering
    const bool start_sig = sig && !ex.faces_by_event && w.has_inner && w.inner.sig_ptr_off >= 0 && ex.start_sig;
    // ... and the face launches behind the interior on the compute stream, their loaders waiting for the halo stream's
    // word: no stream-memory operation on the compute queue at all (the receive buffers are not reused before the next
    // exchange, which waits for the next interior's start — after these faces in stream order)
    bool faces_wait = start_sig && w.faces_on_halo && ex.faces_wait && !w.faces.empty();
    for (const auto& f : w.faces) faces_wait = faces_wait && f.hw_ptr_off >= 0;
    if (start_sig) {
        // the interior launch (which stores seq when it starts) is ENQUEUED before the halo stream's wait for it: streams
        // may share a hardware queue (GPU_MAX_HW_QUEUES), and a wait packet ahead of the launch that satisfies it in
        // one queue would never complete
        g_start_sig_sweeps.fetch_add(1);
        launch_on(w.inner, table, scalars, cur, ex.sig, seq);
        hip_ok(hipStreamWaitValue32(ex.stream, ex.sig, seq, hipStreamWaitValueGte, 0xffffffffu),
               "hipStreamWaitValue32");
    } else if (sig && !ex.faces_by_event) {
        hip_ok(hipStreamWriteValue32(cur, ex.sig, seq, 0), "hipStreamWriteValue32");
        hip_ok(hipStreamWaitValue32(ex.stream, ex.sig, seq, hipStreamWaitValueGte, 0xffffffffu),
               "hipStreamWaitValue32");
    } else if (sig) {
        hip_ok(hipEventRecord(ex.ev_faces, cur), "hipEventRecord");           // the faces are final
        hip_ok(hipStreamWaitEvent(ex.stream, ex.ev_faces, 0), "hipStreamWaitEvent");
    } else if (n) {
        g_event_sweeps.fetch_add(1);
        hip_ok(hipEventRecord(ex.ev_faces, cur), "hipEventRecord");           // the faces are final
        hip_ok(hipStreamWaitEvent(ex.stream, ex.ev_faces, 0), "hipStreamWaitEvent");
    }
    if (n) {
        std::vector<const void*> send_lo(n), send_hi(n);
        for (size_t i = 0; i < n; ++i) {
            char* base = static_cast<char*>(table[ex.slot[i]].data_ptr());
            send_lo[i] = base;
            send_hi[i] = base + ex.last_off[i];
            // RCCL pairs a peer's sends and receives in issue order: on a loopback communicator the lower halo
            // receives the far (upper) face, as with real neighbours — a periodic z boundary
            if (ex.loopback) std::swap(send_lo[i], send_hi[i]);
        }
        int rc = psad_halo_exchange(ex.comm, static_cast<int>(n), send_lo.data(), ex.recv_lo.data(), send_hi.data(),
                                    ex.recv_hi.data(), ex.bytes.data(), ex.peer_lo, ex.peer_hi, ex.stream);
        TORCH_CHECK(rc == 0, "psad: RCCL halo exchange failed: ", psad_rccl_error_string(rc), " (code ", rc, ")");
    }
    if (n && w.faces_on_halo && !faces_wait)                                 // faces beside the interior
        for (const auto& f : w.faces) launch_on(f, table, scalars, ex.stream);
    if (w.has_inner && !start_sig) launch(w.inner, table, scalars, device);   // interior overlaps the exchange
    if (faces_wait) {
        // (the halo stream's write is enqueued before the face launches that wait for it: see start_sig)
        g_face_wait_sweeps.fetch_add(1);
        hip_ok(hipStreamWriteValue32(ex.stream, ex.sig_halo, seq, 0), "hipStreamWriteValue32");
        for (const auto& f : w.faces) launch_on(f, table, scalars, cur, nullptr, 0, ex.sig_halo, seq);
        return;
    }
    if (sig) {
        hip_ok(hipStreamWriteValue32(ex.stream, ex.sig_halo, seq, 0), "hipStreamWriteValue32");
        hip_ok(hipStreamWaitValue32(cur, ex.sig_halo, seq, hipStreamWaitValueGte, 0xffffffffu),
               "hipStreamWaitValue32");
    } else if (n) {
        hip_ok(hipEventRecord(ex.ev_halos, ex.stream), "hipEventRecord");
        hip_ok(hipStreamWaitEvent(cur, ex.ev_halos, 0), "hipStreamWaitEvent");
    }
    if (!(n && w.faces_on_halo))
        for (const auto& f : w.faces) launch(f, table, scalars, device);
}

struct SlabFunction : public torch::autograd::Function<SlabFunction> {
    static torch::autograd::variable_list forward(torch::autograd::AutogradContext* ctx, int64_t id,
                                                  at::TensorList inputs, std::vector<double> scalars) {
        const SlabPlan& p = slab_plan_at(id);
        std::vector<at::Tensor> table(inputs.begin(), inputs.end());
        std::vector<at::Tensor> outs;
        for (const auto& a : p.fwd_out) {
            outs.push_back(allocate(a, p.device));
            table.push_back(outs.back());
        }
        run_sweep(p.fwd, table, scalars, p.device);
        std::vector<at::Tensor> saved;
        for (auto i : p.saved) saved.push_back(table[i]);
        ctx->save_for_backward(saved);
        ctx->saved_data["plan"] = id;
        ctx->saved_data["scalars"] = scalars;
        return outs;
    }

    static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx,
                                                   torch::autograd::variable_list grads) {
        const SlabPlan& p = slab_plan_at(ctx->saved_data["plan"].toInt());
        std::vector<at::Tensor> table = ctx->get_saved_variables();
        for (auto& g : grads) {
            at::Tensor t = g.is_contiguous() ? g : g.contiguous();
            if (!aligned(t)) t = t.clone();
            table.push_back(t);
        }
        std::vector<at::Tensor> outs;
        for (const auto& a : p.bwd_out) {
            outs.push_back(allocate(a, p.device));
            table.push_back(outs.back());
        }
        run_sweep(p.bwd, table, ctx->saved_data["scalars"].toDoubleVector(), p.device);
        torch::autograd::variable_list result(2 + p.grad_of_input.size());   // plan id, inputs..., scalars
        for (size_t i = 0; i < p.grad_of_input.size(); ++i)
            if (p.grad_of_input[i] >= 0) result[1 + i] = table[p.grad_of_input[i]];
        return result;
    }
};

Launch make_launch(uint64_t fn, int64_t grid, int64_t block, const py::bytes& args, std::vector<int64_t> slot,
                   std::vector<std::vector<int64_t>> scal, int64_t n_scalars) {
    Launch l;
    l.fn = reinterpret_cast<void*>(fn);
    l.grid = static_cast<unsigned>(grid);
    l.block = static_cast<unsigned>(block);
    l.args = std::string(args);
    TORCH_CHECK(l.args.size() >= 8 * slot.size(), "psad: argument template shorter than its pointer slots");
    l.slot = std::move(slot);
    for (const auto& sc : scal) {       // (byte offset, is f64, index into the call's scalars)
        TORCH_CHECK(sc.size() == 3, "psad: scalar slot spec is (offset, is_f64, index)");
        const int64_t width = sc[1] ? 8 : 4;
        TORCH_CHECK(sc[0] >= static_cast<int64_t>(8 * l.slot.size()) &&
                        sc[0] + width <= static_cast<int64_t>(l.args.size()) && sc[2] >= 0 && sc[2] < n_scalars,
                    "psad: scalar slot out of range");
        l.s_off.push_back(sc[0]);
        l.s_f64.push_back(sc[1]);
        l.s_idx.push_back(sc[2]);
    }
    return l;
}

std::vector<Alloc> make_allocs(const std::vector<std::vector<int64_t>>& shapes, const std::vector<int64_t>& dtypes,
                               const std::vector<bool>& zero) {
    TORCH_CHECK(shapes.size() == dtypes.size() && shapes.size() == zero.size(), "psad: allocation spec mismatch");
    std::vector<Alloc> r;
    for (size_t i = 0; i < shapes.size(); ++i)
        r.push_back(Alloc{shapes[i], static_cast<at::ScalarType>(dtypes[i]), static_cast<bool>(zero[i])});
    return r;
}

int64_t register_plan(const std::string& name, int64_t device, std::vector<std::vector<int64_t>> in_shape,
                      std::vector<int64_t> in_dtype, std::vector<std::vector<int64_t>> fwd_shape,
                      std::vector<int64_t> fwd_dtype, std::vector<bool> fwd_zero, uint64_t fwd_fn, int64_t fwd_grid,
                      int64_t fwd_block, py::bytes fwd_args, std::vector<int64_t> fwd_slot,
                      std::vector<std::vector<int64_t>> fwd_scal, std::vector<int64_t> saved, std::vector<std::vector<int64_t>> bwd_shape,
                      std::vector<int64_t> bwd_dtype, std::vector<bool> bwd_zero, uint64_t bwd_fn, int64_t bwd_grid,
                      int64_t bwd_block, py::bytes bwd_args, std::vector<int64_t> bwd_slot,
                      std::vector<std::vector<int64_t>> bwd_scal, std::vector<int64_t> grad_of_input,
                      int64_t n_scalars) {
    auto p = std::make_unique<Plan>();
    p->name = name;
    p->device = static_cast<int>(device);
    TORCH_CHECK(in_shape.size() == in_dtype.size() && grad_of_input.size() == in_shape.size(),
                "psad: input spec mismatch");
    p->in_shape = std::move(in_shape);
    for (auto d : in_dtype) p->in_dtype.push_back(static_cast<at::ScalarType>(d));
    p->fwd_out = make_allocs(fwd_shape, fwd_dtype, fwd_zero);
    p->n_scalars = n_scalars;
    p->fwd = make_launch(fwd_fn, fwd_grid, fwd_block, fwd_args, std::move(fwd_slot), fwd_scal, n_scalars);
    p->saved = std::move(saved);
    p->bwd_out = make_allocs(bwd_shape, bwd_dtype, bwd_zero);
    p->bwd = make_launch(bwd_fn, bwd_grid, bwd_block, bwd_args, std::move(bwd_slot), bwd_scal, n_scalars);
    p->grad_of_input = std::move(grad_of_input);
    const int64_t n_fwd = static_cast<int64_t>(p->in_shape.size() + p->fwd_out.size());
    for (auto i : p->fwd.slot) TORCH_CHECK(i >= 0 && i < n_fwd, "psad: forward slot out of range");
    for (auto i : p->saved) TORCH_CHECK(i >= 0 && i < n_fwd, "psad: saved index out of range");
    const int64_t n_bwd = static_cast<int64_t>(p->saved.size() + p->fwd_out.size() + p->bwd_out.size());
    for (auto i : p->bwd.slot) TORCH_CHECK(i >= 0 && i < n_bwd, "psad: backward slot out of range");
    for (auto i : p->grad_of_input) TORCH_CHECK(i >= -1 && i < n_bwd, "psad: gradient index out of range");
    std::lock_guard<std::mutex> lock(g_mutex);
    g_plans.push_back(std::move(p));
    return static_cast<int64_t>(g_plans.size()) - 1;
}


// (fn, grid, block, args, slot, scal) → Launch
Launch launch_from(const py::tuple& t, int64_t n_scalars) {
    TORCH_CHECK(t.size() == 6 || t.size() == 7, "psad: launch spec is (fn, grid, block, args, slot, scal[, sig])");
    Launch l = make_launch(t[0].cast<uint64_t>(), t[1].cast<int64_t>(), t[2].cast<int64_t>(), t[3].cast<py::bytes>(),
                           t[4].cast<std::vector<int64_t>>(), t[5].cast<std::vector<std::vector<int64_t>>>(), n_scalars);
    if (t.size() == 7) {
        // (start-signal word, value, halo-wait word, value) byte offsets, -1 where the kernel has none
        const auto sig = t[6].cast<std::vector<int64_t>>();
        TORCH_CHECK(sig.size() == 4, "psad: signal offsets are (sig word, sig value, wait word, wait value)");
        const int64_t n = static_cast<int64_t>(l.args.size()), lo = 8 * static_cast<int64_t>(l.slot.size());
        for (int k = 0; k < 4; k += 2) {
            if (sig[k] < 0) continue;
            TORCH_CHECK(sig[k] >= lo && sig[k] % 8 == 0 && sig[k] + 8 <= n && sig[k + 1] >= sig[k] + 8 &&
                            sig[k + 1] + 4 <= n, "psad: signal offsets out of range");
        }
        l.sig_ptr_off = sig[0];
        l.sig_val_off = sig[1];
        l.hw_ptr_off = sig[2];
        l.hw_val_off = sig[3];
    }
    return l;
}

// inner (launch spec or None), faces [launch spec], exchange (slot, last_off, recv_lo, recv_hi, bytes, peer_lo,
// peer_hi, loopback), comm, halo stream
Sweep sweep_from(const py::object& inner, const py::list& faces, const py::tuple& ex, uint64_t comm, uint64_t stream,
                 int64_t n_scalars, int64_t n_table) {
    Sweep w;
    if (!inner.is_none()) {
        w.has_inner = true;
        w.inner = launch_from(inner.cast<py::tuple>(), n_scalars);
    }
    for (const auto& f : faces) w.faces.push_back(launch_from(f.cast<py::tuple>(), n_scalars));
    TORCH_CHECK(ex.size() == 8, "psad: exchange spec has 8 entries");
    w.ex.slot = ex[0].cast<std::vector<int64_t>>();
    w.ex.last_off = ex[1].cast<std::vector<int64_t>>();
    for (auto v : ex[2].cast<std::vector<uint64_t>>()) w.ex.recv_lo.push_back(reinterpret_cast<void*>(v));
    for (auto v : ex[3].cast<std::vector<uint64_t>>()) w.ex.recv_hi.push_back(reinterpret_cast<void*>(v));
    for (auto v : ex[4].cast<std::vector<int64_t>>()) w.ex.bytes.push_back(static_cast<size_t>(v));
    w.ex.peer_lo = ex[5].cast<int>();
    w.ex.peer_hi = ex[6].cast<int>();
    w.ex.loopback = ex[7].cast<bool>();
    // face launches on the halo stream right behind the exchange (default; 'compute': after the interior on the
    // compute stream). Loopback proxy, one MI355X (profiles/r04_slab_sync_ab.log): 27-point 96x768^2 fp16 0.120 vs
    // 0.128-0.132 ms per step, 7-point 128x1024^2 fp32 0.398 vs 0.419 (with the stream-memory-op sync below)
    const char* fo = std::getenv("PSAD_SLAB_FACES");
    w.faces_on_halo = !(fo != nullptr && std::string(fo) == "compute");
    const size_t n = w.ex.slot.size();
    TORCH_CHECK(w.ex.last_off.size() == n && w.ex.recv_lo.size() == n && w.ex.recv_hi.size() == n &&
                    w.ex.bytes.size() == n, "psad: exchange spec lengths differ");
    for (size_t i = 0; i < n; ++i) {
        TORCH_CHECK(w.ex.slot[i] >= 0 && w.ex.slot[i] < n_table && w.ex.last_off[i] >= 0, "psad: exchange slot");
        TORCH_CHECK((w.ex.peer_lo < 0 || w.ex.recv_lo[i]) && (w.ex.peer_hi < 0 || w.ex.recv_hi[i]),
                    "psad: a receive buffer is missing for a neighbour");
    }
    for (const auto& l : w.faces)
        for (auto i : l.slot) TORCH_CHECK(i >= 0 && i < n_table, "psad: face slot out of range");
    if (w.has_inner)
        for (auto i : w.inner.slot) TORCH_CHECK(i >= 0 && i < n_table, "psad: interior slot out of range");
    if (n) {
        w.ex.comm = reinterpret_cast<void*>(comm);
        w.ex.stream = reinterpret_cast<hipStream_t>(stream);
        TORCH_CHECK(w.ex.comm != nullptr, "psad: exchange without a communicator");
        hip_ok(hipEventCreateWithFlags(&w.ex.ev_faces, hipEventDisableTiming), "hipEventCreateWithFlags");
        hip_ok(hipEventCreateWithFlags(&w.ex.ev_halos, hipEventDisableTiming), "hipEventCreateWithFlags");
        // the two cross-stream orderings as stream memory operations on signal memory (default) or, with
        // PSAD_SLAB_SYNC=event, event record + wait
        const char* sy = std::getenv("PSAD_SLAB_SYNC");
        if (!(sy != nullptr && std::string(sy) == "event")) {
            void* p = nullptr;
            void* q = nullptr;
            hip_ok(hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory), "hipExtMallocWithFlags");
            hip_ok(hipExtMallocWithFlags(&q, 8, hipMallocSignalMemory), "hipExtMallocWithFlags");
            hip_ok(hipMemset(p, 0, 8), "hipMemset");
            hip_ok(hipMemset(q, 0, 8), "hipMemset");
            hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
            w.ex.sig = static_cast<uint32_t*>(p);
            w.ex.sig_halo = static_cast<uint32_t*>(q);
            w.ex.faces_by_event = sy != nullptr && std::string(sy) == "mixed";
            const char* ss = std::getenv("PSAD_SLAB_START_SIG");
            w.ex.start_sig = !(ss != nullptr && std::string(ss) == "0");
            const char* fw = std::getenv("PSAD_SLAB_FACE_WAIT");
            w.ex.faces_wait = fw != nullptr && std::string(fw) == "1";
        }
    }
    return w;
}

int64_t register_slab_plan(const std::string& name, int64_t device, std::vector<std::vector<int64_t>> in_shape,
                           std::vector<int64_t> in_dtype, std::vector<std::vector<int64_t>> fwd_shape,
                           std::vector<int64_t> fwd_dtype, std::vector<bool> fwd_zero, py::object fwd_inner,
                           py::list fwd_faces, py::tuple fwd_ex, std::vector<int64_t> saved,
                           std::vector<std::vector<int64_t>> bwd_shape, std::vector<int64_t> bwd_dtype,
                           std::vector<bool> bwd_zero, py::object bwd_inner, py::list bwd_faces, py::tuple bwd_ex,
                           std::vector<int64_t> grad_of_input, int64_t n_scalars, uint64_t comm, uint64_t stream) {
    auto p = std::make_unique<SlabPlan>();
    p->name = name;
    p->device = static_cast<int>(device);
    TORCH_CHECK(in_shape.size() == in_dtype.size() && grad_of_input.size() == in_shape.size(),
                "psad: input spec mismatch");
    p->in_shape = std::move(in_shape);
    for (auto d : in_dtype) p->in_dtype.push_back(static_cast<at::ScalarType>(d));
    p->fwd_out = make_allocs(fwd_shape, fwd_dtype, fwd_zero);
    p->bwd_out = make_allocs(bwd_shape, bwd_dtype, bwd_zero);
    p->n_scalars = n_scalars;
    p->saved = std::move(saved);
    p->grad_of_input = std::move(grad_of_input);
    const int64_t n_fwd = static_cast<int64_t>(p->in_shape.size() + p->fwd_out.size());
    for (auto i : p->saved) TORCH_CHECK(i >= 0 && i < n_fwd, "psad: saved index out of range");
    const int64_t n_bwd = static_cast<int64_t>(p->saved.size() + p->fwd_out.size() + p->bwd_out.size());
    for (auto i : p->grad_of_input) TORCH_CHECK(i >= -1 && i < n_bwd, "psad: gradient index out of range");
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
    p->fwd = sweep_from(fwd_inner, fwd_faces, fwd_ex, comm, stream, n_scalars, n_fwd);
    p->bwd = sweep_from(bwd_inner, bwd_faces, bwd_ex, comm, stream, n_scalars, n_bwd);
    std::lock_guard<std::mutex> lock(g_mutex);
    g_slab_plans.push_back(std::move(p));
    return static_cast<int64_t>(g_slab_plans.size()) - 1;
}

py::object apply_slab(int64_t id, const std::vector<at::Tensor>& inputs, const std::vector<double>& scalars) {
    const SlabPlan& p = slab_plan_at(id);
    if (inputs.size() != p.in_shape.size() || static_cast<int64_t>(scalars.size()) != p.n_scalars) return py::none();
    for (size_t i = 0; i < inputs.size(); ++i) {
        const at::Tensor& t = inputs[i];
        if (!t.defined() || !t.is_cuda() || t.get_device() != p.device || t.scalar_type() != p.in_dtype[i] ||
            t.sizes() != at::IntArrayRef(p.in_shape[i]) || !t.is_contiguous() || !aligned(t))
            return py::none();
    }
    auto outs = SlabFunction::apply(id, at::TensorList(inputs), scalars);
    return py::cast(outs);
}

// Forward through the plan, or None when the call does not match it.
py::object apply(int64_t id, const std::vector<at::Tensor>& inputs, const std::vector<double>& scalars) {
    const Plan& p = plan_at(id);
    if (inputs.size() != p.in_shape.size() || static_cast<int64_t>(scalars.size()) != p.n_scalars) return py::none();
    for (size_t i = 0; i < inputs.size(); ++i) {
        const at::Tensor& t = inputs[i];
        if (!t.defined() || !t.is_cuda() || t.get_device() != p.device || t.scalar_type() != p.in_dtype[i] ||
            t.sizes() != at::IntArrayRef(p.in_shape[i]) || !t.is_contiguous() || !aligned(t))
            return py::none();
    }
    auto outs = StencilFunction::apply(id, at::TensorList(inputs), scalars);
    return py::cast(outs);
}

}  // namespace

#ifndef PSAD_SOURCE_HASH
#define PSAD_SOURCE_HASH "0000000000000000"
#endif
__attribute__((used)) static const char k_source_stamp[] = "PSAD_SOURCE_HASH=" PSAD_SOURCE_HASH;

PYBIND11_MODULE(_psad_torch, m) {
    m.doc() = "native autograd node of the torch_native stencil op (see psad_torch.cpp)";
    m.def("source_hash", []() { return std::string(k_source_stamp + 17); },
          "sha256 prefix of csrc/psad_torch.cpp + include/psad.h this module was built from (build.py)");
    m.def("register_plan", &register_plan);
    m.def("apply", &apply);
    m.def("register_slab_plan", &register_slab_plan);
    m.def("apply_slab", &apply_slab);
    m.def("num_slab_plans", []() {
        std::lock_guard<std::mutex> lock(g_mutex);
        return static_cast<int64_t>(g_slab_plans.size());
    });
    m.def("num_event_sweeps", []() { return g_event_sweeps.load(); },
          "exchanging slab sweeps ordered by event record + wait (PSAD_SLAB_SYNC=event, or another compute stream)");
    m.def("num_start_signal_sweeps", []() { return g_start_sig_sweeps.load(); },
          "exchanging slab sweeps whose interior launch signalled the halo stream itself (tests)");
    m.def("num_face_wait_sweeps", []() { return g_face_wait_sweeps.load(); },
          "exchanging slab sweeps whose face launches waited for the halos in-kernel on the compute stream (tests)");
    m.def("set_debug_poison", [](bool on) { g_poison.store(on); },
          "fill the outputs allocated uninitialised with NaN (tests: a kernel that leaves cells unwritten shows)");
    m.def("num_plans", []() {
        std::lock_guard<std::mutex> lock(g_mutex);
        return static_cast<int64_t>(g_plans.size());
    });
}
