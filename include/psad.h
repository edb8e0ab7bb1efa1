/*
 * psad.h — C ABI of the MI355X stencil execution layer (libpsad_hip.so).
 *
 * Drop-in boundary for the reference's compiled torch module
 * (pystencils_autodiff backends/astnodes.py:95-182 TorchModule + compile(),
 *  framework_integration/astnodes.py:224-255 generate_kernel_call,
 *  backends/python_bindings.py:162-176 PYBIND11 "call_<kernel>" wrappers).
 * The reference JIT-compiles a C++/CUDA translation unit per operator with
 * torch.utils.cpp_extension.load and exposes `call_<kernel>(at::Tensor&...)`.
 * Here the emitted HIP source is compiled with hiprtc for gfx950, the code
 * object is loaded as a hipModule, and kernels are launched on the caller's
 * stream with plain pointers and sizes (no torch types cross this boundary).
 *
 * Errors: every entry point returns 0 on success or a hipError_t / hiprtcResult
 * code (hiprtc codes are offset by PSAD_HIPRTC_ERROR_BASE); psad_error_string()
 * describes a code. Unlike the reference's gpuErrchk (framework_integration/
 * astnodes.py:258-286) nothing here calls exit().
 */
#ifndef PSAD_H
#define PSAD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSAD_HIPRTC_ERROR_BASE 10000

/* ABI version of this header; bumped on any signature change (3: psad_source_hash added). */
int psad_abi_version(void);

/* The sources the library was built from: 16 hex digits of sha256 over csrc/psad_hip.cpp, csrc/psad_halo.cpp and
 * this header (pystencils_autodiff_amd/build.py). The Python layer refuses a library whose stamp differs from the
 * sources of the tree it runs from (a stale build). No reference counterpart (plumbing). */
const char* psad_source_hash(void);

/* Compile HIP `source` with hiprtc. `options` e.g. {"--offload-arch=gfx950","-O3"}.
 * On success *code / *code_size receive a malloc'ed code object (free with psad_free).
 * The compiler log (possibly empty) is copied, NUL-terminated, into `log` (size `log_size`).
 * Replaces: TorchModule.compile() (backends/astnodes.py:148-182). */
int psad_rtc_compile(const char* source, const char* program_name, const char* const* options, int n_options,
                     void** code, size_t* code_size, char* log, size_t log_size);

/* hiprtc version (major*100+minor), -1 if unavailable. */
int psad_rtc_version(void);

void psad_free(void* p);

/* Load a code object on the current device. Replaces: cpp_extension.load's import (astnodes.py:171-182). */
int psad_module_load(const void* code, size_t code_size, void** module);
int psad_module_unload(void* module);

/* Look up an extern "C" kernel. Replaces: getattr(compiled_op, "call_" + name) (_torch_native.py:86,116). */
int psad_module_get_function(void* module, const char* name, void** function);

/* Launch `function` on `stream` (a hipStream_t, NULL = legacy default stream) with arguments packed
 * in `args` (`args_size` bytes, each argument at its natural alignment, as hipModuleLaunchKernel's
 * HIP_LAUNCH_PARAM_BUFFER_POINTER expects). Asynchronous; no host synchronisation.
 * Replaces: kernel<<<grid, block>>>(...) + gpuErrchk (printer.py:88-108, astnodes.py:248-251). */
int psad_launch(void* function, unsigned grid_x, unsigned grid_y, unsigned grid_z, unsigned block_x,
                unsigned block_y, unsigned block_z, unsigned shared_bytes, void* stream, const void* args,
                size_t args_size);

/* Registers / LDS / occupancy of a loaded kernel (for diagnostics). */
int psad_function_attributes(void* function, int* num_regs, int* shared_bytes, int* max_threads);

/* Current device, device count, and hipGetLastError(). */
int psad_get_device(int* device);
int psad_device_count(int* count);
int psad_last_error(void);

/* Stream-ordered device-to-device copy (halo staging). */
int psad_memcpy_d2d_async(void* dst, const void* src, size_t bytes, void* stream);

/* --- RCCL halo exchange (z-slab decomposition; no counterpart in the reference, which has no
 * multi-GPU path — SURVEY.md §8e). Codes from RCCL are offset by PSAD_RCCL_ERROR_BASE. --- */
#define PSAD_RCCL_ERROR_BASE 20000

/* dlopen librccl (e.g. torch's bundled copy) and resolve the NCCL 2.x entry points used below. */
int psad_rccl_open(const char* library_path);

/* ncclGetUniqueId into `id` (128 bytes), to be broadcast to every rank by the caller. */
int psad_rccl_unique_id(void* id);

/* ncclCommInitRank over `nranks` ranks (collective: every rank calls it with the same id). */
int psad_rccl_comm_init(const void* id, int nranks, int rank, void** comm);
int psad_rccl_comm_destroy(void* comm);

/* Swap slab boundary planes with the neighbouring ranks in ONE ncclGroupStart/End on `stream`: for
 * each of `n_fields` fields, send `send_lo[i]` to / receive `recv_lo[i]` from `peer_lo`, and
 * `send_hi[i]` / `recv_hi[i]` with `peer_hi` (`bytes[i]` each; a peer < 0 skips that side).
 * Stream-ordered and asynchronous, like the kernels that produce and consume the planes. */
int psad_halo_exchange(void* comm, int n_fields, const void* const* send_lo, void* const* recv_lo,
                       const void* const* send_hi, void* const* recv_hi, const size_t* bytes, int peer_lo,
                       int peer_hi, void* stream);

const char* psad_rccl_error_string(int code);

/* Human-readable description of a code returned above. */
const char* psad_error_string(int code);

#ifdef __cplusplus
}
#endif

#endif /* PSAD_H */
