// spt_jit.h — run-time specialization of the persistent kernels (spt_jit.hip). Internal.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace spt {

constexpr int kJitPaths = 0;  // k_paths<false, false, env, shape>
constexpr int kJitFrame = 1;  // k_frame<false, false, env, shape>
constexpr int kJitPathsChan = 2;  // k_paths<false, false, env, shape, 0, true> (small row shards)
constexpr int kJitPathsNee = 3;   // k_paths<false, false, 2, shape, 0, false, true> (SPT_FLAG_NEE; env = 2)
constexpr int kJitFrameNee = 4;   // k_frame<false, false, 2, shape, false, true> (SPT_FLAG_NEE; env = 2)
constexpr int kJitFrameRgba = 5;     // k_frame<false, false, env, shape, false, 0, true> (the fused resolve)
constexpr int kJitFrameNeeRgba = 6;  // k_frame<false, false, 2, shape, false, 1, true>

// Compile the kernel for a flat scene shape (flat_shape_key) without loading it (no device needed);
// false and the compiler log on failure; `code` (optional) receives the code object. Cached per process.
bool jit_compile(int kernel, int env, uint64_t shape, std::string* log, std::vector<char>* code = nullptr);
// Which compiler the specializations use ("hiprtc MAJOR.MINOR from PATH"), or why there is none.
std::string jit_compiler();
// The loaded kernel on the current device, or nullptr. wait = true: compiled now if it is not yet
// (blocks for the compile, ~1-2 s); nullptr only if it cannot be built. wait = false: never blocks on
// the compiler — nullptr until a background compile (started by this call if none is running) has
// finished, so the caller runs its generic kernel meanwhile.
hipFunction_t jit_function(int kernel, int env, uint64_t shape, std::string* err, bool wait = true);
// Start compiling (kernel, env, shape) on a background thread unless it is compiled or compiling
// (no device needed); returns at once.
void jit_prefetch(int kernel, int env, uint64_t shape);
// true once (kernel, env, shape) has finished compiling, successfully or not.
bool jit_ready(int kernel, int env, uint64_t shape);

}  // namespace spt
