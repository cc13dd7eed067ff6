// spt_jit.hip — run-time specialization of the persistent kernels to a flat scene's shape.
//
// A flat scene (<= 32 primitives, the Cornell box of C2/C3, the App's spheres) is tested in full by
// every ray segment (closest_flat in spt_kernels.hip). Compiled for one shape — the number of
// primitives of each kind, packed in flat_shape_key — the group loops unroll and the compiler
// schedules the scalar record loads ahead of the tests (C2 +7.6 %). Only the
// counts are baked in: positions, materials and the sky stay in device memory, so moving a sphere
// re-uses the kernel, and a new shape costs one hiprtc compile (~1.5-2 s, cached per process).
//
// hiprtc compiles the library's own kernel source (embedded at build time: spt_jit_src.inc, made by
// scripts/embed_sources.py) with the flags of the offline build (Makefile HIPFLAGS: -O3, no FMA
// contraction, no SLP vectorization), so the specialized kernel evaluates the same expressions in
// the same order and gives the same bits as the generic one (tests/test_gpu_parity.py checks both
// against each other and the oracle). If hiprtc is missing or a compile fails, launch_paths /
// launch_frame run the generic kernels and spt_stats.specialized stays 0.
//
// The render path never waits for the compiler (round 3): spt_set_scene queues the new shape's
// compiles on the compile worker thread (jit_prefetch) and launches ask with wait = false, so a frame
// rendered before the compile has finished runs the generic kernel — same bits — and the App's UI
// thread never stalls for seconds on a new shape. spt_specialize_scene (and spt_tuning.specialize = 1)
// wait for the worker instead. Every hiprtc call runs on that one worker thread (see rtc()).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <pthread.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <type_traits>
#include <vector>

#include "spt_jit.h"
#include "spt_jit_src.inc"  // kJitSources: {file name, text} of spt_kernels.hip and its headers

namespace spt {
namespace {

// hiprtc of the ROCm install the library was built for, in a link namespace of its own (dlmopen):
// a host process may already have another ROCm's hiprtc and comgr loaded under the same sonames
// (PyTorch wheels bundle theirs), and an older compiler generates different, slower code for the
// same source (C2: 75.5 vs 79 Gsamples/s with PyTorch's ROCm 7.0 hiprtc).
struct Rtc {
    bool ok = false;
    int major = 0, minor = 0;
    std::string where;
    decltype(&hiprtcCreateProgram) create = nullptr;
    decltype(&hiprtcAddNameExpression) add_name = nullptr;
    decltype(&hiprtcCompileProgram) compile = nullptr;
    decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
    decltype(&hiprtcGetProgramLog) log = nullptr;
    decltype(&hiprtcGetLoweredName) lowered = nullptr;
    decltype(&hiprtcGetCodeSize) code_size = nullptr;
    decltype(&hiprtcGetCode) code = nullptr;
    decltype(&hiprtcDestroyProgram) destroy = nullptr;
    decltype(&hiprtcGetErrorString) error_string = nullptr;
    decltype(&hiprtcVersion) version = nullptr;
};

// Called only on the compile worker thread (worker_main): hiprtc/comgr loaded into their own
// namespace are used only from the thread that loaded them — a compile on a thread created after the
// dlmopen segfaulted in comgr (reproduced on the host with AMD_COMGR_CACHE=0), while compiles on the
// loading thread are fine. Never destroyed: the worker may still be compiling during static teardown.
// A fork()ed child's worker (the parent's did not survive the fork) loads its own copy (at_fork_child).
const Rtc* g_rtc = nullptr;
const Rtc& rtc() {
    if (g_rtc) return *g_rtc;
    g_rtc = new Rtc([] {
        Rtc t;
        const char* root = std::getenv("ROCM_PATH");
        const std::string path = std::string(root && *root ? root : "/opt/rocm") + "/lib/libhiprtc.so.7";
        void* h = dlmopen(LM_ID_NEWLM, path.c_str(), RTLD_NOW | RTLD_LOCAL);
        t.where = path + (h ? " (own namespace)" : "");
        if (!h) {  // e.g. no namespace left: the process's default binding
            h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
            t.where = path + " (shared namespace)";
        }
        if (!h) return t;
        bool all = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            all = all && fn != nullptr;
        };
        sym(t.create, "hiprtcCreateProgram");
        sym(t.add_name, "hiprtcAddNameExpression");
        sym(t.compile, "hiprtcCompileProgram");
        sym(t.log_size, "hiprtcGetProgramLogSize");
        sym(t.log, "hiprtcGetProgramLog");
        sym(t.lowered, "hiprtcGetLoweredName");
        sym(t.code_size, "hiprtcGetCodeSize");
        sym(t.code, "hiprtcGetCode");
        sym(t.destroy, "hiprtcDestroyProgram");
        sym(t.error_string, "hiprtcGetErrorString");
        sym(t.version, "hiprtcVersion");
        t.ok = all && t.version(&t.major, &t.minor) == HIPRTC_SUCCESS;
        return t;
    }());
    return *g_rtc;
}

struct Program {
    std::vector<char> code;  // the compiled code object (empty: the compile failed)
    std::string lowered;     // the kernel's mangled name in it
    std::string log;
    int state = 0;           // 0 not started, 1 compiling, 2 done (code or log set)
};

#ifndef SPT_DEFAULT_ARCH
#define SPT_DEFAULT_ARCH "gfx950"  // Makefile ARCH: the offline build's target, used without a device
#endif

using CodeKey = std::tuple<std::string, int, int, uint64_t>;  // (arch, kernel, env, shape)

// Process-lifetime state, never destroyed: the compile worker may still run while static destructors
// would otherwise tear it down (it is stopped and joined at exit, see stop_worker).
struct JitState {
    std::mutex mu;
    std::condition_variable cv;
    std::map<CodeKey, Program> code;
    std::map<std::tuple<int, int, int, uint64_t>, hipFunction_t> fns;  // (device, kernel, env, shape)
    std::deque<CodeKey> queue;  // compiles waiting for the worker
    std::thread worker;
    bool started = false, stop = false, rtc_known = false;
    std::string compiler;  // jit_compiler()'s answer, set by the worker once hiprtc is loaded
};

JitState* g_state = nullptr;
void at_fork_prepare();
void at_fork_parent();
void at_fork_child();
JitState& st() {
    static const bool registered = [] {
        g_state = new JitState();
        pthread_atfork(at_fork_prepare, at_fork_parent, at_fork_child);
        return true;
    }();
    (void)registered;
    return *g_state;
}

// fork(): a child process has no compile worker (threads do not survive a fork), so it starts over
// with a fresh state and starts a worker of its own on first use — which loads its own hiprtc (the
// loading thread rule above). The compiled code objects are kept; the loaded kernels (fns) are not:
// they belong to the parent's HIP context. The parent's lock is held across the fork, so the state the
// child copies is consistent. The old state is leaked (its std::thread is joinable and must not be
// destroyed in the child).
void at_fork_prepare() { g_state->mu.lock(); }
void at_fork_parent() { g_state->mu.unlock(); }
void at_fork_child() {
    JitState* old = g_state;
    JitState* fresh = new JitState();
    for (auto& kv : old->code)
        if (kv.second.state == 2) fresh->code[kv.first] = kv.second;  // finished compiles only
    g_state = fresh;
    g_rtc = nullptr;
}

Program compile_now(const std::string& arch, int kernel, int env, uint64_t shape);

// The one thread that loads hiprtc and runs every compile, in queue order.
void worker_main() {
    const Rtc& r = rtc();
    {
        std::lock_guard<std::mutex> lock(st().mu);
        st().compiler = r.ok ? "hiprtc " + std::to_string(r.major) + "." + std::to_string(r.minor) + " from " + r.where
                             : "unavailable: " + r.where;
        st().rtc_known = true;
        st().cv.notify_all();
    }
    for (;;) {
        CodeKey key;
        {
            std::unique_lock<std::mutex> lock(st().mu);
            st().cv.wait(lock, [] { return st().stop || !st().queue.empty(); });
            if (st().stop) return;  // exit: queued compiles are dropped
            key = st().queue.front();
            st().queue.pop_front();
        }
        Program p = compile_now(std::get<0>(key), std::get<1>(key), std::get<2>(key), std::get<3>(key));
        std::lock_guard<std::mutex> lock(st().mu);
        p.state = 2;
        st().code[key] = std::move(p);
        st().cv.notify_all();
    }
}

void stop_worker() {
    {
        std::lock_guard<std::mutex> lock(st().mu);
        st().stop = true;
        st().cv.notify_all();
    }
    if (st().worker.joinable()) st().worker.join();  // a compile in flight finishes first (~1-2 s)
}

// st().mu held
void ensure_worker() {
    if (st().started) return;
    st().started = true;
    st().worker = std::thread(worker_main);
    static bool at_exit = false;  // (a fork()ed child inherits the registration)
    if (!at_exit) std::atexit(stop_worker);
    at_exit = true;
}

std::string name_expr(int kernel, int env, uint64_t shape) {
    char buf[160];
    const bool frame = kernel == kJitFrame || kernel == kJitFrameNee || kernel == kJitFrameRgba || kernel == kJitFrameNeeRgba;
    const char* tail = kernel == kJitPathsChan ? ", 0, true"
                       : kernel == kJitPathsNee ? ", 0, false, 1"
                       : kernel == kJitFrameNee ? ", false, 1"  // (kNee = kNeeAll)
                       : kernel == kJitFrameRgba ? ", false, 0, true"
                       : kernel == kJitFrameNeeRgba ? ", false, 1, true" : "";
    std::snprintf(buf, sizeof buf, "spt::%s<false, false, %d, %lluull%s>", frame ? "k_frame" : "k_paths", env,
                  (unsigned long long)shape, tail);
    return buf;
}

// The device's architecture without its feature suffix ("gfx950:sramecc+:xnack-" -> "gfx950"), queried
// once per device (a launch asks while the background compile runs).
std::string device_arch(int device) {
    static std::mutex mu;
    static std::map<int, std::string> cache;
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = cache.find(device);
        if (it != cache.end()) return it->second;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SPT_DEFAULT_ARCH;
    std::string a = prop.gcnArchName;
    const size_t colon = a.find(':');
    if (colon != std::string::npos) a.resize(colon);
    if (a.empty()) a = SPT_DEFAULT_ARCH;
    std::lock_guard<std::mutex> lock(mu);
    cache[device] = a;
    return a;
}

// One hiprtc compile (no lock held).
Program compile_now(const std::string& arch, int kernel, int env, uint64_t shape) {
    Program out;
    const std::string expr = name_expr(kernel, env, shape);
    std::vector<const char*> hdr_src, hdr_name;
    for (size_t i = 1; i < kJitSourceCount; ++i) {
        hdr_name.push_back(kJitSources[i].name);
        hdr_src.push_back(kJitSources[i].text);
    }
    const Rtc& rt = rtc();
    if (!rt.ok) {
        out.log = "hiprtc unavailable: " + rt.where;
        return out;
    }
    hiprtcProgram prog;
    if (rt.create(&prog, kJitSources[0].text, kJitSources[0].name, (int)hdr_src.size(), hdr_src.data(),
                  hdr_name.data()) != HIPRTC_SUCCESS) {
        out.log = "hiprtcCreateProgram failed";
        return out;
    }
    rt.add_name(prog, expr.c_str());
    // the offline build's kernel flags (Makefile HIPFLAGS); -vectorize-slp=false is -fno-slp-vectorize
    std::vector<std::string> opt_s = {"--offload-arch=" + arch, "-O3", "-ffp-contract=off", "-fno-fast-math",
                                      "-std=c++17", "-mllvm", "-vectorize-slp=false"};
#ifdef SPT_JIT_EXTRA_OPTS  // experiment builds (scripts/build_variant.sh): the variant's -D flags
    {
        const std::string extra = SPT_JIT_EXTRA_OPTS;
        size_t i = 0;
        while (i < extra.size()) {
            const size_t j = extra.find(' ', i);
            const std::string w = extra.substr(i, j == std::string::npos ? std::string::npos : j - i);
            if (!w.empty()) opt_s.push_back(w);
            if (j == std::string::npos) break;
            i = j + 1;
        }
    }
#endif
    std::vector<const char*> opts;
    for (const auto& o : opt_s) opts.push_back(o.c_str());
    const hiprtcResult rc = rt.compile(prog, (int)opts.size(), opts.data());
    size_t log_size = 0;
    if (rt.log_size(prog, &log_size) == HIPRTC_SUCCESS && log_size > 1) {
        out.log.resize(log_size);
        rt.log(prog, &out.log[0]);
    }
    if (rc == HIPRTC_SUCCESS) {
        size_t n = 0;
        const char* lowered = nullptr;
        if (rt.lowered(prog, expr.c_str(), &lowered) == HIPRTC_SUCCESS && lowered)
            out.lowered = lowered;
        if (!out.lowered.empty() && rt.code_size(prog, &n) == HIPRTC_SUCCESS && n > 0) {
            out.code.resize(n);
            if (rt.code(prog, out.code.data()) != HIPRTC_SUCCESS) out.code.clear();
        }
    } else if (out.log.empty()) {
        out.log = rt.error_string(rc);
    }
    rt.destroy(&prog);
    return out;
}

// The finished entry `key`, queueing its compile on the worker if it has not started. wait: block until
// it is finished (moved to the front of the queue); !wait: nullptr while it is not finished.
// `lock` holds st().mu on entry and on return.
const Program* get_program(std::unique_lock<std::mutex>& lock, const CodeKey& key, bool wait) {
    Program& p = st().code[key];
    if (p.state == 0) {
        p.state = 1;
        if (wait) st().queue.push_front(key);
        else st().queue.push_back(key);
        ensure_worker();
        st().cv.notify_all();
    } else if (p.state == 1 && wait) {
        auto q = std::find(st().queue.begin(), st().queue.end(), key);
        if (q != st().queue.end() && q != st().queue.begin()) {
            st().queue.erase(q);
            st().queue.push_front(key);
        }
    }
    if (st().code[key].state != 2) {
        if (!wait) return nullptr;
        st().cv.wait(lock, [&] { return st().code[key].state == 2; });
    }
    return &st().code[key];
}

}  // namespace

std::string jit_compiler() {
    std::unique_lock<std::mutex> lock(st().mu);
    ensure_worker();
    st().cv.wait(lock, [] { return st().rtc_known; });
    return st().compiler;
}

bool jit_compile(int kernel, int env, uint64_t shape, std::string* log, std::vector<char>* code) {
    std::unique_lock<std::mutex> lock(st().mu);
    const Program* p = get_program(lock, CodeKey{SPT_DEFAULT_ARCH, kernel, env, shape}, true);
    if (log) *log = p->log;
    if (code) *code = p->code;
    return !p->code.empty();
}

void jit_prefetch(int kernel, int env, uint64_t shape) {
    int device = 0;
    const std::string arch = hipGetDevice(&device) == hipSuccess ? device_arch(device) : std::string(SPT_DEFAULT_ARCH);
    std::unique_lock<std::mutex> lock(st().mu);
    (void)get_program(lock, CodeKey{arch, kernel, env, shape}, false);
}

bool jit_ready(int kernel, int env, uint64_t shape) {
    int device = 0;
    const std::string arch = hipGetDevice(&device) == hipSuccess ? device_arch(device) : std::string(SPT_DEFAULT_ARCH);
    std::lock_guard<std::mutex> lock(st().mu);
    auto it = st().code.find(CodeKey{arch, kernel, env, shape});
    return it != st().code.end() && it->second.state == 2;
}

hipFunction_t jit_function(int kernel, int env, uint64_t shape, std::string* err, bool wait) {
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) return nullptr;
    const auto fkey = std::make_tuple(device, kernel, env, shape);
    {
        std::lock_guard<std::mutex> lock(st().mu);
        auto it = st().fns.find(fkey);
        if (it != st().fns.end()) return it->second;
    }
    const std::string arch = device_arch(device);
    std::unique_lock<std::mutex> lock(st().mu);
    auto it = st().fns.find(fkey);
    if (it != st().fns.end()) return it->second;
    const Program* p = get_program(lock, CodeKey{arch, kernel, env, shape}, wait);
    if (!p) return nullptr;  // still compiling in the background: the caller runs its generic kernel
    hipFunction_t fn = nullptr;
    if (!p->code.empty()) {
        hipModule_t mod = nullptr;
        if (hipModuleLoadData(&mod, p->code.data()) == hipSuccess) {
            if (hipModuleGetFunction(&fn, mod, p->lowered.c_str()) != hipSuccess) {
                fn = nullptr;
                if (err) *err = "hipModuleGetFunction failed for " + p->lowered;
            }
        } else if (err) {
            *err = "hipModuleLoadData failed";
        }
    } else if (err) {
        *err = p->log;
    }
    if (!fn) (void)hipGetLastError();  // a failed load must not surface in the caller's next error check
    st().fns[fkey] = fn;  // a failure is remembered too: the generic kernel runs from then on
    return fn;
}

}  // namespace spt
