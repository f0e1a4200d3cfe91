// Registry of the compile-time-G encoders (rs_encoder.hpp).
//
// k and n arrive per segment from the satellite (metaclient/client.go:1262-1267
// -> eestream.NewRedundancyStrategyFromProto, encode.go:69-87), so any (k, n)
// must reach the fast encoder:
//  * AOT: the configurations of rs_encoder_aot.def are compiled into the
//    library (one translation unit each, rs_encode_aot.hip).
//  * JIT: any other (k, n) inside the encoder's limits is compiled by hiprtc
//    from the same header text (embedded at build time, rs_jit_sources.inc),
//    in a background thread started on first request, and the code object is
//    cached on disk.  Until it is loaded, find_encoder() returns nullptr and
//    the caller runs the runtime-matrix GPU kernel instead, so no call ever
//    waits for the compiler unless it asks to (ec_prepare_encoder).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include "ec_log.hpp"

#include <condition_variable>
#include <cstdio>
#include <dlfcn.h>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <tuple>
#include <unistd.h>
#include <vector>

#include "rs_encoder.hpp"
#include "rs_kernels.hpp"

namespace uplink_ec {

#define UPLINK_AOT(K, N) EncoderKernel aot_encoder_##K##_##N();
#include "rs_encoder_aot.def"
#undef UPLINK_AOT

const EncoderKernel *aot_encoder(int k, int n) {
    static const std::vector<EncoderKernel> table = {
#define UPLINK_AOT(K, N) aot_encoder_##K##_##N(),
#include "rs_encoder_aot.def"
#undef UPLINK_AOT
    };
    for (const EncoderKernel &e : table)
        if (e.k == k && e.n == n) return &e;
    return nullptr;
}

bool encoder_supported(int k, int n) { return enc::supported(k, n); }

namespace {

#include "rs_jit_sources.inc"

uint64_t fnv1a(uint64_t h, const void *p, size_t n) {
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

std::string cache_dir() {
    if (const char *d = getenv("UPLINK_EC_JIT_CACHE")) return d;
    std::string base;
    if (const char *x = getenv("XDG_CACHE_HOME")) base = x;
    else if (const char *h = getenv("HOME")) base = std::string(h) + "/.cache";
    else base = "/tmp";
    return base + "/uplink_ec";
}

void mkdirs(const std::string &path) {
    for (size_t i = 1; i <= path.size(); i++)
        if (i == path.size() || path[i] == '/') (void)mkdir(path.substr(0, i).c_str(), 0700);
}

// The cache directory is trusted only if it is a directory (not a link) owned
// by this user and writable by no one else: its code objects run on the GPU.
bool cache_dir_trusted(const std::string &dir) {
    struct stat st;
    if (lstat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) return false;
    return st.st_uid == geteuid() && (st.st_mode & (S_IWGRP | S_IWOTH)) == 0;
}

std::string hex64(uint64_t h) {
    char hex[32];
    snprintf(hex, sizeof hex, "%016llx", (unsigned long long)h);
    return hex;
}

struct JitEntry {
    enum State { kCompiling, kReady, kFailed } state = kCompiling;
    std::vector<char> code;       // code object, both variants
    std::string full_name, parity_name;
    std::map<int, std::unique_ptr<EncoderKernel>> loaded;  // per device
    std::map<int, hipModule_t> modules;
    bool recompiled = false;  // compiled again after a cached code object failed to load
};

std::mutex g_mu;
std::condition_variable g_cv;
std::map<std::tuple<std::string, int, int>, std::unique_ptr<JitEntry>> g_jit;  // (arch, k, n)
std::vector<std::thread> g_threads;  // compile threads (joined at exit)
std::mutex g_compile_mu;             // one compilation at a time
bool g_exiting = false;              // set at exit: queued compilations are skipped

// Compile threads still running when the process exits must finish before
// anything they use is torn down.  exit() runs the handlers and C++ static
// destructors in the reverse order of their registration.  The HIP runtime
// registers its own on its first use, before any compile.  The compiler
// library (comgr, which hiprtc dlopens on its first compile) registers its
// static destructors when it is loaded: loaded lazily inside the compile
// thread, that was AFTER this handler, so at exit comgr's LLVM state was
// destroyed under a running compile -- the "double free or corruption (!prev)"
// abort of round 2.  So comgr is loaded here first
// (load_compiler), and this handler, registered after it, runs before its
// destructors.  Only the compilation in progress is waited for; the ones queued
// behind it give up (each takes seconds to a minute).
void join_compiles() {
    std::vector<std::thread> t;
    {
        std::lock_guard<std::mutex> g(g_mu);
        g_exiting = true;
        t.swap(g_threads);
    }
    const double t0 = log_ms();
    ec_logf("exit: joining %zu encoder compile thread(s)", t.size());
    for (auto &th : t)
        if (th.joinable()) th.join();
    ec_logf("exit: compile threads joined after %.1f ms", log_ms() - t0);
}

// Load the compiler library hiprtc would load on its first compile, and keep it
// (RTLD_NODELETE), so that its destructors are registered before join_compiles.
void load_compiler() {
    for (const char *so : {"libamd_comgr.so.3", "libamd_comgr.so"})
        if (dlopen(so, RTLD_NOW | RTLD_GLOBAL | RTLD_NODELETE)) return;
}

std::string variant_expr(int k, int n, int nc, int nl, bool copy) {
    return "&uplink_ec::enc::rs_encode_special<" + std::to_string(k) + ", " + std::to_string(n) + ", " +
           std::to_string(nc) + ", " + std::to_string(nl) + (copy ? ", true>" : ", false>");
}

// Compile (or read from the cache) the two variants of (k, n) for `arch`.
void compile_entry(JitEntry *e, std::string arch, int k, int n, bool read_cache) {
    const double t_queued = log_ms();
    std::lock_guard<std::mutex> serial(g_compile_mu);
    {
        std::lock_guard<std::mutex> g(g_mu);
        if (g_exiting) {
            ec_logf("RS(%d,%d) encoder compile skipped (exiting)", k, n);
            e->state = JitEntry::kFailed;
            g_cv.notify_all();
            return;
        }
    }
    const double t_start = log_ms();
    ec_logf("RS(%d,%d) encoder: start (%s, queued %.1f ms)", k, n, read_cache ? "cache allowed" : "no cache",
         t_start - t_queued);
    const std::string src = "#include \"rs_encoder.hpp\"\n";
    const std::string full = variant_expr(k, n, enc::full_compute_waves(k, n), enc::full_loader_waves(k, n), true),
                      parity = variant_expr(k, n, enc::parity_compute_waves(k, n), enc::loader_waves(k, n), false);
    std::vector<std::string> opts = {"--offload-arch=" + arch, "-O3", "-std=c++20"};
    uint64_t h = 0xcbf29ce484222325ull;
    for (int i = 0; i < kJitHeaderCount; i++) h = fnv1a(h, kJitHeaderTexts[i], strlen(kJitHeaderTexts[i]));
    for (const auto &o : opts) h = fnv1a(h, o.data(), o.size());
    h = fnv1a(h, full.data(), full.size());
    h = fnv1a(h, parity.data(), parity.size());
    int ver_major = 0, ver_minor = 0;
    (void)hiprtcVersion(&ver_major, &ver_minor);
    h = fnv1a(h, &ver_major, sizeof ver_major);
    h = fnv1a(h, &ver_minor, sizeof ver_minor);
    const std::string dir = cache_dir(), path = dir + "/enc_" + std::to_string(k) + "_" + std::to_string(n) + "_" + hex64(h);
    mkdirs(dir);
    const bool trusted = cache_dir_trusted(dir);
    std::vector<char> code;
    std::string names[2];
    if (trusted && read_cache) {
        // .names holds the two kernel names and the digest of the code object; an
        // entry that does not match it is removed and compiled again
        std::ifstream in(path + ".co", std::ios::binary);
        std::ifstream nm(path + ".names");
        std::string digest;
        if (in && nm && std::getline(nm, names[0]) && std::getline(nm, names[1]) && std::getline(nm, digest))
            code.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
        if (!code.empty() && hex64(fnv1a(0xcbf29ce484222325ull, code.data(), code.size())) != digest) code.clear();
        if (code.empty()) {
            (void)remove((path + ".co").c_str());
            (void)remove((path + ".names").c_str());
        }
        ec_logf("RS(%d,%d) encoder: disk cache %s (%s)", k, n, code.empty() ? "miss" : "hit", path.c_str());
    } else {
        ec_logf("RS(%d,%d) encoder: disk cache not used (%s: %s)", k, n, dir.c_str(),
             trusted ? "recompiling" : "not a private directory of this user");
    }
    if (code.empty()) {
        hiprtcProgram prog;
        bool ok = hiprtcCreateProgram(&prog, src.c_str(), "rs_encoder_jit.hip", kJitHeaderCount, kJitHeaderTexts,
                                      kJitHeaderNames) == HIPRTC_SUCCESS;
        if (ok) {
            // one expression when both variants are the same instantiation (fewer than 32 parity rows)
            ok = hiprtcAddNameExpression(prog, full.c_str()) == HIPRTC_SUCCESS &&
                 (parity == full || hiprtcAddNameExpression(prog, parity.c_str()) == HIPRTC_SUCCESS);
            std::vector<const char *> o;
            for (const auto &s : opts) o.push_back(s.c_str());
            if (ok && hiprtcCompileProgram(prog, (int)o.size(), o.data()) != HIPRTC_SUCCESS) {
                size_t n_log = 0;
                hiprtcGetProgramLogSize(prog, &n_log);
                std::string log(n_log, '\0');
                hiprtcGetProgramLog(prog, &log[0]);
                fprintf(stderr, "uplink_ec: hiprtc failed for RS(%d,%d):\n%s\n", k, n, log.c_str());
                ok = false;
            }
            const char *lowered[2] = {nullptr, nullptr};
            if (ok) {
                ok = hiprtcGetLoweredName(prog, full.c_str(), &lowered[0]) == HIPRTC_SUCCESS &&
                     hiprtcGetLoweredName(prog, parity.c_str(), &lowered[1]) == HIPRTC_SUCCESS;
                if (parity == full) lowered[1] = lowered[0];
            }
            size_t sz = 0;
            if (ok) ok = hiprtcGetCodeSize(prog, &sz) == HIPRTC_SUCCESS && sz > 0;
            if (ok) {
                code.resize(sz);
                ok = hiprtcGetCode(prog, code.data()) == HIPRTC_SUCCESS;
                names[0] = lowered[0];
                names[1] = lowered[1];
            }
            hiprtcDestroyProgram(&prog);
        }
        if (!ok) code.clear();
        if (!code.empty() && trusted) {  // publish atomically: write a temp file, rename
            const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
            std::ofstream out(tmp + ".co", std::ios::binary);
            out.write(code.data(), (std::streamsize)code.size());
            std::ofstream nm(tmp + ".names");
            nm << names[0] << "\n" << names[1] << "\n" << hex64(fnv1a(0xcbf29ce484222325ull, code.data(), code.size())) << "\n";
            out.close();
            nm.close();
            if (out && nm) {
                (void)rename((tmp + ".names").c_str(), (path + ".names").c_str());
                (void)rename((tmp + ".co").c_str(), (path + ".co").c_str());
            } else {
                (void)remove((tmp + ".co").c_str());
                (void)remove((tmp + ".names").c_str());
            }
        }
    }
    ec_logf("RS(%d,%d) encoder: %s after %.1f ms", k, n, code.empty() ? "FAILED" : "code object ready",
         log_ms() - t_start);
    std::lock_guard<std::mutex> g(g_mu);
    if (code.empty()) {
        e->state = JitEntry::kFailed;
    } else {
        e->code = std::move(code);
        e->full_name = names[0];
        e->parity_name = names[1];
        e->state = JitEntry::kReady;
    }
    g_cv.notify_all();
}

std::string device_arch(int dev) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return "";
    std::string a = p.gcnArchName;
    return a.substr(0, a.find(':'));
}

}  // namespace

// Start (if needed and `start`) the run-time compilation of (k, n); with
// `wait`, block until it is done.  Returns the encoder when it is loaded on
// the current device, else nullptr.
const EncoderKernel *jit_encoder(int k, int n, bool wait, bool start) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    const std::string arch = device_arch(dev);
    if (arch.empty()) return nullptr;
    std::unique_lock<std::mutex> g(g_mu);
    auto key = std::make_tuple(arch, k, n);
    auto it = g_jit.find(key);
    if (it == g_jit.end()) {
        if (!start) return nullptr;
        JitEntry *e = new JitEntry();
        g_jit.emplace(key, std::unique_ptr<JitEntry>(e));
        static std::once_flag once;
        std::call_once(once, [] {
            load_compiler();
            std::atexit(join_compiles);
        });
        g_threads.emplace_back(compile_entry, e, arch, k, n, true);
        it = g_jit.find(key);
    }
    JitEntry *e = it->second.get();
    if (wait) g_cv.wait(g, [&] { return e->state != JitEntry::kCompiling; });
    if (e->state != JitEntry::kReady) return nullptr;
    auto ld = e->loaded.find(dev);
    if (ld != e->loaded.end()) return ld->second.get();
    hipModule_t mod = nullptr;
    hipFunction_t f_full = nullptr, f_par = nullptr;
    if (hipModuleLoadData(&mod, e->code.data()) != hipSuccess ||
        hipModuleGetFunction(&f_full, mod, e->full_name.c_str()) != hipSuccess ||
        hipModuleGetFunction(&f_par, mod, e->parity_name.c_str()) != hipSuccess) {
        if (mod) (void)hipModuleUnload(mod);
        if (!e->recompiled && !g_exiting) {
            // a code object that passed its digest but does not load (another
            // driver, a damaged entry): compiled again once, without the cache
            e->recompiled = true;
            e->state = JitEntry::kCompiling;
            g_threads.emplace_back(compile_entry, e, arch, k, n, false);
            if (!wait) return nullptr;
            g_cv.wait(g, [&] { return e->state != JitEntry::kCompiling; });
            if (e->state == JitEntry::kReady) {
                g.unlock();
                return jit_encoder(k, n, false, false);
            }
        }
        fprintf(stderr, "uplink_ec: loading the RS(%d,%d) encoder failed\n", k, n);
        e->state = JitEntry::kFailed;
        return nullptr;
    }
    e->modules[dev] = mod;
    std::unique_ptr<EncoderKernel> ek(new EncoderKernel());
    ek->k = k;
    ek->n = n;
    ek->jit = true;
    const int pnc = enc::parity_compute_waves(k, n), fnc = enc::full_compute_waves(k, n),
              fnl = enc::full_loader_waves(k, n);
    ek->full = {nullptr, f_full, (fnc + fnl) * 64, enc::wgs_per_cu(k, fnc + fnl), "rs_encode_special (jit)"};
    const int pnl = enc::loader_waves(k, n);
    ek->parity = {nullptr, f_par, (pnc + pnl) * 64, enc::wgs_per_cu(k, pnc + pnl), "rs_encode_special (jit, parity only)"};
    EncoderKernel *out = ek.get();
    e->loaded[dev] = std::move(ek);
    return out;
}

// Run-time compilation is worth it up to k = 48 inputs: measured against the
// runtime-matrix kernel (tools/bench_jit.py) the compiled
// encoder is 10-25 % faster there, while at k = 56-64 the two-chunk body is no
// faster and takes a minute of hiprtc time.
constexpr int kJitMaxK = 48;

// UPLINK_EC_JIT=0: no run-time compilation at all (library-built encoders and
// the runtime-matrix kernel only).  Otherwise a compile starts only for a
// caller that asks for it (find_encoder's `start`: whole-segment launches of
// at least kJitMinTiles tiles, and ec_prepare_encoder), never for per-stripe
// work, which the runtime-matrix kernel serves at the same speed; a process
// that started one waits at exit for the one in progress (join_compiles).
bool jit_allowed() {
    static const bool on = [] {
        const char *e = getenv("UPLINK_EC_JIT");
        return !(e && e[0] == '0' && e[1] == 0);
    }();
    return on;
}

const EncoderKernel *find_encoder(int k, int n, bool wait, bool start) {
    if (const EncoderKernel *e = aot_encoder(k, n)) return e;
    if (!enc::supported(k, n) || k > kJitMaxK || !jit_allowed()) return nullptr;
    return jit_encoder(k, n, wait, start || wait);
}

hipError_t launch_encode_special(const EncoderKernel &e, const RsArgs &args, int grid, hipStream_t s) {
    const bool parity_only = args.copy_off[0] < 0;
    const EncoderKernel::Variant &v = parity_only ? e.parity : e.full;
    if (grid <= 0) grid = default_grid((args.total_blocks + 1) / 2, v.wgs_per_cu);  // tiles = pairs of blocks
    RsArgs a = args;
    void *params[] = {&a};
    if (v.aot) return hipLaunchKernel(v.aot, dim3(grid), dim3(v.threads), params, 0, s);
    return hipModuleLaunchKernel(v.jit, grid, 1, 1, v.threads, 1, 1, 0, s, params, nullptr);
}

}  // namespace uplink_ec
