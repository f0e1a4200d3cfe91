// Wall time of one hiprtc compile of a run-time encoder (RS(k,n), NC compute
// waves, both variants), as rs_encoder_registry.cpp compiles it: on the GPU box
// vs this container.  tools/exp/jit_time K N NC [opts].
#include <hip/hiprtc.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "../../uplink_amd/csrc/rs_jit_sources.inc"
int main(int argc, char **argv) {
    int k = atoi(argv[1]), n = atoi(argv[2]), nc = atoi(argv[3]), nl = 4;
    std::vector<std::string> opts = {"--offload-arch=gfx950", "-O3", "-std=c++20"};
    for (int i = 4; i < argc; i++) opts.push_back(argv[i]);
    auto expr = [&](bool copy) { return "&uplink_ec::enc::rs_encode_special<" + std::to_string(k) + ", " + std::to_string(n) + ", " + std::to_string(nc) + ", " + std::to_string(nl) + (copy ? ", true>" : ", false>"); };
    std::string full = expr(true), par = expr(false);
    auto t0 = std::chrono::steady_clock::now();
    hiprtcProgram prog;
    hiprtcCreateProgram(&prog, "#include \"rs_encoder.hpp\"\n", "x.hip", kJitHeaderCount, kJitHeaderTexts, kJitHeaderNames);
    hiprtcAddNameExpression(prog, full.c_str());
    hiprtcAddNameExpression(prog, par.c_str());
    std::vector<const char *> o; for (auto &s : opts) o.push_back(s.c_str());
    hiprtcResult r = hiprtcCompileProgram(prog, (int)o.size(), o.data());
    size_t sz = 0; hiprtcGetCodeSize(prog, &sz);
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("RS(%d,%d) nc %d: rc %d, %zu B, %.1f s\n", k, n, nc, (int)r, sz, s);
    if (r) { size_t nlg; hiprtcGetProgramLogSize(prog, &nlg); std::string lg(nlg, 0); hiprtcGetProgramLog(prog, &lg[0]); printf("%s\n", lg.c_str()); }
}
