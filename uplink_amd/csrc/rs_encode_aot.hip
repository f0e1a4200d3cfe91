// One library-built compile-time-G encoder, RS(UPLINK_AOT_K, UPLINK_AOT_N):
// the Makefile compiles this file once per line of rs_encoder_aot.def, in
// parallel, and rs_encoder_registry.cpp lists the results.
#include <hip/hip_runtime.h>

#include "rs_encoder.hpp"
#include "rs_kernels.hpp"

#define UPLINK_AOT_NAME2(K, N) aot_encoder_##K##_##N
#define UPLINK_AOT_NAME(K, N) UPLINK_AOT_NAME2(K, N)

namespace uplink_ec {

EncoderKernel UPLINK_AOT_NAME(UPLINK_AOT_K, UPLINK_AOT_N)() {
    constexpr int K = UPLINK_AOT_K, N = UPLINK_AOT_N;
    static_assert(enc::supported(K, N), "outside the compile-time encoder's limits");
    constexpr int PNC = enc::parity_compute_waves(K, N), FNC = enc::full_compute_waves(K, N);
    constexpr int FNL = enc::full_loader_waves(K, N), PNL = enc::loader_waves(K, N);
    EncoderKernel e;
    e.k = K;
    e.n = N;
    e.full = {reinterpret_cast<const void *>(&enc::rs_encode_special<K, N, FNC, FNL, true>), nullptr, (FNC + FNL) * 64,
              enc::wgs_per_cu(K, FNC + FNL), "rs_encode_special (library)"};
    e.parity = {reinterpret_cast<const void *>(&enc::rs_encode_special<K, N, PNC, PNL, false>), nullptr, (PNC + PNL) * 64,
                enc::wgs_per_cu(K, PNC + PNL), "rs_encode_special (library, parity only)"};
    return e;
}

}  // namespace uplink_ec
