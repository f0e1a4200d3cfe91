// One library-built compile-time-G encoder, RS(UPLINK_AOT_K, UPLINK_AOT_N):
// the Makefile compiles this file once per line of rs_encoder_aot.def, in
// parallel, and rs_encoder_registry.cpp lists the results.
#include <hip/hip_runtime.h>

#include "rs_encoder.hpp"
#include "rs_kernels.hpp"

#define UPLINK_STR2(x) #x
#define UPLINK_STR(x) UPLINK_STR2(x)
#define UPLINK_AOT_NAME2(K, N) aot_encoder_##K##_##N
#define UPLINK_AOT_NAME(K, N) UPLINK_AOT_NAME2(K, N)

namespace uplink_ec {

EncoderKernel UPLINK_AOT_NAME(UPLINK_AOT_K, UPLINK_AOT_N)() {
    constexpr int K = UPLINK_AOT_K, N = UPLINK_AOT_N;
    static_assert(enc::supported(K, N), "outside the compile-time encoder's limits");
    constexpr int PNC = enc::parity_compute_waves(K, N), FNC = enc::full_compute_waves(K, N);
    static_assert(FNC == 4, "library-built configurations use the 4 + 4 full encoder (its kernel name below)");
    EncoderKernel e;
    e.k = K;
    e.n = N;
    e.full = {reinterpret_cast<const void *>(&enc::rs_encode_special<K, N, FNC, 4>), nullptr, (FNC + 4) * 64,
              enc::wgs_per_cu(K), "rs_encode_special<" UPLINK_STR(UPLINK_AOT_K) "," UPLINK_STR(UPLINK_AOT_N) ",4,4>"};
    e.parity = {reinterpret_cast<const void *>(&enc::rs_encode_special<K, N, PNC, 4>), nullptr, (PNC + 4) * 64,
                enc::wgs_per_cu(K),
                PNC == 8 ? "rs_encode_special<" UPLINK_STR(UPLINK_AOT_K) "," UPLINK_STR(UPLINK_AOT_N) ",8,4>"
                         : "rs_encode_special<" UPLINK_STR(UPLINK_AOT_K) "," UPLINK_STR(UPLINK_AOT_N) ",4,4>"};
    return e;
}

}  // namespace uplink_ec
