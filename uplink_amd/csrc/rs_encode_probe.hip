// The RS(29,80) encoder's own memory schedule without its arithmetic, built
// into the library for the bench line's on-box ceiling:
// encode_body<..., kDiagNoRowOps> (rs_encoder.hpp) is the product body with
// the multiply-accumulate removed -- the same LDS-DMA loaders, 2-slot LDS ring,
// tile queue, bit-slicing, copy-through stores, un-slicing and parity stores,
// the compute waves reading every input's planes from the LDS and keeping them
// live, and storing the tile's last input in place of each parity row (so the
// stored bytes are as random as the real ones).  Its rate is what the
// encoder's access pattern moves on the box with no GF arithmetic issued.
#include <hip/hip_runtime.h>

#include "rs_encoder.hpp"
#include "rs_kernels.hpp"

namespace uplink_ec {
namespace enc {

template <int K, int N, int NC, int NL, bool COPY>
__global__ __launch_bounds__((NC + NL) * 64, UPLINK_ENC_WGS > 1 ? (NC + NL) * UPLINK_ENC_WGS / 4 : 1) void rs_encode_shape(
    const RsArgs a) {
    encode_body<K, N, NC, NL, COPY, kDiagNoRowOps>(a);
}

}  // namespace enc

const EncoderKernel *shape_probe_encoder(int k, int n) {
    if (k != 29 || n != 80) return nullptr;
    static const EncoderKernel e = [] {
        constexpr int K = 29, N = 80;
        constexpr int PNC = enc::parity_compute_waves(K, N), FNC = enc::full_compute_waves(K, N);
        constexpr int FNL = enc::full_loader_waves(K, N), PNL = enc::loader_waves(K, N);
        EncoderKernel x;
        x.k = K;
        x.n = N;
        x.full = {reinterpret_cast<const void *>(&enc::rs_encode_shape<K, N, FNC, FNL, true>), nullptr,
                  (FNC + FNL) * 64, enc::wgs_per_cu(K, FNC + FNL), "rs_encode_shape (library)"};
        x.parity = {reinterpret_cast<const void *>(&enc::rs_encode_shape<K, N, PNC, PNL, false>), nullptr,
                    (PNC + PNL) * 64, enc::wgs_per_cu(K, PNC + PNL), "rs_encode_shape (library, parity only)"};
        return x;
    }();
    return &e;
}

}  // namespace uplink_ec
