// Launch entry points of the GF(2^8) Reed-Solomon stripe kernels (encode K1,
// rebuild K2 in SURVEY.md §2).  Host-only header: no torch types, plain
// pointers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "rs_args.hpp"

namespace uplink_ec {

// A compile-time-G encoder of one (k, n) (rs_encoder.hpp): built into the
// library for the configurations listed in rs_encoder_registry.cpp, compiled
// with hiprtc for any other (k, n) on first use and cached on disk
// (rs_encoder_jit.cpp).  Two variants: all n pieces, and parity only.
struct EncoderKernel {
    struct Variant {
        const void *aot = nullptr;       // host stub of a library kernel
        hipFunction_t jit = nullptr;     // function of a run-time module
        int threads = 0;                 // workgroup size
        int wgs_per_cu = 1;
        const char *name = "";
    };
    int k = 0, n = 0;
    bool jit = false;
    Variant full, parity;
};

// The encoder for (k, n) on the current device, or nullptr when (k, n) is
// outside the compile-time encoder's limits, its run-time compilation is not
// done (or failed), or -- `start` false -- has not been started (the caller
// then uses the runtime-matrix kernel).  A compilation is started only for a
// caller that passes `start` (launches large enough to pay for it, and
// ec_prepare_encoder); `wait` blocks until it is done.  Thread-safe.
const EncoderKernel *find_encoder(int k, int n, bool wait = false, bool start = true);
// Library-built encoders (rs_encoder_registry.cpp); nullptr if none.
const EncoderKernel *aot_encoder(int k, int n);
// RS(29,80)'s encoder without its arithmetic (rs_encode_probe.hip): the
// on-box ceiling of the encoder's own access pattern; nullptr for other codes.
const EncoderKernel *shape_probe_encoder(int k, int n);
// The same limits find_encoder applies (no compilation).
bool encoder_supported(int k, int n);
hipError_t launch_encode_special(const EncoderKernel &e, const RsArgs &args, int grid, hipStream_t stream);

// Runtime-matrix kernel: args.coef / nin / nout with the leaf addresses of
// that matrix in args.jt_tgt (made by launch_jt_targets into
// jt_targets_bytes(args) bytes of device memory; required).
hipError_t launch_matmul_generic(const RsArgs &args, int grid, hipStream_t stream);
// The same kernel calling a plan's straight-line segments (rs_sl.hpp):
// args.jt_tgt = their absolute addresses, [pass][chunk][group].
hipError_t launch_matmul_sl(const RsArgs &args, int grid, hipStream_t stream);
// Prefetch depth of the straight-line rebuild (chunks of input shares in flight
// by LDS-DMA; 0 = the register-staged kernel), set by ec_create.
void configure_rebuild(int depth);
size_t jt_targets_bytes(const RsArgs &args);
hipError_t launch_jt_targets(const RsArgs &args, uint64_t *targets, hipStream_t stream);
// Byte-wise fallback (any ess, any alignment); coef as above.
hipError_t launch_matmul_bytes(const RsArgs &args, hipStream_t stream);
// out[r] (bs bytes) = share nums[r] of stripe r: stripes [nreq][k][bs],
// parity pieces [n-k][nreq*bs] (batched EncodeSingle)
hipError_t launch_gather_shares(const uint8_t *stripes, const uint8_t *parity, const int *nums, int k, int64_t nreq,
                               int64_t bs, uint8_t *out, hipStream_t stream);

// Default grid (workgroups) for a launch over `total_tiles` tiles.
int default_grid(int64_t total_tiles, int wgs_per_cu);
int cu_count();

}  // namespace uplink_ec
