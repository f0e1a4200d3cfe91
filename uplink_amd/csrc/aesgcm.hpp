// AES-256-GCM segment encryption on the GPU: host-side
// key preparation and launch entry points used by the C-ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace uplink_ec {

// Per-key device data: the AES-256 round keys and 4-bit GHASH tables of
// H^1..H^64 (H = AES_K(0^128)), all words big-endian as GCM defines them.
struct GcmSched {
    uint32_t rk[60];
    uint32_t pad_[4];
    uint32_t htab[64][16][4];  // htab[p][nibble] = nibble * H^(p+1) (Shoup's 4-bit table)
    uint32_t h64_8[256][4];    // byte * H^64 (the 8-bit table of the Horner multiplier)
};

// Fills `out` with the schedule of a 32-byte key (host memory).
void gcm_prepare(const uint8_t key[32], GcmSched *out);

// One batch: nseg segments of nblocks GCM blocks each.  Block b of segment g
// is read from in + g*in_seg_stride + b*in_blk_stride (in_block plaintext
// bytes to seal, or in_block ciphertext bytes + 16-byte tag to open) and
// written to out + g*out_seg_stride + b*out_blk_stride (ciphertext || tag, or
// plaintext).  Its nonce is nonces[12*g..] + b (little-endian increment of
// the 12 bytes).  status[g] (open only, initialised by the launcher) ends as
// the first block of segment g whose tag did not verify, or -1.
struct GcmBatch {
    const uint8_t *in;
    uint8_t *out;
    int64_t in_seg_stride, out_seg_stride;
    int64_t in_blk_stride, out_blk_stride;
    const GcmSched *sched;  // [nseg] device
    const uint8_t *nonces;  // [nseg][12] device
    int32_t *status;        // [nseg] device (open)
    uint32_t nseg, nblocks, in_block;
};

hipError_t gcm_launch(const GcmBatch &b, bool open, hipStream_t stream);

// AES-256 of one block on the host (key setup and tests)
void aes256_encrypt_block(const uint32_t rk[60], const uint8_t in[16], uint8_t out[16]);

}  // namespace uplink_ec
