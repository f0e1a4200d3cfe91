/*
 * uplink_ec.h — C ABI of the MI355X erasure-coding engine that replaces the
 * Reed-Solomon stripe loop of storj/uplink's private/eestream (+ the piece
 * fan-out of private/ecclient).  Plain pointers and sizes only; every compute
 * entry point runs on the GPU (HIP, gfx950).  There is no CPU fallback: if no
 * GPU is usable, ec_create returns EC_ERR_DEVICE.
 *
 * Reference interface each export replaces (storj/uplink @ /root/reference):
 *
 *   ec_create / ec_destroy   eestream.NewFEC + eestream.NewRSScheme
 *                            private/eestream/fec.go:15-17, rs.go:17-19
 *                            (called from encode.go:69-87)
 *   ec_required/total/share_size/stripe_size
 *                            ErasureScheme.RequiredCount/TotalCount/
 *                            ErasureShareSize/StripeSize   rs.go:47-61
 *   ec_encode_single         ErasureScheme.EncodeSingle    scheme.go:18, rs.go:21-23
 *                            (caller segmentupload/encode.go:58, eestream/encode.go:187)
 *   ec_encode                ErasureScheme.Encode          scheme.go:15, rs.go:25-30
 *   ec_rebuild               ErasureScheme.Rebuild         scheme.go:26, rs.go:40-45
 *                            (caller stripe.go:410-412)
 *   ec_decode                ErasureScheme.Decode          scheme.go:22, rs.go:32-38
 *                            (caller stripe.go:407-408; layout unsafe_rs.go:38-46)
 *   ec_encode_segments       batch form of EncodeSingle over every (piece, stripe)
 *                            of whole segments: segmentupload/encode.go:39-75 driven
 *                            by single.go:228-238 (pieceReader.PieceReader)
 *   ec_rebuild_segments      batch form of the per-stripe Rebuild loop of
 *                            StripeReader.ReadStripes  stripe.go:382-428
 *   ec_*_segments_sets       the same for many segments with a share set each:
 *                            one StripeReader per download, ecclient/client.go:273-308
 *   ec_*_segments_host       the same batches from/to host memory (PCIe pipeline)
 *   ec_*blake3* / ec_hash_segments / ec_encode_segments_host_hashed
 *                            BLAKE3 piece hash of the upload (piecestore/upload.go:
 *                            133,155,270; hash.go:20-26), SURVEY §8f row 4
 *   ec_gcm_*                 AES-256-GCM segment encryption: splitter/splitter.go:156,170
 *                            (upload), streams/store.go:347-382 (download), SURVEY §8f row 4
 *   ec_strerror/ec_format_error  error texts of infectious / eestream
 *
 * Error codes map to the errors eestream's callers test:
 *   EC_ERR_NUM_NEGATIVE  "num must be non-negative"   (segmentupload/encode_test.go:53)
 *   EC_ERR_NUM_RANGE     "num must be less than %d"   (segmentupload/encode_test.go:63)
 *   EC_ERR_NOT_ENOUGH_SHARES  infectious.NotEnoughShares (stripe.go:446-449)
 *   EC_ERR_TOO_MANY_ERRORS    infectious.TooManyErrors   (stripe.go:446-449)
 *
 * Threading: an ec_ctx is immutable after ec_create except for internal
 * caches guarded by a mutex; every export is reentrant (uplink calls
 * EncodeSingle from up to 300 goroutines, private/testuplink/uplink.go:83).
 * No pointer passed in is retained after a call returns (cgo rules);
 * the *_segments calls are asynchronous on `stream` and the caller keeps the
 * device buffers alive until the stream is synchronised.
 */
#ifndef UPLINK_EC_H
#define UPLINK_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EC_OK 0
#define EC_ERR_PARAMS (-1)            /* "requires 1 <= k <= n <= 256" */
#define EC_ERR_NUM_NEGATIVE (-2)      /* "num must be non-negative" */
#define EC_ERR_NUM_RANGE (-3)         /* "num must be less than %d" (n) */
#define EC_ERR_INPUT_LENGTH (-4)      /* "input length must be a multiple of %d" (k) */
#define EC_ERR_OUTPUT_LENGTH (-5)     /* "output length must be %d" */
#define EC_ERR_NOT_ENOUGH_SHARES (-6) /* infectious.NotEnoughShares */
#define EC_ERR_TOO_MANY_ERRORS (-7)   /* infectious.TooManyErrors */
#define EC_ERR_INVALID_SHARE (-8)     /* "invalid share id: %d" */
#define EC_ERR_SINGULAR (-9)          /* decode matrix not invertible */
#define EC_ERR_INVALID_ARG (-10)      /* null pointer / bad size / layout */
#define EC_ERR_DEVICE (-11)           /* HIP runtime error or no GPU */
#define EC_ERR_UNSUPPORTED (-12)      /* outside the engine's limits */
#define EC_ERR_SHARE_SIZE (-13)       /* shares of different lengths */
#define EC_ERR_AUTH (-14)             /* "cipher: message authentication failed" (a GCM tag did not verify) */

/* flags for ec_encode_segments */
#define EC_FLAG_PARITY_ONLY 0x1 /* write only the n-k parity pieces */
#define EC_FLAG_HASH_PIECES 0x2 /* ec_upload_begin: also the BLAKE3 of every piece (ec_upload_hashes) */

typedef struct ec_ctx ec_ctx;
typedef void *ec_stream; /* hipStream_t; NULL = the default stream */

int ec_create(int k, int n, int erasure_share_size, ec_ctx **out);
/* Every streamed upload (ec_upload_begin) of the context must have ended
 * (ec_upload_end) before ec_destroy; launches still queued on callers' streams
 * are waited for. */
void ec_destroy(ec_ctx *ctx);

int ec_required(const ec_ctx *ctx);
int ec_total(const ec_ctx *ctx);
int ec_share_size(const ec_ctx *ctx);
int ec_stripe_size(const ec_ctx *ctx);
/* copies the n x k generator matrix (row-major) into out (n*k bytes) */
int ec_generator(const ec_ctx *ctx, uint8_t *out);

const char *ec_strerror(int code);
/* message with the %d filled from ctx (n for NUM_RANGE, k for INPUT_LENGTH,
 * `arg` for OUTPUT_LENGTH / INVALID_SHARE); returns the message length */
int ec_format_error(const ec_ctx *ctx, int code, long long arg, char *buf, size_t len);

/* ---- ErasureScheme surface: host buffers, synchronous, GPU-computed ---- */

/* out (len(in)/k bytes) = erasure share `num` of the stripe `in` */
int ec_encode_single(const ec_ctx *ctx, const uint8_t *in, size_t in_len, uint8_t *out, size_t out_len, int num);
/* all n shares of `in`: share i written to out + i*(in_len/k) */
int ec_encode(const ec_ctx *ctx, const uint8_t *in, size_t in_len, uint8_t *out);
/* Rebuild: `nums` (nshares entries) is sorted in place together with
 * `shares`, exactly as infectious sorts its []Share; the k data shares are
 * written to out + i*share_len. */
int ec_rebuild(const ec_ctx *ctx, int nshares, int *nums, const uint8_t **shares, size_t share_len, uint8_t *out);
/* Decode: Correct (Berlekamp-Welch when nshares > k) + Rebuild; `shares`
 * are corrected in place like infectious' share.Data.  out = k*share_len. */
int ec_decode(const ec_ctx *ctx, int nshares, int *nums, uint8_t **shares, size_t share_len, uint8_t *out);

/* ---- batched, device-resident (HIP device pointers), async on stream ---- */

/* segs: nseg padded segments, each nstripes*k*ess bytes, stripe-major
 *       [stripe][k][ess] (the PadReader output of single.go:234-236).
 * pieces: [nseg][n][nstripes*ess]  (or [nseg][n-k][...] with
 *       EC_FLAG_PARITY_ONLY).  Piece i of a segment = the concatenation of
 *       EncodeSingle(stripe, num=i) over its stripes. */
int ec_encode_segments(const ec_ctx *ctx, const uint8_t *segs, size_t nseg, size_t nstripes, uint8_t *pieces,
                       int flags, ec_stream stream);
/* Rebuild whole segments from nshares >= k pieces (each nstripes*ess bytes,
 * device pointers in `pieces`, piece numbers in `nums`, any order).  The
 * share choice follows infectious Rebuild; out = nstripes*k*ess bytes,
 * stripe-major.  nseg segments may be batched with strides (in bytes,
 * 0 when nseg == 1). */
int ec_rebuild_segments(const ec_ctx *ctx, int nshares, const int *nums, const uint8_t *const *pieces,
                        size_t nstripes, uint8_t *out, ec_stream stream);
int ec_rebuild_segments_batched(const ec_ctx *ctx, int nshares, const int *nums, const uint8_t *const *pieces,
                                size_t nstripes, size_t nseg, long long piece_seg_stride, long long out_seg_stride,
                                uint8_t *out, ec_stream stream);
/* Decode whole segments with error detection: FEC.Decode (Correct +
 * Rebuild) on every stripe of the pieces at once -- what StripeReader runs
 * per stripe when error detection is on (private/eestream/stripe.go:407-408
 * -> rsScheme.Decode, rs.go:32-38).  Same arguments as ec_rebuild_segments;
 * with nshares > k every column is checked against the code (syndrome rows
 * computed and tested for zero inside the kernel, nothing stored) and, where
 * a column is not a codeword, corrected by Berlekamp-Welch.  Corrected
 * shares are written back into the caller's pieces, as infectious corrects
 * share.Data in place.  The check and the rebuild are one pass over the shares
 * (the rebuilt rows stored, the syndrome rows tested in the same kernel); a
 * segment with errors is then corrected and rebuilt again on its own.  Returns
 * when done (the check's outcome is read back), also when nshares == k:
 * EC_ERR_TOO_MANY_ERRORS / EC_ERR_NOT_ENOUGH_SHARES as Decode returns them.
 * Every share given is checked and corrected, as infectious' Correct uses
 * them all: of more than 128 (n > 128), the first 128 in number order go
 * through the one-pass check and the syndromes of the rest are checked in
 * further launches of up to 128 - k at a time. */
int ec_decode_segments(const ec_ctx *ctx, int nshares, const int *nums, uint8_t *const *pieces, size_t nstripes,
                       uint8_t *out, ec_stream stream);
/* The same over nseg segments in one check and one rebuild launch (strides as
 * ec_rebuild_segments_batched); a segment with errors is corrected on its own. */
int ec_decode_segments_batched(const ec_ctx *ctx, int nshares, const int *nums, uint8_t *const *pieces,
                               size_t nstripes, size_t nseg, long long piece_seg_stride, long long out_seg_stride,
                               uint8_t *out, ec_stream stream);

/* ---- a share set per segment (the download path as uplink runs it) ----
 * Every segment a download fetches is decoded from whichever k (or more)
 * pieces arrived first (StripeReader, private/eestream/stripe.go:314-354,
 * via ecclient GetWithOptions, private/ecclient/client.go:273-308, one per
 * segment, several at once under prefetch, private/storage/streams/
 * store.go:240-253,385-403): share sets are almost never repeated.  These
 * calls take nseg segments, each with its own set, in one pass: segment g's
 * shares are entries [off_g, off_g + nshares[g]) of nums / pieces (off_g the
 * sum of the nshares before it; device pointers, nstripes*ess bytes each, any
 * order), its output outs[g] (nstripes*k*ess bytes, stripe-major).  The share
 * choice is infectious Rebuild's per segment.  The decode rows of every
 * segment are solved on the GPU in stream order; the host only chooses the
 * shares (no synchronisation, no plan, no code generation on the call path).
 * A Rebuild of one segment (up to 64 shares) is one launch whose decode rows
 * the host solves and passes in the launch's arguments.
 *
 * ec_rebuild_segments_sets: Rebuild (stripe.go:410-412); async on stream. */
int ec_rebuild_segments_sets(const ec_ctx *ctx, size_t nseg, const int *nshares, const int *nums,
                             const uint8_t *const *pieces, size_t nstripes, uint8_t *const *outs, ec_stream stream);
/* Decode with error detection (stripe.go:407-408 -> rs.go:32-38) over the
 * same layout: one pass reads every share of every segment, stores the rebuilt
 * data and checks each segment's syndromes; a segment with errors is then
 * corrected in its pieces and rebuilt as ec_decode_segments does.  Returns
 * when done.  Segments of more than 128 shares go through ec_decode_segments. */
int ec_decode_segments_sets(const ec_ctx *ctx, size_t nseg, const int *nshares, const int *nums,
                            uint8_t *const *pieces, size_t nstripes, uint8_t *const *outs, ec_stream stream);
/* ec_rebuild_segments[_batched] with a share set the context has no
 * straight-line code for runs the share-set pass and has the code made in the
 * background (DESIGN.md §4 "Straight-line rebuild bodies"); later launches of
 * the set use it.  This queues that for (nshares, nums) ahead of time; with
 * wait != 0 it returns after it is made.  Returns 1 when the code is ready, 0
 * when not (or the set has none: every data share present).  No reference
 * counterpart (an engine knob). */
int ec_prepare_rebuild(const ec_ctx *ctx, int nshares, const int *nums, int wait);

/* ---- host-memory pipeline (end-to-end path, PCIe-inclusive) ----
 * Same layouts as the device calls, but in host memory (pinned memory from
 * ec_host_alloc gives full-speed DMA).  Segments are streamed through a ring
 * of device slots on 3 HIP streams so H2D, kernel and D2H of consecutive
 * segments overlap; synchronous (returns when every piece is in host memory).
 * This is the form the Go side calls from segmentupload (SegmentEncoder,
 * single.go:233-238) and StripeReader (BatchRebuilder, stripe.go:382-428). */
int ec_encode_segments_host(const ec_ctx *ctx, const uint8_t *segs, size_t nseg, size_t nstripes, uint8_t *pieces,
                            int flags);
/* pieces[i]: host pointer of share nums[i] for segment 0; segment g's copy of
 * that share is at pieces[i] + g*piece_seg_stride. out: [nseg][stripes*k*ess] */
int ec_rebuild_segments_host(const ec_ctx *ctx, int nshares, const int *nums, const uint8_t *const *pieces,
                             size_t nstripes, size_t nseg, long long piece_seg_stride, uint8_t *out);
/* ec_encode_segments_host + the BLAKE3-256 hash of every piece (all n, also
 * with EC_FLAG_PARITY_ONLY): hashes = [nseg][n][32] host bytes, the value
 * piecestore's upload sends as PieceHash.Hash (piecestore/upload.go:133,155,270)
 * when the piece hash algorithm is BLAKE3 (the default, piecestore/hash.go:20-26). */
int ec_encode_segments_host_hashed(const ec_ctx *ctx, const uint8_t *segs, size_t nseg, size_t nstripes,
                                   uint8_t *pieces, uint8_t *hashes, int flags);
/* Streamed form for one segment, for piece readers that serve each piece
 * stripe by stripe as the reference does (segmentupload/encode.go:39-75,
 * pieceReader.PieceReader single.go:228-238): the segment goes through the
 * engine in chunks of stripes (chunk_stripes, or 0 for the library's choice:
 * 128 stripes first, doubling up to 2048) and each chunk of every piece is in
 * `pieces` (host, [rows][nstripes*ess] as ec_encode_segments_host) as soon as
 * it is encoded.  ec_upload_begin queues everything and returns;
 * ec_upload_wait blocks until stripes [0, stripes) of every piece are in host
 * memory; ec_upload_ready returns how many leading stripes are, without
 * blocking; ec_upload_end waits for the rest, frees the handle and returns the
 * first error.  The caller keeps seg and pieces alive until ec_upload_end.
 * With EC_FLAG_HASH_PIECES the BLAKE3-256 of all n pieces (also with
 * EC_FLAG_PARITY_ONLY) is computed as the chunks stream, as piecestore's
 * upload hashes each piece through a TeeReader (piecestore/upload.go:155,
 * 262-270); ec_upload_hashes waits for them (the last chunk's tree fold) and
 * copies n*32 bytes into `hashes`.  Any number of threads may be inside
 * ec_upload_wait / _ready / _hashes at once; ec_upload_end waits for those
 * inside to return before it frees the handle, and no call may start on a
 * handle once ec_upload_end has been called (callers arriving while it waits
 * get EC_ERR_INVALID_ARG / 0). */
typedef struct ec_upload ec_upload;
int ec_upload_begin(const ec_ctx *ctx, const uint8_t *seg, size_t nstripes, uint8_t *pieces, int flags,
                    size_t chunk_stripes, ec_upload **out);
int ec_upload_wait(ec_upload *u, size_t stripes);
size_t ec_upload_ready(ec_upload *u);
int ec_upload_hashes(ec_upload *u, uint8_t *hashes);
int ec_upload_end(ec_upload *u);
void *ec_host_alloc(size_t bytes); /* pinned (hipHostMalloc); NULL on failure */
void ec_host_free(void *p);
/* Device memory on the current device for the device-pointer calls (the
 * share-set calls' pieces and outputs; a Go binding has no other allocator),
 * and a synchronous copy between any two of host / pinned / device memory. */
void *ec_device_alloc(size_t bytes); /* hipMalloc; NULL on failure */
void ec_device_free(void *p);
int ec_copy(void *dst, const void *src, size_t bytes); /* hipMemcpy(hipMemcpyDefault) */

/* ---- BLAKE3-256 piece hashes (github.com/zeebo/blake3 v0.2.3, go.mod:29) ----
 * Replace the per-piece hash.Hash fed by io.TeeReader during upload
 * (piecestore/upload.go:133 NewHashFromAlgorithm, :155 TeeReader, :270
 * Sum(nil)); 32-byte digests, BLAKE3 hash mode, no key. */

/* Device pieces: byte t of piece j is at
 *   base + j*piece_stride + (t / run)*run_stride + t % run
 * (run = piece_len or 0 for contiguous pieces).  hashes: npieces*32 device
 * bytes.  Async on stream (scratch from hipMallocAsync on that stream). */
int ec_blake3_pieces(const uint8_t *base, size_t npieces, long long piece_stride, size_t piece_len, size_t run,
                     long long run_stride, uint8_t *hashes, ec_stream stream);
/* Every piece of nseg segments already on the device: data piece j of
 * segment s is share j of each stripe of segs + s*nstripes*k*ess; parity
 * piece k+r is parity + (s*(n-k) + r)*nstripes*ess (the EC_FLAG_PARITY_ONLY
 * output).  hashes: [nseg][n][32] device bytes.  Async on stream. */
int ec_hash_segments(const ec_ctx *ctx, const uint8_t *segs, const uint8_t *parity, size_t nseg, size_t nstripes,
                     uint8_t *hashes, ec_stream stream);
/* Host buffers, synchronous: hashes[32*j] = BLAKE3(data + j*stride, piece_len) */
int ec_blake3_host(const uint8_t *data, size_t npieces, long long stride, size_t piece_len, uint8_t *hashes);

/* ---- AES-256-GCM segment encryption (storj.io/common/encryption, EncAESGCM) ----
 * Replace encryption.TransformWriterPadded(buf, NewEncrypter(EncAESGCM, key,
 * nonce, BlockSize)) on upload (splitter/splitter.go:156,170) and
 * Transform(rr, NewDecrypter(...)) on download (streams/store.go:354-377):
 * blocks of in_block = BlockSize - 16 plaintext bytes (7408 for BlockSize
 * 29*256, project.go:84), block b sealed under the 12-byte nonce + b
 * (little-endian increment, as calcGCMNonce), written as ciphertext || tag.
 * Padding of the plaintext (PadReader rule) and Unpad are the caller's.
 * in_block must be a multiple of 16, buffers 16-byte aligned. */

/* device bytes of one prepared key */
size_t ec_gcm_key_bytes(void);
/* expands nkeys 32-byte keys (host) into dev_keys (nkeys * ec_gcm_key_bytes()
 * device bytes): round keys + GHASH tables; synchronous */
int ec_gcm_prepare_keys(const uint8_t *keys, size_t nkeys, void *dev_keys, ec_stream stream);
/* plain: [nseg][nblocks*in_block] -> out: [nseg][nblocks*(in_block+16)];
 * segment g uses prepared key g and nonce dev_nonces[12*g..]; async */
int ec_gcm_seal_segments(const uint8_t *plain, size_t nseg, size_t nblocks, size_t in_block, const void *dev_keys,
                         const uint8_t *dev_nonces, uint8_t *out, ec_stream stream);
/* the inverse; dev_status[g] = -1 when every block of segment g verified,
 * else the first block whose tag did not (its plaintext must not be used) */
int ec_gcm_open_segments(const uint8_t *cipher, size_t nseg, size_t nblocks, size_t in_block, const void *dev_keys,
                         const uint8_t *dev_nonces, uint8_t *out, int32_t *dev_status, ec_stream stream);
/* the same with explicit segment strides in bytes (multiples of 16, at least
 * the dense size), e.g. to seal straight into the RS encoder's padded input */
int ec_gcm_seal_segments_strided(const uint8_t *plain, long long plain_seg_stride, size_t nseg, size_t nblocks,
                                 size_t in_block, const void *dev_keys, const uint8_t *dev_nonces, uint8_t *out,
                                 long long out_seg_stride, ec_stream stream);
int ec_gcm_open_segments_strided(const uint8_t *cipher, long long cipher_seg_stride, size_t nseg, size_t nblocks,
                                 size_t in_block, const void *dev_keys, const uint8_t *dev_nonces, uint8_t *out,
                                 long long out_seg_stride, int32_t *dev_status, ec_stream stream);
/* PadReader padding (single.go:236) on the device: after
 * data_len bytes of each of nseg segments (seg_stride apart) write
 * p = 4 + (block - (data_len+4) % block) % block bytes of byte(p), the last
 * four the big-endian uint32 p.  Async on stream. */
int ec_pad_segments(uint8_t *segs, size_t nseg, long long seg_stride, size_t data_len, size_t block, ec_stream stream);
/* host buffers, one segment, synchronous; open returns EC_ERR_AUTH and the
 * first failing block in *bad_block when a tag does not verify */
int ec_gcm_seal_host(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *plain, size_t nblocks,
                     size_t in_block, uint8_t *out);
int ec_gcm_open_host(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *cipher, size_t nblocks,
                     size_t in_block, uint8_t *out, long long *bad_block);

/* ---- on-box ceilings (the bench's roofline context; no reference counterpart) ----
 * A plain streaming kernel, no arithmetic, in the read:write mix of an erasure
 * kernel: each wave reads R KiB of src and writes W KiB to dst, one-shot grid,
 * 16 B per lane per access (DESIGN.md §4 HBM table).  dst must hold
 * read_bytes * W / R bytes.  *moved = the bytes read + written.  Async. */
#define EC_PROBE_COPY 0       /* 1 : 1     (the rebuild) */
#define EC_PROBE_ENCODE_MIX 1 /* 4 : 11    (the full encode's 29 : 80) */
#define EC_PROBE_PARITY_MIX 2 /* 4 : 7     (the parity-only encode's 29 : 51) */
int ec_bw_probe(int shape, const uint8_t *src, size_t read_bytes, uint8_t *dst, size_t *moved, ec_stream stream);
/* The RS(29,80) encoder's own memory schedule without its arithmetic: exactly
 * ec_encode_segments' launch (same loaders, LDS ring, tile queue, slicing,
 * copy-through and parity stores, flags as there), with the GF
 * multiply-accumulate removed -- each parity row stored is a copy of the
 * tile's last input share, so the pieces written are NOT the code's.  The
 * on-box ceiling of the encoder's access pattern (bench.py); measurement only.
 * EC_ERR_UNSUPPORTED for any other (k, n), or ess / pointers not 16-aligned. */
int ec_encode_shape_probe(const ec_ctx *ctx, const uint8_t *segs, size_t nseg, size_t nstripes, uint8_t *pieces,
                          int flags, ec_stream stream);

/* ---- device helpers ---- */
int ec_device_count(void);
int ec_set_device(int device);
/* name of the kernel ec_encode_segments uses for whole segments of this ctx
 * right now: "straight-line" (at most 32 parity rows: the runtime-matrix
 * kernel with the parity rows as generated straight-line code, unless
 * ec_set_body selected the jump table), "special" (compile-time G, built into
 * the library), "special-jit" (compiled for this (k, n) at run time),
 * "generic" (runtime matrix), "bytes" (ess not a multiple of 16) or "copy"
 * (n == k) */
const char *ec_encode_kernel_name(const ec_ctx *ctx);
/* The compile-time-G encoder of a (k, n) that is not built into the library
 * is compiled in the background from its first whole-segment encode call (at
 * least 256 tiles: a few MiB of stripes) or this call on (hiprtc, ~1 s; the
 * code object is cached on disk); per-stripe and few-stripe calls never start
 * one.  Until it is ready the encode calls use the runtime-matrix kernel, with
 * identical results.  A process that started a compile waits at exit for the
 * one in progress.  Returns 1 when it is ready (with wait != 0: after waiting
 * for the compilation), 0 when this (k, n) has none.  UPLINK_EC_JIT=0 in the
 * environment turns run-time compilation off. */
int ec_prepare_encoder(const ec_ctx *ctx, int wait);
/* Body of the runtime-matrix kernel for this ctx's decode (and other
 * runtime-matrix) plans, DESIGN.md §4 "Straight-line rebuild":
 *   EC_BODY_AUTO (default): the plan's generated straight-line code for
 *     launches of at least 64 tiles (131,072 byte columns per share), the
 *     jump table for smaller ones (per-stripe calls);
 *   EC_BODY_JUMP_TABLE: always the jump table;
 *   EC_BODY_STRAIGHT_LINE: generated code for every launch it fits, and
 *     every encode on it (also those a compile-time encoder would take).
 * The results are identical.  No reference counterpart (an engine knob). */
#define EC_BODY_AUTO 0
#define EC_BODY_JUMP_TABLE 1
#define EC_BODY_STRAIGHT_LINE 2
int ec_set_body(ec_ctx *ctx, int body);
/* which body the ctx's last runtime-matrix launch used: EC_BODY_JUMP_TABLE,
 * EC_BODY_STRAIGHT_LINE, or EC_BODY_AUTO when there was none yet */
int ec_last_body(const ec_ctx *ctx);
/* Compile-time encoder launches of this ctx so far that took a work-counter
 * slot (tiles handed out by a queue) and that assigned their tiles statically
 * because no slot was free without waiting for another stream (identical
 * results; a diagnostic).  No reference counterpart. */
int ec_encoder_queue_stats(const ec_ctx *ctx, unsigned long long *queued, unsigned long long *static_tiles);
/* Identity of this build: 16 hex digits of a SHA-256 over the library's
 * sources, generators and build flags (uplink_amd/csrc/Makefile).  Measurement
 * records taken from one build (profiles/pmc_traffic.json) carry it, so a bench
 * run of another build can tell they are stale.  No reference counterpart. */
const char *ec_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* UPLINK_EC_H */
