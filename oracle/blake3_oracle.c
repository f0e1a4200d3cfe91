/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Nothing in the product path
 * (uplink_amd/, include/) may link, load or call this file.  Only tests/,
 * __graft_entry__.smoke() and the CPU-baseline legs of the benches use it.
 *
 * CPU restatement of BLAKE3-256 (unkeyed hash mode), the default piece hash
 * of storj/uplink's piecestore upload:
 *
 *   GetPieceHashAlgo -> pb.PieceHashAlgorithm_BLAKE3   private/piecestore/hash.go:20-26
 *   hash := pb.NewHashFromAlgorithm(algo)              private/piecestore/upload.go:133
 *   data = io.TeeReader(data, client.hash)             private/piecestore/upload.go:155
 *   Hash: client.hash.Sum(nil)                         private/piecestore/upload.go:270
 *
 * The implementation behind NewHashFromAlgorithm is github.com/zeebo/blake3
 * v0.2.3 (go.mod:29), which is not vendored in the reference tree and is
 * absent from this container.  This file restates the published BLAKE3
 * algorithm (O'Connor, Aumasson, Neves, Wilcox-O'Hearn, "BLAKE3: one
 * function, fast everywhere", 2020, §2): BLAKE2s-style compression with 7
 * rounds and the fixed message permutation, 1024-byte chunks of 64-byte
 * blocks, a left-complete binary tree of parent nodes built with the
 * incremental chaining-value stack of §5.1.1.  It is pinned against the
 * official test vectors (tests/golden/blake3_vectors.json, see
 * tests/test_blake3.py).
 *
 * The GPU kernel builds the same tree a different way (pairwise levels with
 * the odd right-edge node promoted), so agreement also checks that the two
 * tree constructions coincide.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { B3_CHUNK_START = 1, B3_CHUNK_END = 2, B3_PARENT = 4, B3_ROOT = 8 };
#define B3_BLOCK 64
#define B3_CHUNK 1024

static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                  0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static inline void g(uint32_t *v, int a, int b, int c, int d, uint32_t x, uint32_t y) {
    v[a] += v[b] + x;
    v[d] = rotr(v[d] ^ v[a], 16);
    v[c] += v[d];
    v[b] = rotr(v[b] ^ v[c], 12);
    v[a] += v[b] + y;
    v[d] = rotr(v[d] ^ v[a], 8);
    v[c] += v[d];
    v[b] = rotr(v[b] ^ v[c], 7);
}

/* compression function (§2.2): returns the full 16-word output state */
static void compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter, uint32_t block_len,
                     uint32_t flags, uint32_t out[16]) {
    uint32_t v[16], m[16], t[16];
    for (int i = 0; i < 8; i++) v[i] = cv[i];
    for (int i = 0; i < 4; i++) v[8 + i] = B3_IV[i];
    v[12] = (uint32_t)counter;
    v[13] = (uint32_t)(counter >> 32);
    v[14] = block_len;
    v[15] = flags;
    memcpy(m, block, sizeof m);
    for (int r = 0; r < 7; r++) {
        g(v, 0, 4, 8, 12, m[0], m[1]);
        g(v, 1, 5, 9, 13, m[2], m[3]);
        g(v, 2, 6, 10, 14, m[4], m[5]);
        g(v, 3, 7, 11, 15, m[6], m[7]);
        g(v, 0, 5, 10, 15, m[8], m[9]);
        g(v, 1, 6, 11, 12, m[10], m[11]);
        g(v, 2, 7, 8, 13, m[12], m[13]);
        g(v, 3, 4, 9, 14, m[14], m[15]);
        for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
        memcpy(m, t, sizeof m);
    }
    for (int i = 0; i < 8; i++) {
        out[i] = v[i] ^ v[i + 8];
        out[i + 8] = v[i + 8] ^ cv[i];
    }
}

static void load_block(const uint8_t *p, size_t n, uint32_t w[16]) {
    uint8_t buf[B3_BLOCK] = {0};
    memcpy(buf, p, n);
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)buf[4 * i] | (uint32_t)buf[4 * i + 1] << 8 | (uint32_t)buf[4 * i + 2] << 16 |
               (uint32_t)buf[4 * i + 3] << 24;
}

/* A node whose compression is still pending: either the last block of a
 * chunk or a parent block.  Its CV (non-root) or its root output is taken
 * from it once we know whether it is the root. */
typedef struct {
    uint32_t cv[8];
    uint32_t block[16];
    uint64_t counter;
    uint32_t block_len, flags;
} pending;

static void pending_cv(const pending *p, uint32_t cv[8]) {
    uint32_t o[16];
    compress(p->cv, p->block, p->counter, p->block_len, p->flags, o);
    memcpy(cv, o, 32);
}

/* chunk `index` (len <= 1024 bytes): compresses every block but the last and
 * returns the last one pending (§2.4) */
static void chunk_pending(const uint8_t *p, size_t len, uint64_t index, pending *out) {
    uint32_t cv[8], w[16], o[16];
    memcpy(cv, B3_IV, 32);
    size_t nblocks = len ? (len + B3_BLOCK - 1) / B3_BLOCK : 1;
    for (size_t b = 0; b + 1 < nblocks; b++) {
        load_block(p + b * B3_BLOCK, B3_BLOCK, w);
        compress(cv, w, index, B3_BLOCK, b == 0 ? B3_CHUNK_START : 0, o);
        memcpy(cv, o, 32);
    }
    size_t last = len - (nblocks - 1) * B3_BLOCK;
    memcpy(out->cv, cv, 32);
    load_block(p + (nblocks - 1) * B3_BLOCK, last, out->block);
    out->counter = index;
    out->block_len = (uint32_t)last;
    out->flags = (nblocks == 1 ? B3_CHUNK_START : 0) | B3_CHUNK_END;
}

static void parent_pending(const uint32_t l[8], const uint32_t r[8], pending *out) {
    memcpy(out->cv, B3_IV, 32);
    memcpy(out->block, l, 32);
    memcpy(out->block + 8, r, 32);
    out->counter = 0;
    out->block_len = B3_BLOCK;
    out->flags = B3_PARENT;
}

/* BLAKE3-256 of in[0..len) (hash mode, 32-byte output), built with the
 * incremental CV stack: after chunk c (c >= 1 chunks done) merge while the
 * chunk count has trailing zero bits (§5.1.1); finalize right to left. */
void b3_hash(const uint8_t *in, size_t len, uint8_t out[32]) {
    uint32_t stack[64][8];
    int depth = 0;
    size_t nchunks = len ? (len + B3_CHUNK - 1) / B3_CHUNK : 1;
    pending cur = {{0}, {0}, 0, 0, 0};
    for (size_t c = 0; c < nchunks; c++) {
        size_t off = c * B3_CHUNK, n = len - off < B3_CHUNK ? len - off : B3_CHUNK;
        if (len == 0) n = 0;
        chunk_pending(in + off, n, c, &cur);
        if (c + 1 == nchunks) break;
        uint32_t cv[8];
        pending_cv(&cur, cv);
        uint64_t total = c + 1;
        while ((total & 1) == 0) {
            pending par;
            parent_pending(stack[--depth], cv, &par);
            pending_cv(&par, cv);
            total >>= 1;
        }
        memcpy(stack[depth++], cv, 32);
    }
    while (depth > 0) {
        uint32_t cv[8];
        pending_cv(&cur, cv);
        parent_pending(stack[--depth], cv, &cur);
    }
    uint32_t o[16];
    compress(cur.cv, cur.block, cur.counter, cur.block_len, cur.flags | B3_ROOT, o);
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(o[i] >> (8 * j));
}

/* ---- CPU baseline: many pieces, one thread each ---- */
typedef struct {
    const uint8_t *base;
    size_t stride, len, first, count;
    uint8_t *out;
} b3_job;

static void *b3_worker(void *a) {
    b3_job *j = (b3_job *)a;
    for (size_t i = j->first; i < j->first + j->count; i++) b3_hash(j->base + i * j->stride, j->len, j->out + 32 * i);
    return NULL;
}

/* out[32*i] = BLAKE3(base + i*stride, len) for i < npieces, on `threads`
 * threads (pieces split evenly) */
void b3_hash_many(const uint8_t *base, size_t npieces, size_t stride, size_t len, uint8_t *out, int threads) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > npieces) threads = (int)(npieces ? npieces : 1);
    pthread_t th[256];
    b3_job jobs[256];
    if (threads > 256) threads = 256;
    size_t per = npieces / threads, extra = npieces % threads, first = 0;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (b3_job){base, stride, len, first, per + ((size_t)t < extra), out};
        first += jobs[t].count;
        if (t == threads - 1)
            b3_worker(&jobs[t]);
        else
            pthread_create(&th[t], NULL, b3_worker, &jobs[t]);
    }
    for (int t = 0; t < threads - 1; t++) pthread_join(th[t], NULL);
}
