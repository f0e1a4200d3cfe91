// C-ABI, streamed upload (include/uplink_ec.h ec_upload_*): one host segment
// through the GPU in chunks of stripes, every piece's chunk in host memory as
// soon as it is encoded, with every piece's BLAKE3 folded along (DESIGN.md §5
// "Upload path").
#include "ec_internal.hpp"

extern "C" {

// ---------------------------------------------------------------- streamed upload
// One segment through the engine in chunks of stripes, each chunk of every
// piece in host memory as soon as it is encoded, for piece readers that serve
// a piece stripe by stripe (segmentupload/encode.go:39-75, single.go:228-238):
// an upload starts sending after the first chunk instead of the whole segment.
// Chunks grow from kUploadFirstChunk stripes, doubling up to kUploadMaxChunk,
// so the first bytes come early and the later chunks keep the PCIe pipeline
// (H2D of chunk i+1, encode of chunk i, D2H of chunk i-1) busy.
constexpr size_t kUploadFirstChunk = 128, kUploadMaxChunk = 2048;

struct ec_upload {
    ec_ctx *c = nullptr;
    std::unique_ptr<UploadSlot> slot;
    std::vector<size_t> end;  // end stripe of each chunk
    std::atomic<int> rc{EC_OK};
    std::atomic<int> done{0};  // leading chunks known to be in host memory
    int n = 0;                 // pieces hashed (EC_FLAG_HASH_PIECES), 0 without
    // the hash work, queued by the first caller that waits on the upload or asks for the hashes
    // (not by ec_upload_begin, so the first chunk's copies and encode start without waiting for
    // the host to queue ~10 more operations)
    std::once_flag hash_once;
    int hash_rc = EC_OK;
    bool streamed_hash = false, parity_only = false;
    size_t nstripes = 0;
    B3View dv{}, pv{};
    uint32_t *cvs = nullptr;
    uint8_t *d_hashes = nullptr, *d_scratch = nullptr, *d_parity = nullptr;
    // ec_upload_end waits for the callers inside ec_upload_wait / _ready /
    // _hashes before it frees the handle (piece readers block in
    // those while another thread closes the segment)
    std::mutex mu;
    std::condition_variable cv;
    int inside = 0;
    bool ending = false;
};

static void upload_release(ec_upload *u) {
    if (!u->slot) return;
    for (auto st : u->slot->st)
        if (st) (void)hipStreamSynchronize(st);
    std::lock_guard<std::mutex> g(u->c->upload_mu);
    u->c->upload_free.push_back(std::move(u->slot));
}

// A caller inside one of the waiting calls on u (released by the destructor).
struct UploadUse {
    ec_upload *u;
    bool ok;
    explicit UploadUse(ec_upload *x) : u(x) {
        std::lock_guard<std::mutex> g(u->mu);
        ok = !u->ending;
        if (ok) u->inside++;
    }
    ~UploadUse() {
        if (!ok) return;
        std::lock_guard<std::mutex> g(u->mu);
        if (--u->inside == 0) u->cv.notify_all();
    }
};

// The piece hashes of a streamed upload, chunk by chunk: after the encode of
// each chunk of stripes, the chaining values of the BLAKE3 chunks that chunk
// completes in every piece (data pieces straight from the segment, parity from
// the encoder's output), on a stream of their own; after the last, the tree
// fold and the hashes' copy to pinned memory.  The reference hashes each piece
// as it streams through a TeeReader and needs the sum only at the end
// (piecestore/upload.go:155,262-270): so does this.  A chunk boundary that
// does not fall on a 1-KiB boundary of the pieces (a caller's chunk size), or
// pieces of one BLAKE3 chunk, hash everything after the last chunk instead.
static bool upload_hash_streamed(const ec_ctx *c, const std::vector<size_t> &end, size_t nstripes) {
    const uint64_t plen = (uint64_t)nstripes * c->ess;
    if (plen < 2048) return false;
    for (size_t i = 0; i + 1 < end.size(); i++)
        if ((end[i] * (uint64_t)c->ess) % 1024) return false;
    return true;
}

int ec_upload_begin(const ec_ctx *cc, const uint8_t *seg, size_t nstripes, uint8_t *pieces, int flags,
                    size_t chunk_stripes, ec_upload **out) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!out) return EC_ERR_INVALID_ARG;
    *out = nullptr;
    if (!c || !seg || !pieces) return EC_ERR_INVALID_ARG;
    if (flags & ~(EC_FLAG_PARITY_ONLY | EC_FLAG_HASH_PIECES)) return EC_ERR_INVALID_ARG;
    DeviceGuard dg(c->device);
    std::unique_ptr<ec_upload> u(new ec_upload());
    u->c = c;
    for (size_t s0 = 0, len = chunk_stripes ? chunk_stripes : kUploadFirstChunk; s0 < nstripes;) {
        const size_t s1 = std::min(nstripes, s0 + len);
        u->end.push_back(s1);
        s0 = s1;
        if (!chunk_stripes) len = std::min(kUploadMaxChunk, 2 * len);
    }
    const size_t nch = u->end.size();
    const size_t ess = c->ess, stripe = (size_t)c->k * ess, spad = nstripes * stripe;
    const bool parity_only = (flags & EC_FLAG_PARITY_ONLY) != 0;
    const bool hashed = (flags & EC_FLAG_HASH_PIECES) != 0;
    const int rows = parity_only ? c->n - c->k : c->n;
    const size_t plen = nstripes * ess, pbytes = (size_t)rows * plen;
    const bool streamed_hash = hashed && upload_hash_streamed(c, u->end, nstripes);
    const uint64_t nb3 = (plen + 1023) / 1024;  // BLAKE3 chunks per piece
    // hash area: [n][nb3][8] chunk CVs | n*32 hashes | scratch (fold, or the one-pass hash's)
    const size_t cvs_bytes = streamed_hash ? align_up((size_t)c->n * nb3 * 32, 256) : 0;
    const size_t hash_bytes = align_up(32 * (size_t)c->n, 256);
    const size_t scratch = streamed_hash ? b3_fold_ws_bytes(c->n, nb3) : b3_segment_ws_bytes(c, 1, nstripes);
    const size_t hcap = hashed ? cvs_bytes + hash_bytes + std::max<size_t>(scratch, 256) : 0;
    {
        std::lock_guard<std::mutex> g(c->upload_mu);
        if (!c->upload_free.empty()) {
            u->slot = std::move(c->upload_free.back());
            c->upload_free.pop_back();
        }
    }
    if (!u->slot) u->slot.reset(new UploadSlot());
    UploadSlot &sl = *u->slot;
    for (auto &st : sl.st)
        if (!st) HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    if (sl.in_cap < spad) {
        if (sl.d_in) (void)hipFree(sl.d_in);
        sl.d_in = nullptr;
        sl.in_cap = 0;
        HIP_TRY(hipMalloc(&sl.d_in, std::max<size_t>(spad, 1)));
        sl.in_cap = spad;
    }
    if (sl.out_cap < pbytes) {
        if (sl.d_out) (void)hipFree(sl.d_out);
        sl.d_out = nullptr;
        sl.out_cap = 0;
        HIP_TRY(hipMalloc(&sl.d_out, std::max<size_t>(pbytes, 1)));
        sl.out_cap = pbytes;
    }
    if (hashed && sl.hash_cap < hcap) {
        if (sl.d_hash) (void)hipFree(sl.d_hash);
        sl.d_hash = nullptr;
        sl.hash_cap = 0;
        HIP_TRY(hipMalloc(&sl.d_hash, hcap));
        sl.hash_cap = hcap;
    }
    if (hashed && sl.h_hash_cap < 32 * (size_t)c->n) {
        if (sl.h_hash) (void)hipHostFree(sl.h_hash);
        sl.h_hash = nullptr;
        sl.h_hash_cap = 0;
        HIP_TRY(hipHostMalloc((void **)&sl.h_hash, 32 * (size_t)c->n, hipHostMallocDefault));
        sl.h_hash_cap = 32 * (size_t)c->n;
    }
    while (sl.ev.size() < 3 * nch + 1) {
        hipEvent_t e = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        sl.ev.push_back(e);
    }
    hipStream_t h2d = sl.st[0], comp = sl.st[1], d2h = sl.st[2];
    uint32_t *cvs = (uint32_t *)sl.d_hash;
    uint8_t *d_hashes = sl.d_hash + cvs_bytes, *d_scratch = d_hashes + hash_bytes;
    const uint8_t *d_parity = sl.d_out + (parity_only ? 0 : (size_t)c->k * plen);
    B3View pv = parity_view(c, d_parity, 1, nstripes);
    if (c->n == c->k) pv.npieces = 0;
    const B3View dv = data_view(c, sl.d_in, 1, nstripes);
    int rc = EC_OK;
    for (size_t ch = 0; ch < nch && rc == EC_OK; ch++) {
        const size_t s0 = ch ? u->end[ch - 1] : 0, s1 = u->end[ch];
        hipEvent_t e_in = sl.ev[ch], e_enc = sl.ev[nch + ch], e_out = sl.ev[2 * nch + ch];
        if (hipMemcpyAsync(sl.d_in + s0 * stripe, seg + s0 * stripe, (s1 - s0) * stripe, hipMemcpyHostToDevice,
                           h2d) != hipSuccess ||
            hipEventRecord(e_in, h2d) != hipSuccess || hipStreamWaitEvent(comp, e_in, 0) != hipSuccess) {
            rc = EC_ERR_DEVICE;
            break;
        }
        if (rows > 0) rc = encode_range(c, sl.d_in, 1, nstripes, s0, s1, sl.d_out, flags & EC_FLAG_PARITY_ONLY, comp);
        if (rc) break;
        if (hipEventRecord(e_enc, comp) != hipSuccess || hipStreamWaitEvent(d2h, e_enc, 0) != hipSuccess ||
            (rows > 0 && hipMemcpy2DAsync(pieces + s0 * ess, plen, sl.d_out + s0 * ess, plen, (s1 - s0) * ess, rows,
                                          hipMemcpyDeviceToHost, d2h) != hipSuccess) ||
            hipEventRecord(e_out, d2h) != hipSuccess)
            rc = EC_ERR_DEVICE;
    }
    if (hashed) {  // queued later (upload_queue_hashes): the first chunk is not held up by it
        u->n = c->n;
        u->streamed_hash = streamed_hash;
        u->parity_only = parity_only;
        u->nstripes = nstripes;
        u->dv = dv;
        u->pv = pv;
        u->cvs = cvs;
        u->d_hashes = d_hashes;
        u->d_scratch = d_scratch;
        u->d_parity = (uint8_t *)d_parity;
    }
    u->rc.store(rc);
    if (rc) {
        upload_release(u.get());
        return rc;
    }
    *out = u.release();
    return EC_OK;
}

// The piece-hash work of an EC_FLAG_HASH_PIECES upload, on its hash stream:
// each group of about a third of the chunks hashed as soon as its last chunk
// is encoded (a stream wait on that chunk's encode event), then the tree fold
// and the hashes' copy to pinned memory.  Queued once, by the first caller of
// ec_upload_wait or ec_upload_hashes.
static void upload_queue_hashes(ec_upload *u) {
    std::call_once(u->hash_once, [u] {
        ec_ctx *c = u->c;
        UploadSlot &sl = *u->slot;
        const size_t nch = u->end.size(), ess = c->ess;
        const uint64_t nb3 = (u->nstripes * ess + 1023) / 1024;
        hipStream_t hs = sl.st[3];
        hipError_t e = hipSuccess;
        if (u->streamed_hash) {
            size_t from = 0;  // first stripe not yet hashed
            for (size_t ch = 0; ch < nch && e == hipSuccess; ch++) {
                const bool last = ch + 1 == nch;
                if (!last && (u->end[ch] - from) * 3 < u->nstripes) continue;  // (groups of ~1/3 of the segment)
                const uint64_t c0 = from * ess / 1024, c1 = last ? nb3 : u->end[ch] * ess / 1024;
                e = hipStreamWaitEvent(hs, sl.ev[nch + ch], 0);
                if (e == hipSuccess) e = b3_launch_chunk_range(u->dv, u->pv, c0, c1, u->cvs, hs);
                from = u->end[ch];
            }
        }
        if (e == hipSuccess) e = hipStreamWaitEvent(hs, sl.ev[2 * nch - 1], 0);  // (the last encode)
        if (e == hipSuccess)
            e = u->streamed_hash ? b3_launch_fold(u->cvs, c->n, nb3, u->d_hashes, u->d_scratch, hs)
                                 : (hash_segments(c, sl.d_in, u->d_parity, 1, u->nstripes, u->d_hashes, u->d_scratch,
                                                  hs) == EC_OK ? hipSuccess : hipErrorUnknown);
        if (e == hipSuccess) e = hipMemcpyAsync(sl.h_hash, u->d_hashes, 32 * (size_t)c->n, hipMemcpyDeviceToHost, hs);
        if (e == hipSuccess) e = hipEventRecord(sl.ev[3 * nch], hs);
        u->hash_rc = e == hipSuccess ? EC_OK : hip_fail(e);
    });
}

static int upload_wait_chunks(ec_upload *u, size_t stripes) {
    const int nch = (int)u->end.size();
    for (;;) {
        if (const int rc = u->rc.load()) return rc;
        int d = u->done.load();
        if (d == nch || (d > 0 && u->end[d - 1] >= stripes)) return EC_OK;
        if (hipEventSynchronize(u->slot->ev[2 * nch + d]) != hipSuccess) {
            u->rc.store(EC_ERR_DEVICE);
            return EC_ERR_DEVICE;
        }
        u->done.compare_exchange_strong(d, d + 1);
    }
}

// Any number of threads may wait on one upload (one per piece reader); the
// event waits run without a lock, and the count of done chunks only grows.
int ec_upload_wait(ec_upload *u, size_t stripes) {
    if (!u) return EC_ERR_INVALID_ARG;
    UploadUse use(u);
    if (!use.ok) return EC_ERR_INVALID_ARG;
    DeviceGuard dg(u->c->device);
    if (u->n && u->rc.load() == EC_OK) upload_queue_hashes(u);  // (while the first chunk is on its way)
    return upload_wait_chunks(u, stripes);
}

size_t ec_upload_ready(ec_upload *u) {
    if (!u || u->rc.load()) return 0;
    UploadUse use(u);
    if (!use.ok) return 0;
    DeviceGuard dg(u->c->device);
    const int nch = (int)u->end.size();
    for (int d = u->done.load(); d < nch && hipEventQuery(u->slot->ev[2 * nch + d]) == hipSuccess; d = u->done.load())
        u->done.compare_exchange_strong(d, d + 1);
    const int d = u->done.load();
    return d ? u->end[d - 1] : 0;
}

int ec_upload_hashes(ec_upload *u, uint8_t *hashes) {
    if (!u || !hashes) return EC_ERR_INVALID_ARG;
    UploadUse use(u);
    if (!use.ok || u->n == 0) return EC_ERR_INVALID_ARG;  // (begun without EC_FLAG_HASH_PIECES)
    if (const int rc = u->rc.load()) return rc;
    DeviceGuard dg(u->c->device);
    upload_queue_hashes(u);
    if (u->hash_rc) return u->hash_rc;
    if (hipEventSynchronize(u->slot->ev[3 * u->end.size()]) != hipSuccess) return EC_ERR_DEVICE;
    memcpy(hashes, u->slot->h_hash, 32 * (size_t)u->n);
    return EC_OK;
}

int ec_upload_end(ec_upload *u) {
    if (!u) return EC_ERR_INVALID_ARG;
    int rc = u->rc.load();
    {
        DeviceGuard dg(u->c->device);
        if (rc == EC_OK) rc = upload_wait_chunks(u, SIZE_MAX);
        std::unique_lock<std::mutex> g(u->mu);
        u->ending = true;  // new callers are turned away; those inside finish first
        u->cv.wait(g, [&] { return u->inside == 0; });
        g.unlock();
        upload_release(u);
    }
    delete u;
    return rc;
}

}  // extern "C"
