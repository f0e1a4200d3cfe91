// C-ABI, share-set calls (include/uplink_ec.h ec_rebuild_segments_sets,
// ec_decode_segments_sets, ec_rebuild_segments_batched, ec_prepare_rebuild):
// a batch of segments each rebuilt or decoded from its own share set in one
// stream-ordered pass (rs_sets.hpp), and the per-context background builder
// of decode plans' straight-line code.
#include "ec_internal.hpp"

namespace uplink_ec {
namespace capi {
namespace {

// ---------------------------------------------------------------- share-set calls (rs_sets.hpp)

// One segment of a share-set call as the host prepares it: the inputs in the
// kernel's order (infectious' k chosen shares by position, then -- Decode --
// the other shares by number) and the rows (missing data positions, then one
// syndrome row per non-basis input).
struct SetSeg {
    const uint8_t *in[kMaxOps];
    int num[kMaxOps];
    int missing[kMaxOps];
    int nin = 0, nstore = 0, rows = 0, nw = 2;
    uint8_t *out = nullptr;
};

// Fill `sg` for one segment given as (nshares, nums, pieces).  Errors as
// Rebuild / Decode report them (NotEnoughShares, invalid share id, a repeated
// share chosen twice: singular).
int set_segment(const ec_ctx *c, int nshares, const int *nums, const uint8_t *const *pieces, uint8_t *out,
                bool decode, SetSeg &sg) {
    const int k = c->k;
    std::vector<int> order, ids;
    int rc = choose_shares(c, nshares, nums, order, ids);
    if (rc) return rc;
    if (decode)
        for (int i = 0; i < nshares; i++)
            if (nums[i] < 0 || nums[i] >= c->n) return EC_ERR_INVALID_SHARE;
    bool seen[256] = {};
    sg.nin = k;
    sg.nstore = 0;
    for (int i = 0; i < k; i++) {
        if (seen[ids[i]]) return EC_ERR_SINGULAR;
        seen[ids[i]] = true;
        sg.in[i] = pieces[order[i]];
        sg.num[i] = ids[i];
        if (ids[i] >= k) sg.missing[sg.nstore++] = i;
    }
    if (decode) {
        if (nshares > kMaxOps) return EC_ERR_UNSUPPORTED;
        std::vector<char> chosen(nshares, 0);
        for (int i = 0; i < k; i++) chosen[order[i]] = 1;
        std::vector<int> rest;
        for (int i = 0; i < nshares; i++)
            if (!chosen[i]) rest.push_back(i);
        std::stable_sort(rest.begin(), rest.end(), [&](int x, int y) { return nums[x] < nums[y]; });
        for (int i : rest) {
            sg.in[sg.nin] = pieces[i];
            sg.num[sg.nin++] = nums[i];
        }
    }
    sg.rows = sg.nstore + (sg.nin - k);
    sg.nw = sets_waves(sg.rows);
    sg.out = out;
    return EC_OK;
}

// The rows of a Rebuild segment as rs_sets_prep solves them (rs_sets.hip,
// closed-form Lagrange weights through the basis shares' points), into
// coef[r * nin + j]: missing data position r from basis input j.
void solve_rows_host(const SetSeg &sg, int k, uint8_t *coef) {
    uint8_t x[kMaxOps];
    int lw[kMaxOps];
    for (int p = 0; p < k; p++) x[p] = gf_point(sg.num[p]);
    for (int p = 0; p < k; p++) {
        int l = 0;
        for (int t = 0; t < k; t++)
            if (t != p) l += kGf.log[x[p] ^ x[t]];
        lw[p] = l % 255;
    }
    for (int r = 0; r < sg.nstore; r++) {
        const uint8_t y = gf_point(sg.missing[r]);
        int ln = 0, hit = -1;
        for (int t = 0; t < k; t++) {
            if (y == x[t]) hit = t;
            else ln += kGf.log[y ^ x[t]];
        }
        for (int j = 0; j < k; j++)
            coef[r * sg.nin + j] = hit >= 0 ? (uint8_t)(hit == j)
                                            : kGf.exp[(((ln - kGf.log[y ^ x[j]] - lw[j]) % 255) + 255) % 255];
    }
}

// The slots' host memory is read by rs_sets_prep and written by the launches'
// last workgroup straight over the bus: coherent (uncached on the GPU side), so
// a slot reused by the next call is never read from a stale cache line.
constexpr unsigned kSetsHostFlags = hipHostMallocCoherent | hipHostMallocMapped;

// A free slot of the ring with room for nseg segments and tgt_words words of
// leaf tables.  Waits while kMaxSlots live calls are in flight on the GPU, at
// most kAcquireTimeoutMs; dead slots (a failed launch the device did not
// recover from) do not count against the ring.  nullptr: no slot (timeout, or
// no memory).
SetsSlot *sets_acquire(ec_ctx *c, size_t nseg, size_t tgt_words) {
    SetsRing &R = c->sets;
    SetsSlot *sl = nullptr;
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(SetsRing::kAcquireTimeoutMs);
    for (;;) {
        {
            std::lock_guard<std::mutex> g(R.mu);
            size_t live = 0;
            for (auto &x : R.slots) {
                live += !x->dead;
                if (!sl && x->idle()) sl = x.get();
            }
            if (!sl && live < SetsRing::kMaxSlots) {
                auto x = std::make_unique<SetsSlot>();
                if (hipHostMalloc((void **)&x->h_words, 4 * (SetsRing::kInitSegs + 1), kSetsHostFlags) != hipSuccess)
                    return nullptr;
                memset(x->h_words, 0, 4 * (SetsRing::kInitSegs + 1));
                x->words_cap = SetsRing::kInitSegs + 1;
                x->stage_cap = 0;
                R.slots.push_back(std::move(x));
                sl = R.slots.back().get();
            }
            if (sl) sl->busy = true;
        }
        if (sl) break;
        if (std::chrono::steady_clock::now() > t_end) return nullptr;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    // (the slot is ours, and the GPU is done with it: its buffers may be replaced; the ones it
    // outgrows are kept until the slot goes, so no free synchronises the device here)
    bool ok = true;
    if (sl->stage_cap < nseg) {
        size_t cap = std::max(sl->stage_cap ? 2 * sl->stage_cap : SetsRing::kInitSegs, (size_t)32);
        while (cap < nseg) cap *= 2;
        if (sl->h_stage) sl->old_host.push_back(sl->h_stage);
        for (void *p : {(void *)sl->d_stage, (void *)sl->d_desc, (void *)sl->d_words})
            if (p) sl->old_dev.push_back(p);
        sl->h_stage = nullptr, sl->d_stage = nullptr, sl->d_desc = nullptr, sl->d_words = nullptr;
        ok = hipHostMalloc((void **)&sl->h_stage, cap * sizeof(SetStage),
                           c->sets_stage_dma ? hipHostMallocDefault : kSetsHostFlags) == hipSuccess &&
             (!c->sets_stage_dma || hipMalloc(&sl->d_stage, cap * sizeof(SetStage)) == hipSuccess) &&
             hipMalloc(&sl->d_desc, cap * sizeof(SetDesc)) == hipSuccess &&
             hipMalloc(&sl->d_words, 4 * (cap + 1)) == hipSuccess;
        if (ok && cap + 1 > sl->words_cap) {
            uint32_t *hw = nullptr;
            ok = hipHostMalloc((void **)&hw, 4 * (cap + 1), kSetsHostFlags) == hipSuccess;
            if (ok) {
                hw[0] = sl->seq;
                sl->old_host.push_back(sl->h_words);
                sl->h_words = hw;
                sl->words_cap = cap + 1;
            }
        }
        sl->stage_cap = ok ? cap : 0;
    }
    if (ok && sl->tgt_cap < tgt_words) {
        size_t cap = std::max(sl->tgt_cap ? 2 * sl->tgt_cap : SetsRing::kInitTgtWords, (size_t)1);
        while (cap < tgt_words) cap *= 2;
        if (sl->d_tgt) sl->old_dev.push_back(sl->d_tgt);
        sl->d_tgt = nullptr;
        ok = hipMalloc(&sl->d_tgt, cap * 8) == hipSuccess;
        sl->tgt_cap = ok ? cap : 0;
    }
    if (!ok) {
        std::lock_guard<std::mutex> g(R.mu);
        sl->busy = false;
        return nullptr;
    }
    return sl;
}

void sets_release(ec_ctx *c, SetsSlot *sl) {
    std::lock_guard<std::mutex> g(c->sets.mu);
    sl->busy = false;
}

// The share-set pass over segs (each nstripes stripes): rs_sets_prep, then one
// rs_matmul_sets launch per wave-count class, all on stream s.  With `bad`
// (Decode), waits and returns per segment the count of syndrome failures.
int sets_call(ec_ctx *c, std::vector<SetSeg> &segs, int64_t nstripes, hipStream_t s, std::vector<uint32_t> *bad) {
    const int k = c->k, ess = c->ess;
    const size_t nseg = segs.size();
    if (nseg == 0 || nstripes == 0) return EC_OK;
    if (c->sets_merge) {  // every segment on the widest class's workgroups: one launch, one tail
        int nw = 2;
        for (auto &sg : segs) nw = std::max(nw, sg.nw);
        for (auto &sg : segs) sg.nw = nw;
    }
    {  // more tiles than one launch takes: in parts (each a call of its own)
        const int64_t tiles_seg = (nstripes * (ess / 16) + kTileChunksHost - 1) / kTileChunksHost;
        const int64_t per = sets_max_tiles(4) / tiles_seg;
        if (per < 1) return EC_ERR_UNSUPPORTED;
        if ((int64_t)nseg > per) {
            for (size_t g0 = 0; g0 < nseg; g0 += (size_t)per) {
                std::vector<SetSeg> part(segs.begin() + g0, segs.begin() + std::min(nseg, g0 + (size_t)per));
                std::vector<uint32_t> pbad;
                const int rc = sets_call(c, part, nstripes, s, bad ? &pbad : nullptr);
                if (rc) return rc;
                if (bad) bad->insert(bad->end(), pbad.begin(), pbad.end());
            }
            return EC_OK;
        }
    }
    std::vector<int> idx(nseg);
    for (size_t g = 0; g < nseg; g++) idx[g] = (int)g;
    std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return segs[x].nw < segs[y].nw; });
    std::vector<size_t> toff(nseg);
    size_t words = 0;
    for (size_t q = 0; q < nseg; q++) {
        toff[q] = words;
        words += (sets_tgt_entries(segs[idx[q]].nin, segs[idx[q]].rows, segs[idx[q]].nw) + 7) & ~(size_t)7;
    }
    // the completion-word protocol needs the launches to run: not under stream capture
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return EC_ERR_UNSUPPORTED;
    SetsSlot *sl = sets_acquire(c, nseg, words);
    if (!sl) return EC_ERR_DEVICE;
    // one segment: its record goes in the prep launch's arguments (no read over the bus)
    SetStage one{};
    const bool in_args = nseg == 1 && !sl->d_stage;
    SetStage *stage = in_args ? &one : sl->h_stage;
    for (size_t q = 0; q < nseg; q++) {
        const SetSeg &sg = segs[idx[q]];
        SetStage &st = stage[q];
        SetDesc &d = st.d;
        for (int j = 0; j < sg.nin; j++) {
            d.in[j] = sg.in[j];
            d.copy_off[j] = j < k && sg.num[j] < k ? sg.num[j] * ess : -1;
            st.num[j] = sg.num[j];
        }
        for (int r = 0; r < sg.nstore; r++) {
            d.out_off[r] = sg.missing[r] * ess;
            st.missing[r] = sg.missing[r];
        }
        d.out = sg.out;
        d.tgt = sl->d_tgt + toff[q];
        d.zero_check = bad ? sl->d_words + 1 + q : nullptr;
        d.nin = sg.nin;
        d.nout = sg.rows;
        d.nstore = sg.nstore;
        d.status = 0;
        st.k = k;
        st.nw = sg.nw;
    }
    const uint32_t seq = sl->seq + 1;
    const int64_t chunks = nstripes * (ess / 16), tiles = (chunks + kTileChunksHost - 1) / kTileChunksHost;
    // a pass's arguments, but for its segments (desc, total_tiles)
    auto pass_args = [&](SetsArgs &a) {
        a.nstripes = nstripes;
        a.chunks_per_seg = chunks;
        a.tiles_per_seg = tiles;
        a.ess = ess;
        a.cps = ess / 16;
        a.k = k;
        a.done_ctr = sl->d_words;
        a.host_done = sl->h_words;
        a.seq = seq;
        a.total_wgs = (uint32_t)(tiles * (int64_t)nseg);
        a.chk_flag = c->d_chk;
        a.jt_base = c->jt_base;
    };
    hipError_t e = hipSuccess;
    if (in_args && !bad && c->sets_one && segs[0].nin <= kOneMaxIn && segs[0].nin * segs[0].rows <= kOneMaxCoef) {
        // one segment, one launch: its rows solved here, its record and coefficients in the
        // launch's arguments
        const SetSeg &sg = segs[0];
        SetOne p{};
        pass_args(p.a);
        p.a.total_tiles = tiles;
        for (int j = 0; j < sg.nin; j++) {
            p.in[j] = one.d.in[j];
            p.copy_off[j] = one.d.copy_off[j];
        }
        for (int r = 0; r < sg.nstore; r++) p.out_off[r] = one.d.out_off[r];
        p.out = sg.out;
        p.tgt = sl->d_tgt;
        p.nin = sg.nin;
        p.nout = sg.rows;
        p.nstore = sg.nstore;
        solve_rows_host(sg, k, p.coef);
        e = launch_sets_one(p, sg.nw, s);
        if (e != hipSuccess) {  // nothing was queued
            sets_release(c, sl);
            return hip_fail(e);
        }
        sl->seq = seq;
        c->last_body = EC_BODY_JUMP_TABLE;
        const int rc = after_launch(c->d_chk, s);
        sets_release(c, sl);
        return rc;
    }
    if (sl->d_stage)  // (the host's writes went to cached memory; one DMA takes them to the device)
        e = hipMemcpyAsync(sl->d_stage, sl->h_stage, nseg * sizeof(SetStage), hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = in_args ? launch_sets_prep1(one, sl->d_desc, c->jt_base, sl->d_words, s)
                    : launch_sets_prep(sl->d_stage ? sl->d_stage : sl->h_stage, sl->d_desc, (int)nseg, c->jt_base,
                                       sl->d_words, s);
    if (e != hipSuccess) {  // nothing was queued: the slot is as it was
        sets_release(c, sl);
        return hip_fail(e);
    }
    for (size_t q0 = 0; q0 < nseg && e == hipSuccess;) {
        size_t q1 = q0;
        while (q1 < nseg && segs[idx[q1]].nw == segs[idx[q0]].nw) q1++;
        SetsArgs a{};
        pass_args(a);
        a.desc = sl->d_desc + q0;
        a.total_tiles = tiles * (int64_t)(q1 - q0);
        e = launch_matmul_sets(a, segs[idx[q0]].nw, s);
        q0 = q1;
    }
    if (e != hipSuccess) {
        // the slot's prep (and maybe a class launch) is queued but its completion
        // word will never be written: once the stream has run what was queued, the
        // slot is free again (the next call's prep zeroes its counter); if the
        // device does not get there, the slot is never reused
        // (a one-segment pass, rs_sets_one, relies on the completion counter being zero: a pass that ran
        // in part left it counting)
        const bool drained = hipStreamSynchronize(s) == hipSuccess && hipMemset(sl->d_words, 0, 4) == hipSuccess;
        std::lock_guard<std::mutex> g(c->sets.mu);
        sl->dead = !drained;
        sl->busy = false;
        return hip_fail(e);
    }
    sl->seq = seq;
    c->last_body = EC_BODY_JUMP_TABLE;
    int rc = after_launch(c->d_chk, s);
    if (bad && rc == EC_OK) {
        // (the slot stays busy until the counts are read: another call may not reuse it before)
        if (hipMemcpyAsync(sl->h_words + 1, sl->d_words + 1, 4 * nseg, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            rc = EC_ERR_DEVICE;
        bad->assign(nseg, 0);
        for (size_t q = 0; q < nseg && rc == EC_OK; q++) (*bad)[idx[q]] = sl->h_words[1 + q];
    }
    sets_release(c, sl);
    return rc;
}

// ---------------------------------------------------------------- straight-line code in the background

std::mutex g_builders_mu;
std::set<ec_ctx *> g_builders;  // contexts whose builder thread runs

void sl_worker(ec_ctx *c) {
    (void)hipSetDevice(c->device);
    SlBuilder &B = c->slb;
    for (;;) {
        std::vector<int> ids;
        {
            std::unique_lock<std::mutex> g(B.mu);
            B.cv.wait(g, [&] { return B.stop || !B.q.empty(); });
            if (B.stop) break;
            ids = std::move(B.q.front());
            B.q.pop_front();
        }
        PlanPtr plan;
        if (get_plan(c, ids, &plan) == EC_OK && plan->rows >= 1 && plan->rows <= kMaxOps) ensure_sl(c, *plan);
        {
            std::lock_guard<std::mutex> g(B.mu);
            B.pending.erase(ids);
        }
        B.cv.notify_all();
    }
    std::lock_guard<std::mutex> g(B.mu);
    B.pending.clear();
    B.q.clear();
    B.cv.notify_all();
}

// At exit, builders still running finish the plan in hand before the HIP
// runtime's own exit handlers (registered before this one, on the first HIP
// call) tear the runtime down under a module load.
void stop_builders() {
    std::lock_guard<std::mutex> g(g_builders_mu);
    for (ec_ctx *c : g_builders) {
        {
            std::lock_guard<std::mutex> b(c->slb.mu);
            c->slb.stop = true;
        }
        c->slb.cv.notify_all();
        if (c->slb.th.joinable()) c->slb.th.join();
    }
    g_builders.clear();
}

void stop_builder_impl(ec_ctx *c) {
    {
        std::lock_guard<std::mutex> g(g_builders_mu);
        g_builders.erase(c);
        {
            std::lock_guard<std::mutex> b(c->slb.mu);
            c->slb.stop = true;
        }
        c->slb.cv.notify_all();
    }
    if (c->slb.th.joinable()) c->slb.th.join();
}

// Queue the straight-line code of share set `ids` (no-op if queued already).
void sl_request(ec_ctx *c, const std::vector<int> &ids) {
    SlBuilder &B = c->slb;
    std::lock_guard<std::mutex> g(B.mu);
    if (B.stop || B.pending.count(ids)) return;
    if (!B.th.joinable()) {
        static std::once_flag once;
        std::call_once(once, [] { atexit(stop_builders); });
        std::lock_guard<std::mutex> r(g_builders_mu);
        B.th = std::thread(sl_worker, c);
        g_builders.insert(c);
    }
    B.pending.insert(ids);
    B.q.push_back(ids);
    B.cv.notify_all();
}

// The context's plan for share set ids, if it has one (no plan is made).
PlanPtr find_plan(ec_ctx *c, const std::vector<int> &ids) {
    std::lock_guard<std::mutex> g(c->mu);
    for (auto it = c->plans.begin(); it != c->plans.end(); ++it)
        if ((*it)->key == ids) {
            c->plans.splice(c->plans.begin(), c->plans, it);
            return c->plans.front();
        }
    return nullptr;
}

// The batched rebuild as ec_rebuild_segments_batched runs it: nothing on the
// launch path waits for the host or another stream.  A share set whose
// straight-line code is ready runs it; any other runs the share-set pass (its
// decode rows solved on the GPU, stream-ordered) and, for launches large
// enough to use it, has its code made in the background.
int rebuild_async(ec_ctx *c, int nshares, const int *nums, const uint8_t *const *pieces, int64_t nstripes,
                  int64_t nseg, int64_t pss, int64_t oss, uint8_t *out, hipStream_t s) {
    const int k = c->k, ess = c->ess;
    if (k > kMaxOps) return EC_ERR_UNSUPPORTED;
    std::vector<int> order, ids;
    int rc = choose_shares(c, nshares, nums, order, ids);
    if (rc) return rc;
    bool bits = ess % 16 == 0 && aligned16(out) && pss % 16 == 0 && oss % 16 == 0;
    int m = 0;
    for (int i = 0; i < k; i++) {
        bits = bits && aligned16(pieces[order[i]]);
        m += ids[i] >= k;
    }
    // byte kernel, forced straight-line code, or nothing to compute (the copy
    // kernel; its plan has no tables to wait for): the plan path
    if (!bits || m == 0 || c->body == EC_BODY_STRAIGHT_LINE)
        return rebuild_device(c, nshares, nums, pieces, ess, nstripes, nseg, pss, oss, out, s);
    const int64_t tiles = (nstripes * (ess / 16) + kTileChunksHost - 1) / kTileChunksHost * nseg;
    if (c->body == EC_BODY_AUTO && tiles >= kSlMinTiles) {
        if (PlanPtr plan = find_plan(c, ids); plan && plan->sl_ready.load(std::memory_order_acquire))
            return rebuild_with_plan(c, *plan, order, ids, pieces, ess, nstripes, nseg, pss, oss, out, s);
        sl_request(c, ids);
    }
    std::vector<SetSeg> segs(nseg);
    std::vector<const uint8_t *> pg(nshares);
    for (int64_t g = 0; g < nseg; g++) {
        for (int i = 0; i < nshares; i++) pg[i] = pieces[i] + g * pss;
        rc = set_segment(c, nshares, nums, pg.data(), out + g * oss, false, segs[g]);
        if (rc) return rc;
    }
    return sets_call(c, segs, nstripes, s, nullptr);
}

}  // namespace

void stop_builder(ec_ctx *c) { stop_builder_impl(c); }

}  // namespace capi
}  // namespace uplink_ec

extern "C" {

int ec_rebuild_segments_batched(const ec_ctx *cc, int nshares, const int *nums, const uint8_t *const *pieces,
                                size_t nstripes, size_t nseg, long long piece_seg_stride, long long out_seg_stride,
                                uint8_t *out, ec_stream stream) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c || !nums || !pieces || !out) return EC_ERR_INVALID_ARG;
    if (nshares < c->k) return EC_ERR_NOT_ENOUGH_SHARES;
    if (nstripes == 0 || nseg == 0) return EC_OK;
    DeviceGuard dg(c->device);
    return rebuild_async(c, nshares, nums, pieces, (int64_t)nstripes, (int64_t)nseg, piece_seg_stride, out_seg_stride,
                         out, (hipStream_t)stream);
}

// Segment g's shares are entries [off_g, off_g + nshares[g]) of nums / pieces.
static int sets_export(ec_ctx *c, size_t nseg, const int *nshares, const int *nums, const uint8_t *const *pieces,
                       size_t nstripes, uint8_t *const *outs, hipStream_t s, bool decode) {
    const int ess = c->ess;
    if (c->k > kMaxOps) return EC_ERR_UNSUPPORTED;
    // a call of many segments goes in passes of at most kPass (bounded staging per slot)
    constexpr size_t kPass = 64;
    std::vector<SetSeg> segs;
    std::vector<size_t> seg_of;  // segs[i] is segment seg_of[i] of the call
    std::vector<size_t> off(nseg + 1, 0);
    for (size_t g = 0; g < nseg; g++) off[g + 1] = off[g] + (size_t)std::max(nshares[g], 0);
    auto flush = [&]() -> int {
        std::vector<uint32_t> bad;
        int rc = sets_call(c, segs, (int64_t)nstripes, s, decode ? &bad : nullptr);
        // Decode: a segment whose syndromes are not all zero is corrected (in the
        // caller's pieces, as infectious corrects share.Data) and rebuilt on its own
        for (size_t i = 0; i < segs.size() && rc == EC_OK && decode; i++)
            if (bad[i]) {
                const size_t g = seg_of[i];
                rc = ec_decode_segments(c, nshares[g], nums + off[g], (uint8_t *const *)pieces + off[g], nstripes,
                                        outs[g], (ec_stream)s);
            }
        segs.clear();
        seg_of.clear();
        return rc;
    };
    for (size_t g = 0; g < nseg; g++) {
        const int ns = nshares[g];
        if (ns < c->k) return EC_ERR_NOT_ENOUGH_SHARES;
        bool bits = ess % 16 == 0 && aligned16(outs[g]) && (!decode || ns <= kMaxOps);
        for (int i = 0; i < ns; i++) bits = bits && aligned16(pieces[off[g] + i]);
        if (!bits) {  // byte kernel / more inputs than a launch takes: this segment on its own
            const int rc = decode ? ec_decode_segments(c, ns, nums + off[g], (uint8_t *const *)pieces + off[g], nstripes,
                                                       outs[g], (ec_stream)s)
                                  : rebuild_device(c, ns, nums + off[g], pieces + off[g], ess, (int64_t)nstripes, 1,
                                                   0, 0, outs[g], s);
            if (rc) return rc;
            continue;
        }
        segs.emplace_back();
        seg_of.push_back(g);
        if (int rc = set_segment(c, ns, nums + off[g], pieces + off[g], outs[g], decode, segs.back())) return rc;
        if (segs.size() == kPass)
            if (int rc = flush()) return rc;
    }
    return segs.empty() ? EC_OK : flush();
}

int ec_rebuild_segments_sets(const ec_ctx *cc, size_t nseg, const int *nshares, const int *nums,
                             const uint8_t *const *pieces, size_t nstripes, uint8_t *const *outs, ec_stream stream) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c || (nseg && (!nshares || !nums || !pieces || !outs))) return EC_ERR_INVALID_ARG;
    if (nseg == 0 || nstripes == 0) return EC_OK;
    for (size_t g = 0; g < nseg; g++)
        if (!outs[g]) return EC_ERR_INVALID_ARG;
    DeviceGuard dg(c->device);
    return sets_export(c, nseg, nshares, nums, pieces, nstripes, outs, (hipStream_t)stream, false);
}

int ec_decode_segments_sets(const ec_ctx *cc, size_t nseg, const int *nshares, const int *nums,
                            uint8_t *const *pieces, size_t nstripes, uint8_t *const *outs, ec_stream stream) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c || (nseg && (!nshares || !nums || !pieces || !outs))) return EC_ERR_INVALID_ARG;
    if (nseg == 0 || nstripes == 0) return EC_OK;
    for (size_t g = 0; g < nseg; g++)
        if (!outs[g]) return EC_ERR_INVALID_ARG;
    DeviceGuard dg(c->device);
    int rc = sets_export(c, nseg, nshares, nums, (const uint8_t *const *)pieces, nstripes, outs, (hipStream_t)stream,
                         true);
    if (rc == EC_OK && hipStreamSynchronize((hipStream_t)stream) != hipSuccess) rc = EC_ERR_DEVICE;
    return rc;
}

int ec_prepare_rebuild(const ec_ctx *cc, int nshares, const int *nums, int wait) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c || !nums) return EC_ERR_INVALID_ARG;
    DeviceGuard dg(c->device);
    std::vector<int> order, ids;
    if (int rc = choose_shares(c, nshares, nums, order, ids)) return rc;
    int m = 0;
    for (int i = 0; i < c->k; i++) m += ids[i] >= c->k;
    if (m == 0 || c->k > kMaxOps || c->ess % 16) return 0;  // (no code to make: copies, or the byte kernel)
    if (PlanPtr p = find_plan(c, ids); p && p->sl_ready.load(std::memory_order_acquire)) return 1;
    sl_request(c, ids);
    if (wait) {
        std::unique_lock<std::mutex> g(c->slb.mu);
        c->slb.cv.wait(g, [&] { return c->slb.pending.count(ids) == 0; });
    }
    PlanPtr p = find_plan(c, ids);
    return p && p->sl_ready.load(std::memory_order_acquire) ? 1 : 0;
}

}  // extern "C"
