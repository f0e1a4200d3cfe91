// C ABI (include/uplink_ec.h) over the HIP stripe kernels.
//
// Host-side responsibilities only: argument validation with the reference's
// error semantics, the choice of the k shares a Rebuild uses (infectious'
// sort + front/back rule), the k x k inversion of
// the decode matrix (once per share set, cached), and staging of
// host buffers for the per-stripe ErasureScheme calls.  Every byte of share
// data is produced by a GPU kernel.
//
// This file: the context, plans, encode, rebuild, per-stripe calls, the host
// pipeline, hashing, Decode with correction.  ec_sets.cpp: the share-set
// calls and the background builder of straight-line code.  ec_upload.cpp: the
// streamed upload.  ec_internal.hpp: what the three share.
#include "ec_internal.hpp"

#pragma GCC visibility push(hidden)  // (the library's internals: not in its dynamic symbol table)
namespace uplink_ec {
namespace capi {


constexpr size_t kMaxPlans = 64;
// coefficient rows are read as whole 32-bit words past the last row (OPW slots)
constexpr size_t kCoefPad = 64;

int round16(int x) { return (x + 15) & ~15; }

int hip_fail(hipError_t e) {
    if (e == hipSuccess) return EC_OK;
    fprintf(stderr, "uplink_ec: HIP error %d (%s)\n", (int)e, hipGetErrorString(e));
    return EC_ERR_DEVICE;
}


// At most kMaxWorkspaces per context: each has its own stream, and beyond a
// few the streams only share the device's hardware queues (GPU_MAX_HW_QUEUES,
// 4) while every new one costs a stream and pinned memory.  Callers beyond
// that wait in arrival order and get a workspace handed over on release, so no
// caller starves (300 threads of per-stripe calls: DESIGN.md §5a).
constexpr size_t kMaxWorkspaces = 8;

Workspace *acquire_ws(ec_ctx *c, size_t need, size_t host_need = 0) {
    Workspace *w = nullptr;
    {
        std::unique_lock<std::mutex> g(c->mu);
        if (!c->free_ws.empty()) {
            w = c->free_ws.back();
            c->free_ws.pop_back();
        } else if (c->all_ws.size() < kMaxWorkspaces) {
            c->all_ws.emplace_back(new Workspace());
            w = c->all_ws.back().get();
        } else {
            WsWaiter me;
            c->ws_waiters.push_back(&me);
            me.cv.wait(g, [&] { return me.w != nullptr; });
            w = me.w;
        }
    }
    if (!w->stream && hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess) w->stream = nullptr;
    if (w->cap < need) {
        if (w->d_buf) (void)hipFree(w->d_buf);
        w->d_buf = nullptr;
        w->cap = 0;
        size_t cap = std::max(need, (size_t)1 << 20);
        if (hipMalloc(&w->d_buf, cap) == hipSuccess) w->cap = cap;
    }
    if (host_need && w->h_cap < host_need) {
        if (w->h_buf) (void)hipHostFree(w->h_buf);
        w->h_buf = nullptr;
        w->h_cap = 0;
        size_t cap = std::max(host_need, (size_t)1 << 20);
        if (hipHostMalloc((void **)&w->h_buf, cap, hipHostMallocDefault) == hipSuccess) w->h_cap = cap;
    }
    return w;
}

// Staging above this size is given back after use rather than kept for the
// life of the context (a burst of large per-stripe calls would otherwise pin it).
constexpr size_t kWsKeepBytes = (size_t)32 << 20;

void shrink_ws(Workspace *w) {
    if (w->cap > kWsKeepBytes && w->d_buf) {
        if (w->stream) (void)hipStreamSynchronize(w->stream);
        (void)hipFree(w->d_buf);
        w->d_buf = nullptr;
        w->cap = 0;
    }
    if (w->h_cap > kWsKeepBytes && w->h_buf) {
        (void)hipHostFree(w->h_buf);
        w->h_buf = nullptr;
        w->h_cap = 0;
    }
}

void release_ws(ec_ctx *c, Workspace *w) {
    shrink_ws(w);
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->ws_waiters.empty()) {
        WsWaiter *next = c->ws_waiters.front();
        c->ws_waiters.pop_front();
        next->w = w;
        next->cv.notify_one();
        return;
    }
    c->free_ws.push_back(w);
}

void fill_geometry(RsArgs &a, int ess, int64_t nstripes, int64_t nseg) {
    a.ess = ess;
    a.cps = ess / 16;
    a.nstripes = nstripes;
    a.chunks_per_seg = nstripes * (ess / 16);
    a.tiles_per_seg = (a.chunks_per_seg + 127) / 128;
    a.total_tiles = a.tiles_per_seg * nseg;
    a.blocks_per_seg = (a.chunks_per_seg + 63) / 64;
    a.total_blocks = a.blocks_per_seg * nseg;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// The byte ranges a launch may touch, from its geometry (RsArgs::chk_*).
void set_extents(RsArgs &a, int64_t nseg, uint32_t *chk) {
    a.chk_flag = chk;
    int64_t ilo = INT64_MAX, ihi = 0, olo = INT64_MAX, ohi = 0;
    for (int j = 0; j < a.nin; j++) {
        ilo = std::min(ilo, a.in_off[j]);
        ihi = std::max(ihi, a.in_off[j]);
        if (a.copy_off[j] >= 0) olo = std::min(olo, a.copy_off[j]), ohi = std::max(ohi, a.copy_off[j]);
    }
    for (int r = 0; r < a.nout; r++) olo = std::min(olo, a.out_off[r]), ohi = std::max(ohi, a.out_off[r]);
    const int64_t last = nseg > 0 && a.nstripes > 0;
    a.chk_in_lo = a.in_base + (ilo == INT64_MAX ? 0 : ilo);
    a.chk_in_hi = a.in_base + ihi + last * ((nseg - 1) * a.in_seg_stride + (a.nstripes - 1) * a.in_stripe_stride + a.ess);
    a.chk_out_lo = a.out_base + (olo == INT64_MAX ? 0 : olo);
    a.chk_out_hi =
        a.out_base + ohi + last * ((nseg - 1) * a.out_seg_stride + (a.nstripes - 1) * a.out_stripe_stride + a.ess);
}

// Upload M (rows x nin, row-major) and its leaf-address tables; synchronous.
int build_plan(ec_ctx *c, std::vector<int> key, const uint8_t *M, int rows, int nin, PlanPtr *out) {
    PlanPtr p = std::make_shared<MatPlan>();
    p->arena = c->arena;
    p->marks = c->marks;
    p->key = std::move(key);
    p->rows = rows;
    p->nin = nin;
    p->M.assign(M, M + (size_t)rows * nin);
    p->coef_ld = round16(std::max(rows, 1));
    std::vector<uint8_t> coef((size_t)nin * p->coef_ld + kCoefPad, 0);
    for (int r = 0; r < rows; r++)
        for (int j = 0; j < nin; j++) coef[(size_t)j * p->coef_ld + r] = M[(size_t)r * nin + j];
    std::lock_guard<std::mutex> g(c->setup_mu);
    p->coef_bytes = coef.size();
    p->d_coef = p->arena->alloc(coef.size());
    if (!p->d_coef) return hip_fail(hipErrorOutOfMemory);
    HIP_TRY(hipMemcpyAsync(p->d_coef, coef.data(), coef.size(), hipMemcpyHostToDevice, c->setup));
    for (int r0 = 0; r0 < std::max(rows, 1); r0 += kMaxOps) {
        RsArgs t{};
        t.coef = p->d_coef + r0;
        t.coef_ld = p->coef_ld;
        t.nin = nin;
        t.nout = std::min(kMaxOps, rows - r0);
        uint64_t *tgt = (uint64_t *)p->arena->alloc(jt_targets_bytes(t));
        if (!tgt) return hip_fail(hipErrorOutOfMemory);
        p->d_tgt.push_back(tgt);
        p->tgt_bytes.push_back(jt_targets_bytes(t));
        HIP_TRY(launch_jt_targets(t, tgt, c->setup));
    }
    HIP_TRY(hipStreamSynchronize(c->setup));  // `coef` (pageable) is consumed before it goes away
    *out = p;
    return EC_OK;
}

// Cached plan for `key`, built from make_matrix() on a miss.
template <typename F>
int cached_plan(ec_ctx *c, const std::vector<int> &key, F &&make_matrix, PlanPtr *out, int nin = -1) {
    {
        std::lock_guard<std::mutex> g(c->mu);
        for (auto it = c->plans.begin(); it != c->plans.end(); ++it) {
            if ((*it)->key == key) {
                c->plans.splice(c->plans.begin(), c->plans, it);
                *out = c->plans.front();
                return EC_OK;
            }
        }
    }
    std::vector<uint8_t> M;
    std::vector<int> missing;
    int rows = 0;
    int rc = make_matrix(M, rows, missing);
    if (rc) return rc;
    PlanPtr p;
    rc = build_plan(c, key, M.data(), rows, nin < 0 ? c->k : nin, &p);
    if (rc) return rc;
    p->missing = std::move(missing);
    std::vector<PlanPtr> reaped;
    {
        std::lock_guard<std::mutex> g(c->mu);
        c->plans.push_front(p);
        // an evicted plan may still be read by launches in flight on callers'
        // streams: it waits in the graveyard until its launches are known
        // complete (MatPlan::idle, no wait); past kMaxPlans waiting, the device
        // is synchronised once and all of them go
        while (c->plans.size() > kMaxPlans) {
            c->graveyard.push_back(c->plans.back());
            c->plans.pop_back();
        }
        for (auto it = c->graveyard.begin(); it != c->graveyard.end();) {
            if ((*it)->idle()) {
                reaped.push_back(*it);
                it = c->graveyard.erase(it);
            } else {
                ++it;
            }
        }
        if (c->graveyard.size() > kMaxPlans) {
            (void)hipDeviceSynchronize();
            for (auto &x : c->graveyard) reaped.push_back(x);
            c->graveyard.clear();
        }
    }
    reaped.clear();  // (destroyed outside the lock)
    *out = p;
    return EC_OK;
}

// Plan of the parity rows k..n-1 (encode for (k, n) without a compile-time kernel)
int parity_plan(ec_ctx *c, PlanPtr *out) {
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (c->enc_parity) {
            *out = c->enc_parity;
            return EC_OK;
        }
    }
    PlanPtr p;
    int rc = build_plan(c, {-3}, c->G.data() + (size_t)c->k * c->k, c->n - c->k, c->k, &p);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->enc_parity) c->enc_parity = p;
    *out = c->enc_parity;
    return EC_OK;
}

// Plan of row `num` of G (ErasureScheme.EncodeSingle)
int row_plan(ec_ctx *c, int num, PlanPtr *out) {
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (c->enc_row[num]) {
            *out = c->enc_row[num];
            return EC_OK;
        }
    }
    PlanPtr p;
    int rc = build_plan(c, {-4, num}, c->G.data() + (size_t)num * c->k, 1, c->k, &p);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->enc_row[num]) c->enc_row[num] = p;
    *out = c->enc_row[num];
    return EC_OK;
}

// Checked build: wait for the launch just made and fail if a kernel skipped an
// access outside the launch's declared ranges (rs_tile.hpp in_range).
int after_launch(uint32_t *chk, hipStream_t s) {
#ifdef UPLINK_EC_CHECKED
    uint32_t site = 0;
    HIP_TRY(hipMemcpyAsync(&site, chk, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (site) {
        fprintf(stderr, "uplink_ec checked: a kernel addressed memory outside its launch's ranges (site %u)\n", site);
        return EC_ERR_INVALID_ARG;
    }
#else
    (void)chk, (void)s;
#endif
    return EC_OK;
}

// A zeroed work counter for one encoder launch on stream s (slot in *slot, the
// launch's sequence number in *seq and the slot's completion word in *done;
// queue_done after the launch).  nullptr when none can be had without waiting
// for another stream: the kernel then assigns its tiles statically, with
// identical results.  (A stream handle is taken to name one stream while work
// queued on it is in flight.)
uint32_t *queue_take(ec_ctx *c, hipStream_t s, int *slot, uint32_t *seq, uint32_t **done) {
    QueueRing &q = c->qring;
    std::lock_guard<std::mutex> g(q.mu);
    if (!q.d) {
        const size_t bytes = sizeof(uint32_t) * QueueRing::kStride * QueueRing::kSlots;
        if (hipMalloc(&q.d, bytes) != hipSuccess) {
            q.d = nullptr;
            return nullptr;
        }
        if (hipHostMalloc((void **)&q.h_done, sizeof(uint32_t) * QueueRing::kSlots,
                          hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            q.h_done = nullptr;
            (void)hipFree(q.d);
            q.d = nullptr;
            return nullptr;
        }
        memset(q.h_done, 0, sizeof(uint32_t) * QueueRing::kSlots);
        if (hipMemset(q.d, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            (void)hipHostFree(q.h_done);
            (void)hipFree(q.d);
            q.d = nullptr, q.h_done = nullptr;
            return nullptr;
        }
    }
    int pick = -1;
    // the slot this stream used last: its previous launch precedes this one in stream order
    for (int i = 0; i < QueueRing::kSlots && pick < 0; i++)
        if (q.used[i] && !q.busy[i] && q.owner[i] == s) pick = i;
    // else a fresh slot, or one whose latest launch (on any stream) has finished
    for (int i = 0; i < QueueRing::kSlots && pick < 0; i++)
        if (!q.busy[i] && (!q.used[i] || q.done(i))) pick = i;
    if (pick < 0) return nullptr;
    q.busy[pick] = true;
    *slot = pick;
    *seq = q.seq[pick] + 1;
    *done = q.h_done + pick;
    return q.d + (size_t)pick * QueueRing::kStride;
}

void queue_done(ec_ctx *c, hipStream_t s, int slot, uint32_t seq, bool launched) {
    QueueRing &q = c->qring;
    std::lock_guard<std::mutex> g(q.mu);
    if (launched) {
        q.used[slot] = true;
        q.owner[slot] = s;
        q.seq[slot] = seq;
    }
    q.busy[slot] = false;
}


// Whole-segment encodes with at most this many parity rows run on the
// parity plan's straight-line code instead of a compile-time encoder: one
// pass of the runtime-matrix kernel (up to 4 waves of 8 rows), 16 waves per
// CU that all load and compute, measured equal or faster for RS(20,50),
// (30,60), (50,80) (parity-only 3-17 % faster); with 40 and 51 parity rows
// (RS(20,60), RS(29,80)) the compile-time encoder stays ahead.
constexpr int kSlEncodeMaxRows = 32;

// (EC_BODY_STRAIGHT_LINE: every encode the runtime-matrix kernel takes.)
bool sl_encoder(const ec_ctx *c) {
    return c->ess % 16 == 0 && c->n > c->k && c->k <= kMaxOps && c->n - c->k <= kMaxOps &&
           (c->body == EC_BODY_STRAIGHT_LINE || (c->body == EC_BODY_AUTO && c->n - c->k <= kSlEncodeMaxRows));
}

// Make the plan's straight-line module (once; on failure the plan keeps
// using the jump table).  Synchronous, on the context's setup stream.
void ensure_sl(ec_ctx *c, MatPlan &plan) {
    std::lock_guard<std::mutex> g(plan.sl_mu);
    if (plan.sl_tried) return;
    plan.sl_tried = true;
    if (plan.rows < 1 || plan.rows > kMaxOps || plan.nin < 1 || plan.nin > kMaxOps) return;
    std::vector<uint32_t> code(sl::kRegionWords, 0xbf810000u);  // s_endpgm
    std::vector<uint32_t> offs;
    const size_t used = sl::generate(plan.M.data(), plan.rows, plan.nin, code.data(), code.size(), offs);
    if (!used) return;  // does not fit
    size_t roff = 0, rwords = 0;
    const double t0 = log_ms();
    std::vector<uint8_t> img = sl::template_image(used, &roff, &rwords);
    memcpy(img.data() + roff + 16, code.data() + 4, (used - 4) * 4);  // the marker words stay
    std::lock_guard<std::mutex> gs(c->setup_mu);
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    uint64_t *d = nullptr;
    const size_t dbytes = (offs.size() + 1) * sizeof(uint64_t);
    auto fail = [&](hipError_t e) {
        hip_fail(e);
        if (d) plan.arena->release((uint8_t *)d, dbytes);
        if (mod) (void)hipModuleUnload(mod);
    };
    hipError_t e = hipModuleLoadData(&mod, img.data());
    if (e == hipSuccess) e = hipModuleGetFunction(&fn, mod, "rs_sl_where");
    if (e == hipSuccess && !(d = (uint64_t *)plan.arena->alloc(dbytes))) e = hipErrorOutOfMemory;
    if (e != hipSuccess) return fail(e);
    void *args[] = {&d};
    uint64_t base = 0;
    e = hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, c->setup, args, nullptr);
    if (e == hipSuccess) e = hipMemcpyAsync(&base, d, sizeof(base), hipMemcpyDeviceToHost, c->setup);
    if (e == hipSuccess) e = hipStreamSynchronize(c->setup);
    if (e != hipSuccess || base == 0) return fail(e == hipSuccess ? hipErrorInvalidValue : e);
    std::vector<uint64_t> tab(offs.size());
    for (size_t i = 0; i < offs.size(); i++) tab[i] = offs[i] == sl::kNoSegment ? 0 : base + offs[i];
    e = hipMemcpyAsync(d, tab.data(), tab.size() * sizeof(uint64_t), hipMemcpyHostToDevice, c->setup);
    if (e == hipSuccess) e = hipStreamSynchronize(c->setup);
    if (e != hipSuccess) return fail(e);
    plan.sl_mod = mod;
    plan.d_sl = d;
    plan.sl_bytes = dbytes;
    plan.sl_ready.store(true, std::memory_order_release);
    ec_logf("straight-line module: %d rows x %d inputs, %zu words of code, made and loaded in %.1f ms", plan.rows,
         plan.nin, used, log_ms() - t0);
}

// Launch the product described by `a` with the rows of `plan` (out_off gives
// every row's offset; more than kMaxOps rows go in several launches, copies
// in the first one only).
int run_matmul(ec_ctx *c, RsArgs a, const int64_t *out_off, MatPlan &plan, int64_t nseg, bool bitsliced,
               hipStream_t s) {
    const int total_rows = plan.rows;
    int done = 0, blk = 0;
    do {
        const int rows = std::min(kMaxOps, total_rows - done);
        a.nout = rows;
        a.nin = plan.nin;
        a.coef = plan.d_coef + done;
        a.coef_ld = plan.coef_ld;
        a.jt_tgt = bitsliced ? plan.d_tgt[blk] : nullptr;
        for (int r = 0; r < rows; r++) a.out_off[r] = out_off[done + r];
        if (done > 0)
            for (int j = 0; j < a.nin; j++) a.copy_off[j] = -1;
        set_extents(a, nseg, c->d_chk);
        // EC_BODY_AUTO: a plan's first launch runs the jump table, the straight-line
        // code is made for its second (a share set seen once -- a download's
        // segment, most often -- never pays the code generation and module load,
        // ~0.9 ms against ~50 us of kernel time per segment)
        const bool want_sl = bitsliced && total_rows <= kMaxOps && c->body != EC_BODY_JUMP_TABLE &&
                             (c->body == EC_BODY_STRAIGHT_LINE ||
                              (a.total_tiles >= kSlMinTiles &&
                               (plan.launches.load() > 0 || plan.sl_ready.load(std::memory_order_acquire))));
        if (want_sl) ensure_sl(c, plan);
        if (want_sl && plan.sl_ready.load(std::memory_order_acquire)) {
            a.jt_tgt = plan.d_sl;
            c->last_body = EC_BODY_STRAIGHT_LINE;
            HIP_TRY(launch_matmul_sl(a, 0, s));
        } else if (bitsliced) {
            c->last_body = EC_BODY_JUMP_TABLE;
            HIP_TRY(launch_matmul_generic(a, 0, s));
        } else {
            const int64_t keep = a.total_tiles;
            a.total_tiles = nseg;  // byte kernel: total_tiles carries the segment count
            HIP_TRY(launch_matmul_bytes(a, s));
            a.total_tiles = keep;
        }
        plan.note_use(s);
        plan.launches++;
        if (int rc = after_launch(c->d_chk, s)) return rc;
        done += rows;
        blk++;
    } while (done < total_rows);
    return EC_OK;
}

// infectious Rebuild share choice: sort by number, then for i in 0..k-1 take
// the front share if its number == i else take from the back.
int choose_shares(const ec_ctx *c, int nshares, const int *nums, std::vector<int> &order_out,
                  std::vector<int> &ids_out) {
    if (nshares < c->k) return EC_ERR_NOT_ENOUGH_SHARES;
    std::vector<int> order(nshares);
    for (int i = 0; i < nshares; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return nums[a] < nums[b]; });
    int b = 0, e = nshares - 1;
    order_out.clear();
    ids_out.clear();
    for (int i = 0; i < c->k; i++) {
        int pick;
        if (nums[order[b]] == i) pick = order[b++];
        else pick = order[e--];
        if (nums[pick] >= c->n || nums[pick] < 0) return EC_ERR_INVALID_SHARE;
        order_out.push_back(pick);
        ids_out.push_back(nums[pick]);
    }
    return EC_OK;
}

// Decode plan for the chosen ids (one inversion per share set).
int get_plan(ec_ctx *c, const std::vector<int> &ids, PlanPtr *out) {
    return cached_plan(c, ids, [&](std::vector<uint8_t> &M, int &rows, std::vector<int> &missing) {
        const int k = c->k;
        std::vector<uint8_t> m((size_t)k * k, 0);
        for (int i = 0; i < k; i++) {
            if (ids[i] < k) m[(size_t)i * k + i] = 1;
            else memcpy(&m[(size_t)i * k], &c->G[(size_t)ids[i] * k], k);
        }
        if (!gf_invert(m.data(), k)) return EC_ERR_SINGULAR;
        for (int i = 0; i < k; i++)
            if (ids[i] >= k) missing.push_back(i);
        rows = (int)missing.size();
        M.assign((size_t)std::max(rows, 1) * k, 0);
        for (int r = 0; r < rows; r++) memcpy(&M[(size_t)r * k], &m[(size_t)missing[r] * k], k);
        return EC_OK;
    }, out);
}

// The rebuild of nseg segments from the chosen shares (order: their indices in
// `pieces`, ids: their numbers) with a decode plan.
int rebuild_with_plan(ec_ctx *c, MatPlan &plan, const std::vector<int> &order, const std::vector<int> &ids,
                      const uint8_t *const *pieces, int ess, int64_t nstripes, int64_t nseg, int64_t piece_seg_stride,
                      int64_t out_seg_stride, uint8_t *out, hipStream_t s) {
    const int k = c->k;
    RsArgs a{};
    const uint8_t *base = pieces[order[0]];
    for (int i = 0; i < k; i++) base = std::min(base, pieces[order[i]]);
    a.in_base = base;
    a.out_base = out;
    a.in_stripe_stride = ess;
    a.out_stripe_stride = (int64_t)k * ess;
    a.in_seg_stride = piece_seg_stride;
    a.out_seg_stride = out_seg_stride;
    bool bits = (ess % 16) == 0 && aligned16(out);
    for (int i = 0; i < k; i++) {
        const uint8_t *p = pieces[order[i]];
        a.in_off[i] = p - base;
        a.copy_off[i] = ids[i] < k ? (int64_t)ids[i] * ess : -1;
        bits = bits && aligned16(p);
    }
    std::vector<int64_t> out_off(std::max<size_t>(plan.missing.size(), 1));
    for (size_t r = 0; r < plan.missing.size(); r++) out_off[r] = (int64_t)plan.missing[r] * ess;
    fill_geometry(a, ess, nstripes, nseg);
    if (!bits) a.cps = 1;
    return run_matmul(c, a, out_off.data(), plan, nseg, bits, s);
}

// Core rebuild: device pointers of the nshares pieces, nstripes stripes of
// share size `ess`, out stripe-major; batched over nseg with strides.  The
// plan is made here if the context has none (synchronous: the per-stripe
// calls, the host pipeline and Decode's correction path, which all wait anyway;
// the asynchronous batched rebuild goes through rebuild_async).
int rebuild_device(ec_ctx *c, int nshares, const int *nums, const uint8_t *const *pieces, int ess, int64_t nstripes,
                   int64_t nseg, int64_t piece_seg_stride, int64_t out_seg_stride, uint8_t *out, hipStream_t s) {
    std::vector<int> order, ids;
    int rc = choose_shares(c, nshares, nums, order, ids);
    if (rc) return rc;
    if (c->k > kMaxOps) return EC_ERR_UNSUPPORTED;
    PlanPtr plan;
    rc = get_plan(c, ids, &plan);
    if (rc) return rc;
    return rebuild_with_plan(c, *plan, order, ids, pieces, ess, nstripes, nseg, piece_seg_stride, out_seg_stride, out,
                             s);
}

}  // namespace capi
}  // namespace uplink_ec
#pragma GCC visibility pop

extern "C" {


int ec_set_body(ec_ctx *c, int body) {
    if (!c || body < EC_BODY_AUTO || body > EC_BODY_STRAIGHT_LINE) return EC_ERR_INVALID_ARG;
    c->body = body;
    return EC_OK;
}

int ec_last_body(const ec_ctx *c) { return c ? c->last_body : EC_BODY_AUTO; }

int ec_encoder_queue_stats(const ec_ctx *c, unsigned long long *queued, unsigned long long *static_tiles) {
    if (!c || !queued || !static_tiles) return EC_ERR_INVALID_ARG;
    *queued = c->q_taken.load(std::memory_order_relaxed);
    *static_tiles = c->q_static.load(std::memory_order_relaxed);
    return EC_OK;
}

// UPLINK_EC_BUILD_ID: generated by the Makefile into the build directory
// (build_id.inc) from a digest of the sources, generators and flags.
const char *ec_build_id(void) {
    static const char id[] =
#include "build_id.inc"
        ;
    return id;
}

int ec_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ec_set_device(int device) { return hip_fail(hipSetDevice(device)); }

int ec_create(int k, int n, int ess, ec_ctx **out) {
    if (!out) return EC_ERR_INVALID_ARG;
    *out = nullptr;
    if (k <= 0 || n <= 0 || k > 256 || n > 256 || k > n) return EC_ERR_PARAMS;
    if (ess <= 0) return EC_ERR_INVALID_ARG;
    if (ec_device_count() <= 0) {
        fprintf(stderr, "uplink_ec: no HIP device available\n");
        return EC_ERR_DEVICE;
    }
    std::unique_ptr<ec_ctx> c(new ec_ctx());
    c->k = k;
    c->n = n;
    c->ess = ess;
    HIP_TRY(hipGetDevice(&c->device));
    c->G.resize((size_t)n * k);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < k; j++) c->G[(size_t)i * k + j] = gen_entry(k, i, j);
    c->enc_row.resize(n);
    HIP_TRY(hipStreamCreateWithFlags(&c->setup, hipStreamNonBlocking));
    // for the share-set pass (rs_sets_prep): where the jump table's leaves are
    HIP_TRY(jt_table_base_addr(&c->jt_base, c->setup));
    // Scratch of ec_hash_segments / ec_blake3_pieces comes from the default pool
    // in stream order: keep the pool's memory mapped between calls instead of
    // returning it to the driver at every synchronisation.
    hipMemPool_t pool = nullptr;
    if (hipDeviceGetDefaultMemPool(&pool, c->device) == hipSuccess && pool) {
        uint64_t keep = UINT64_MAX;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
#ifdef UPLINK_EC_CHECKED
    HIP_TRY(hipMalloc(&c->d_chk, 4));
    HIP_TRY(hipMemset(c->d_chk, 0, 4));
#endif
    if (const char *e = getenv("UPLINK_EC_SETS_MERGE")) c->sets_merge = atoi(e) != 0;
    if (const char *e = getenv("UPLINK_EC_SETS_STAGE_DMA")) c->sets_stage_dma = atoi(e) != 0;
    if (const char *e = getenv("UPLINK_EC_SETS_ONE")) c->sets_one = atoi(e) != 0;
    configure_rebuild(getenv("UPLINK_EC_REBUILD_DEPTH") ? atoi(getenv("UPLINK_EC_REBUILD_DEPTH")) : 1);
    if (const char *f = getenv("UPLINK_EC_FAULT_SINGLE"))
        if (sscanf(f, "max=%d,num=%d", &c->fault_max_batch, &c->fault_fail_num) != 2) c->fault_max_batch = 0;
    *out = c.release();
    return EC_OK;
}

void ec_destroy(ec_ctx *c) {
    if (!c) return;
    DeviceGuard dg(c->device);
    stop_builder(c);  // (before anything its plan in hand uses goes)
    // share-set slots still read by launches in flight: wait for the device once
    {
        bool busy = false;
        std::lock_guard<std::mutex> g(c->sets.mu);
        for (auto &x : c->sets.slots)  // (a dead slot's launches before the failed one may still run)
            busy = busy || x->dead || __atomic_load_n(x->h_words, __ATOMIC_ACQUIRE) != x->seq;
        if (busy) (void)hipDeviceSynchronize();
        c->sets.slots.clear();
    }
    for (int s = 0; s < HostPipe::kSlots; s++) {
        if (c->pipe.st[s]) (void)hipStreamSynchronize(c->pipe.st[s]), (void)hipStreamDestroy(c->pipe.st[s]);
        if (c->pipe.d_in[s]) (void)hipFree(c->pipe.d_in[s]);
        if (c->pipe.d_out[s]) (void)hipFree(c->pipe.d_out[s]);
    }
    c->upload_free.clear();  // (UploadSlot's destructor waits for and frees each)
    for (auto &w : c->all_ws) {
        if (w->stream) (void)hipStreamSynchronize(w->stream), (void)hipStreamDestroy(w->stream);
        if (w->d_buf) (void)hipFree(w->d_buf);
        if (w->h_buf) (void)hipHostFree(w->h_buf);
    }
    c->plans.clear();
    c->graveyard.clear();
    c->enc_parity.reset();
    c->enc_row.clear();
    if (c->setup) (void)hipStreamSynchronize(c->setup), (void)hipStreamDestroy(c->setup);
    if (c->d_chk) (void)hipFree(c->d_chk);
    // a counter slot whose latest launch has not finished may still be in use on a caller's
    // stream: then wait for the device before the counters are freed
    bool pending = false;
    for (int i = 0; i < QueueRing::kSlots && c->qring.h_done; i++) pending = pending || (c->qring.used[i] && !c->qring.done(i));
    if (pending) (void)hipDeviceSynchronize();
    if (c->qring.d) (void)hipFree(c->qring.d);
    if (c->qring.h_done) (void)hipHostFree(c->qring.h_done);
    delete c;
}

int ec_required(const ec_ctx *c) { return c ? c->k : EC_ERR_INVALID_ARG; }
int ec_total(const ec_ctx *c) { return c ? c->n : EC_ERR_INVALID_ARG; }
int ec_share_size(const ec_ctx *c) { return c ? c->ess : EC_ERR_INVALID_ARG; }
int ec_stripe_size(const ec_ctx *c) { return c ? c->ess * c->k : EC_ERR_INVALID_ARG; }

int ec_generator(const ec_ctx *c, uint8_t *out) {
    if (!c || !out) return EC_ERR_INVALID_ARG;
    memcpy(out, c->G.data(), c->G.size());
    return EC_OK;
}

const char *ec_strerror(int code) {
    switch (code) {
        case EC_OK: return "ok";
        case EC_ERR_PARAMS: return "requires 1 <= k <= n <= 256";
        case EC_ERR_NUM_NEGATIVE: return "num must be non-negative";
        case EC_ERR_NUM_RANGE: return "num must be less than %d";
        case EC_ERR_INPUT_LENGTH: return "input length must be a multiple of %d";
        case EC_ERR_OUTPUT_LENGTH: return "output length must be %d";
        case EC_ERR_NOT_ENOUGH_SHARES: return "not enough shares";
        case EC_ERR_TOO_MANY_ERRORS: return "too many errors to reconstruct";
        case EC_ERR_INVALID_SHARE: return "invalid share id: %d";
        case EC_ERR_SINGULAR: return "matrix is singular";
        case EC_ERR_INVALID_ARG: return "invalid argument";
        case EC_ERR_DEVICE: return "HIP device error";
        case EC_ERR_UNSUPPORTED: return "unsupported parameters";
        case EC_ERR_SHARE_SIZE: return "shares must all have the same length";
        case EC_ERR_AUTH: return "cipher: message authentication failed";
        default: return "unknown error";
    }
}

int ec_format_error(const ec_ctx *c, int code, long long arg, char *buf, size_t len) {
    const char *fmt = ec_strerror(code);
    long long v = arg;
    if (code == EC_ERR_NUM_RANGE && c) v = c->n;
    if (code == EC_ERR_INPUT_LENGTH && c) v = c->k;
    int r = snprintf(buf, len, fmt, v);
    return r;
}

const char *ec_encode_kernel_name(const ec_ctx *c) {
    if (!c) return "";
    if (c->ess % 16) return "bytes";
    if (c->n == c->k) return "copy";
    if (sl_encoder(c)) return "straight-line";
    DeviceGuard dg(c->device);
    const EncoderKernel *e = find_encoder(c->k, c->n, false, false);  // (a query: starts no compile)
    return e ? (e->jit ? "special-jit" : "special") : "generic";
}

int ec_prepare_encoder(const ec_ctx *c, int wait) {
    if (!c) return EC_ERR_INVALID_ARG;
    if (c->n == c->k || !encoder_supported(c->k, c->n)) return 0;
    DeviceGuard dg(c->device);
    return find_encoder(c->k, c->n, wait != 0) ? 1 : 0;
}

// Encode stripes [s0, s1) of nseg segments of nstripes stripes each: the
// pieces keep their full layout ([seg][rows][nstripes*ess]), the range
// writes its part of every piece (used to pipeline one segment through PCIe
// in chunks of stripes).
}  // extern "C"
namespace uplink_ec {
namespace capi {
int encode_range(ec_ctx *c, const uint8_t *segs, size_t nseg, size_t nstripes, size_t s0, size_t s1,
                        uint8_t *pieces, int flags, hipStream_t s, bool shape_probe) {
    if (!c || !segs || !pieces) return EC_ERR_INVALID_ARG;
    if (nseg == 0 || s1 <= s0) return EC_OK;
    const int k = c->k, n = c->n, ess = c->ess;
    if (k > kMaxOps) return EC_ERR_UNSUPPORTED;
    const bool parity_only = (flags & EC_FLAG_PARITY_ONLY) != 0;
    const int64_t piece_len = (int64_t)nstripes * ess;
    segs += s0 * (size_t)k * ess;
    pieces += s0 * (size_t)ess;
    RsArgs a{};
    a.in_base = segs;
    a.out_base = pieces;
    a.in_stripe_stride = (int64_t)k * ess;
    a.out_stripe_stride = ess;
    a.in_seg_stride = (int64_t)nstripes * k * ess;
    a.out_seg_stride = (int64_t)(parity_only ? n - k : n) * piece_len;
    a.nin = k;
    a.nout = n - k;
    for (int j = 0; j < k; j++) {
        a.in_off[j] = (int64_t)j * ess;
        a.copy_off[j] = parity_only ? -1 : (int64_t)j * piece_len;
    }
    std::vector<int64_t> out_off(std::max(n - k, 1));
    for (int r = 0; r < n - k; r++) out_off[r] = (int64_t)(parity_only ? r : k + r) * piece_len;
    for (int r = 0; r < std::min(n - k, kMaxOps); r++) a.out_off[r] = out_off[r];
    fill_geometry(a, ess, (int64_t)(s1 - s0), (int64_t)nseg);
    const bool bits = (ess % 16) == 0 && aligned16(segs) && aligned16(pieces);
    if (shape_probe && (!bits || !shape_probe_encoder(k, n))) return EC_ERR_UNSUPPORTED;
    if (n == k) {  // replication of the data only: copies, no parity rows
        if (parity_only) return EC_OK;
    } else if (bits) {
        // few parity rows: the runtime-matrix kernel with the parity plan's
        // straight-line code (run_matmul picks it for launches this large)
        const bool sl = sl_encoder(c) && (c->body == EC_BODY_STRAIGHT_LINE || a.total_tiles >= kSlMinTiles);
        // (a run-time compile of this code's encoder is started only by launches
        // large enough to pay for it: never by per-stripe or few-stripe work)
        const EncoderKernel *ek = shape_probe ? shape_probe_encoder(k, n)
                                  : sl        ? nullptr
                                              : find_encoder(c->k, c->n, false, a.total_tiles >= kJitMinTiles);
        if (ek) {
            a.coef = nullptr;
            set_extents(a, (int64_t)nseg, c->d_chk);
            int slot = -1;
            a.queue = queue_take(c, s, &slot, &a.queue_seq, &a.queue_host_done);
            (a.queue ? c->q_taken : c->q_static).fetch_add(1, std::memory_order_relaxed);
            const hipError_t e = launch_encode_special(*ek, a, 0, s);
            if (slot >= 0) queue_done(c, s, slot, a.queue_seq, e == hipSuccess);
            HIP_TRY(e);
            return after_launch(c->d_chk, s);
        }
    }
    if (!bits) a.cps = 1;
    PlanPtr plan;
    int rc = parity_plan(c, &plan);
    if (rc) return rc;
    return run_matmul(c, a, out_off.data(), *plan, (int64_t)nseg, bits, s);
}
}  // namespace capi
}  // namespace uplink_ec
extern "C" {

int ec_encode_segments(const ec_ctx *cc, const uint8_t *segs, size_t nseg, size_t nstripes, uint8_t *pieces,
                       int flags, ec_stream stream) {
    if (!cc) return EC_ERR_INVALID_ARG;
    DeviceGuard dg(cc->device);
    return encode_range(const_cast<ec_ctx *>(cc), segs, nseg, nstripes, 0, nstripes, pieces, flags,
                        (hipStream_t)stream);
}

int ec_encode_shape_probe(const ec_ctx *cc, const uint8_t *segs, size_t nseg, size_t nstripes, uint8_t *pieces,
                          int flags, ec_stream stream) {
    if (!cc) return EC_ERR_INVALID_ARG;
    DeviceGuard dg(cc->device);
    return encode_range(const_cast<ec_ctx *>(cc), segs, nseg, nstripes, 0, nstripes, pieces, flags,
                        (hipStream_t)stream, true);
}

int ec_rebuild_segments(const ec_ctx *c, int nshares, const int *nums, const uint8_t *const *pieces,
                        size_t nstripes, uint8_t *out, ec_stream stream) {
    return ec_rebuild_segments_batched(c, nshares, nums, pieces, nstripes, 1, 0, 0, out, stream);
}

// ---------------------------------------------------------------- host pipeline
static int pipe_reserve(ec_ctx *c, size_t in_bytes, size_t out_bytes) {
    HostPipe &p = c->pipe;
    for (int s = 0; s < HostPipe::kSlots; s++)
        if (!p.st[s]) HIP_TRY(hipStreamCreateWithFlags(&p.st[s], hipStreamNonBlocking));
    if (p.in_cap < in_bytes) {
        for (int s = 0; s < HostPipe::kSlots; s++) {
            if (p.d_in[s]) (void)hipFree(p.d_in[s]);
            p.d_in[s] = nullptr;
            HIP_TRY(hipMalloc(&p.d_in[s], in_bytes));
        }
        p.in_cap = in_bytes;
    }
    if (p.out_cap < out_bytes) {
        for (int s = 0; s < HostPipe::kSlots; s++) {
            if (p.d_out[s]) (void)hipFree(p.d_out[s]);
            p.d_out[s] = nullptr;
            HIP_TRY(hipMalloc(&p.d_out[s], out_bytes));
        }
        p.out_cap = out_bytes;
    }
    return EC_OK;
}

static int pipe_drain(ec_ctx *c, int rc) {
    for (int s = 0; s < HostPipe::kSlots; s++)
        if (c->pipe.st[s] && hipStreamSynchronize(c->pipe.st[s]) != hipSuccess && rc == EC_OK) rc = EC_ERR_DEVICE;
    return rc;
}

}  // extern "C"
namespace uplink_ec {
namespace capi {
size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
}  // namespace capi
}  // namespace uplink_ec
extern "C" {

// ---------------------------------------------------------------- per-stripe
// single_batch_once: one launch sequence for the whole batch, or kSplit when
// the staging for it cannot be had (and the batch has more than one request)
constexpr int kSplit = 1;
static int single_batch_once(ec_ctx *c, SingleReq *const *req, size_t nreq, size_t bs);

// One launch sequence for EncodeSingle requests of one share size bs: the
// stripes are packed into pinned staging, copied in with one transfer, the
// parity of every stripe is encoded in one launch (the compile-time encoder
// where there is one), a gather kernel picks each request's share, and one
// transfer brings them back.  Sets every request's rc: the outcome of the
// launch sequence that carried it (a batch split for want of staging carries
// each half on its own, and each half's requests get that half's outcome).
static void run_single_batch(ec_ctx *c, SingleReq *const *req, size_t nreq, size_t bs) {
    const int rc = single_batch_once(c, req, nreq, bs);
    if (rc == kSplit) {
        // no room for the whole batch: each half on its own (a request that
        // would succeed alone does not fail for sharing a batch)
        const size_t h = nreq / 2;
        run_single_batch(c, req, h, bs);
        run_single_batch(c, req + h, nreq - h, bs);
        return;
    }
    for (size_t r = 0; r < nreq; r++) req[r]->rc = rc;
}

static int single_batch_once(ec_ctx *c, SingleReq *const *req, size_t nreq, size_t bs) {
    const int k = c->k, n = c->n;
    const size_t stripe = (size_t)k * bs;
    const size_t in_bytes = nreq * stripe, par_bytes = (size_t)(n - k) * nreq * bs, out_bytes = nreq * bs;
    // device: [stripes | nums | parity | out]; pinned host: [stripes | nums | out]
    const size_t nums_at = align_up(in_bytes, 256), par_at = nums_at + align_up(nreq * 4, 256);
    const size_t out_at = par_at + align_up(par_bytes, 256), h_out = par_at;
    if (c->fault_max_batch > 0 &&
        (nreq > (size_t)c->fault_max_batch || (nreq == 1 && req[0]->num == c->fault_fail_num)))
        return nreq == 1 ? EC_ERR_DEVICE : kSplit;  // (test hook, see ec_ctx)
    Workspace *w = acquire_ws(c, out_at + out_bytes + 64, h_out + out_bytes);
    if (!w->d_buf || !w->stream || !w->h_buf) {
        release_ws(c, w);
        return nreq == 1 ? EC_ERR_DEVICE : kSplit;
    }
    for (size_t r = 0; r < nreq; r++) {
        memcpy(w->h_buf + r * stripe, req[r]->in, stripe);
        ((int *)(w->h_buf + nums_at))[r] = req[r]->num;
    }
    uint8_t *d = w->d_buf;
    hipStream_t st = w->stream;
    int rc = EC_OK;
    do {
        if (hipMemcpyAsync(d, w->h_buf, nums_at + nreq * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
            rc = EC_ERR_DEVICE;
            break;
        }
        if (n > k) {  // parity of every stripe of the batch
            RsArgs a{};
            a.in_base = d;
            a.out_base = d + par_at;
            a.in_stripe_stride = (int64_t)stripe;
            a.out_stripe_stride = (int64_t)bs;
            a.nin = k;
            a.nout = n - k;
            for (int j = 0; j < k; j++) a.in_off[j] = (int64_t)j * bs, a.copy_off[j] = -1;
            std::vector<int64_t> out_off(n - k);
            for (int r = 0; r < n - k; r++) out_off[r] = (int64_t)r * nreq * bs;
            for (int r = 0; r < std::min(n - k, kMaxOps); r++) a.out_off[r] = out_off[r];
            fill_geometry(a, (int)bs, (int64_t)nreq, 1);
            const bool bits = bs % 16 == 0;
            const EncoderKernel *ek = bits ? find_encoder(k, n, false, false) : nullptr;  // (starts no compile)
            if (ek) {
                set_extents(a, 1, c->d_chk);
                if (launch_encode_special(*ek, a, 0, st) != hipSuccess) {
                    rc = EC_ERR_DEVICE;
                    break;
                }
                rc = after_launch(c->d_chk, st);
            } else {
                if (!bits) a.cps = 1;
                PlanPtr plan;
                rc = parity_plan(c, &plan);
                if (rc == EC_OK) rc = run_matmul(c, a, out_off.data(), *plan, 1, bits, st);
            }
            if (rc) break;
        }
        if (launch_gather_shares(d, d + par_at, (const int *)(d + nums_at), k, (int64_t)nreq, (int64_t)bs, d + out_at,
                                 st) != hipSuccess ||
            hipMemcpyAsync(w->h_buf + h_out, d + out_at, out_bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            rc = EC_ERR_DEVICE;
            break;
        }
        for (size_t r = 0; r < nreq; r++) memcpy(req[r]->out, w->h_buf + h_out + r * bs, bs);
    } while (0);
    if (rc) (void)hipStreamSynchronize(st);
    release_ws(c, w);
    return rc;
}

// A batch takes queued requests up to this many, and up to kMaxSingleBatchBytes
// of stripes (at least one request): the staging it needs stays bounded however
// large the callers' stripes are.
constexpr size_t kMaxSingleBatch = 2048;
constexpr size_t kMaxSingleBatchBytes = (size_t)16 << 20;
constexpr int kSingleLeaders = 2;  // batches in flight at once: one's host copies overlap the other's GPU work

// EncodeSingle (rs.go:21-23), called by uplink per (piece, stripe) from up to
// 300 goroutines at once (segmentupload/encode.go:58, testuplink/uplink.go:83).
// Concurrent calls are coalesced by group commit: a caller that finds fewer
// than kSingleLeaders batches running becomes a leader, takes every queued
// request (its own included) and runs them as one batch; calls arriving
// meanwhile queue for the next one.  Each caller sleeps on its own condition
// variable and is woken once -- when its result is ready, or when it heads the
// queue and a leader slot frees -- so 300 waiting threads cost no thundering
// herd.  A lone caller pays one transfer-kernel-transfer round trip; many
// callers share it (tools/per_stripe_bench.c).
int ec_encode_single(const ec_ctx *cc, const uint8_t *in, size_t in_len, uint8_t *out, size_t out_len, int num) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c) return EC_ERR_INVALID_ARG;
    if (num < 0) return EC_ERR_NUM_NEGATIVE;
    if (num >= c->n) return EC_ERR_NUM_RANGE;
    if (in_len % (size_t)c->k) return EC_ERR_INPUT_LENGTH;
    const size_t bs = in_len / c->k;
    if (out_len != bs) return EC_ERR_OUTPUT_LENGTH;
    if (bs == 0) return EC_OK;
    if (!in || !out) return EC_ERR_INVALID_ARG;
    if (c->k > kMaxOps) return EC_ERR_UNSUPPORTED;
    DeviceGuard dg(c->device);
    SingleReq r{in, bs, out, num};
    std::unique_lock<std::mutex> lk(c->single_mu);
    c->single_q.push_back(&r);
    while (!r.done) {
        if (r.taken || c->single_leaders >= kSingleLeaders) {
            r.cv.wait(lk);
            continue;
        }
        c->single_leaders++;
        size_t take = 0, bytes = 0;
        while (take < c->single_q.size() && take < kMaxSingleBatch &&
               (take == 0 || bytes + c->single_q[take]->bs * c->k <= kMaxSingleBatchBytes))
            bytes += c->single_q[take++]->bs * c->k;
        std::vector<SingleReq *> batch(c->single_q.begin(), c->single_q.begin() + take);
        c->single_q.erase(c->single_q.begin(), c->single_q.begin() + take);
        for (SingleReq *q : batch) q->taken = true;
        lk.unlock();
        // group by share size (one launch sequence per size)
        std::stable_sort(batch.begin(), batch.end(), [](const SingleReq *a, const SingleReq *b) { return a->bs < b->bs; });
        for (size_t i = 0; i < batch.size();) {
            size_t j = i;
            while (j < batch.size() && batch[j]->bs == batch[i]->bs) j++;
            run_single_batch(c, batch.data() + i, j - i, batch[i]->bs);  // sets each request's rc
            i = j;
        }
        lk.lock();
        c->single_leaders--;
        for (SingleReq *q : batch) {
            q->done = true;
            if (q != &r) q->cv.notify_one();
        }
        // the leader slot passes to the oldest queued caller
        if (!c->single_q.empty()) c->single_q.front()->cv.notify_one();
    }
    return r.rc;
}

int ec_encode(const ec_ctx *cc, const uint8_t *in, size_t in_len, uint8_t *out) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c) return EC_ERR_INVALID_ARG;
    if (in_len % (size_t)c->k) return EC_ERR_INPUT_LENGTH;
    const size_t bs = in_len / c->k;
    if (bs == 0) return EC_OK;
    if (!in || !out) return EC_ERR_INVALID_ARG;
    if (c->k > kMaxOps) return EC_ERR_UNSUPPORTED;
    DeviceGuard dg(c->device);
    PlanPtr plan;
    int rc = parity_plan(c, &plan);
    if (rc) return rc;
    const size_t out_at = (in_len + 15) & ~(size_t)15;
    Workspace *w = acquire_ws(c, out_at + bs * c->n + 64);
    if (!w->d_buf || !w->stream) { release_ws(c, w); return EC_ERR_DEVICE; }
    do {
        if (hipMemcpyAsync(w->d_buf, in, in_len, hipMemcpyHostToDevice, w->stream) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        RsArgs a{};
        a.in_base = w->d_buf;
        a.out_base = w->d_buf + out_at;
        a.in_stripe_stride = (int64_t)in_len;
        a.out_stripe_stride = (int64_t)bs;
        for (int j = 0; j < c->k; j++) { a.in_off[j] = (int64_t)j * bs; a.copy_off[j] = (int64_t)j * bs; }
        std::vector<int64_t> out_off(std::max(c->n - c->k, 1));
        for (int r = 0; r < c->n - c->k; r++) out_off[r] = (int64_t)(c->k + r) * bs;
        fill_geometry(a, (int)bs, 1, 1);
        const bool bits = (bs % 16) == 0;
        if (!bits) a.cps = 1;
        rc = run_matmul(c, a, out_off.data(), *plan, 1, bits, w->stream);
        if (rc) break;
        if (hipMemcpyAsync(out, w->d_buf + out_at, bs * c->n, hipMemcpyDeviceToHost, w->stream) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        if (hipStreamSynchronize(w->stream) != hipSuccess) rc = EC_ERR_DEVICE;
    } while (0);
    release_ws(c, w);
    return rc;
}

static void sort_shares_inplace(int ns, int *nums, const uint8_t **shares) {
    // stable insertion sort, like sort.Sort on a small []Share
    for (int a = 1; a < ns; a++) {
        int kn = nums[a];
        const uint8_t *kd = shares[a];
        int b = a - 1;
        while (b >= 0 && nums[b] > kn) {
            nums[b + 1] = nums[b];
            shares[b + 1] = shares[b];
            b--;
        }
        nums[b + 1] = kn;
        shares[b + 1] = kd;
    }
}

int ec_rebuild(const ec_ctx *cc, int nshares, int *nums, const uint8_t **shares, size_t share_len, uint8_t *out) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c || (nshares > 0 && (!nums || !shares))) return EC_ERR_INVALID_ARG;
    if (nshares < c->k) return EC_ERR_NOT_ENOUGH_SHARES;
    DeviceGuard dg(c->device);
    sort_shares_inplace(nshares, nums, shares);
    if (share_len == 0) return EC_OK;
    if (!out) return EC_ERR_INVALID_ARG;
    const size_t slot = (share_len + 15) & ~(size_t)15;
    const size_t out_at = slot * nshares;
    // the shares go through pinned staging in one transfer each way
    Workspace *w = acquire_ws(c, out_at + share_len * c->k + 64, out_at + share_len * c->k);
    if (!w->d_buf || !w->stream || !w->h_buf) { release_ws(c, w); return EC_ERR_DEVICE; }
    int rc = EC_OK;
    do {
        std::vector<const uint8_t *> dptr(nshares);
        for (int i = 0; i < nshares; i++) {
            memcpy(w->h_buf + slot * i, shares[i], share_len);
            dptr[i] = w->d_buf + slot * i;
        }
        if (hipMemcpyAsync(w->d_buf, w->h_buf, out_at, hipMemcpyHostToDevice, w->stream) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        rc = rebuild_device(c, nshares, nums, dptr.data(), (int)share_len, 1, 1, 0, 0, w->d_buf + out_at, w->stream);
        if (rc) break;
        if (hipMemcpyAsync(w->h_buf + out_at, w->d_buf + out_at, share_len * c->k, hipMemcpyDeviceToHost, w->stream) != hipSuccess ||
            hipStreamSynchronize(w->stream) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        memcpy(out, w->h_buf + out_at, share_len * c->k);
    } while (0);
    if (rc) (void)hipStreamSynchronize(w->stream);
    release_ws(c, w);
    return rc;
}

// Decode = Correct + Rebuild (rsScheme.Decode, rs.go:32-38).  Correct: the
// shares beyond the first k (sorted) are re-encoded from the first k on the
// GPU, mismatching byte columns are flagged, and each flagged column is
// corrected by Berlekamp-Welch on the GPU; shares are corrected in place.
void *ec_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void ec_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

void *ec_device_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) return nullptr;
    return p;
}

void ec_device_free(void *p) {
    if (p) (void)hipFree(p);
}

int ec_copy(void *dst, const void *src, size_t bytes) {
    if (!bytes) return EC_OK;
    if (!dst || !src) return EC_ERR_INVALID_ARG;
    return hipMemcpy(dst, src, bytes, hipMemcpyDefault) == hipSuccess ? EC_OK : EC_ERR_DEVICE;
}

// Segment g goes through slot g % 3: H2D on that slot's stream, then the
// kernel, then D2H, all stream-ordered, so a slot's device buffers are never
// reused before its previous segment has left the GPU; the three streams
// overlap the copies of neighbouring segments with each other and the kernel.

// BLAKE3 of every piece of one segment resident on the device: parity pieces
// are contiguous in `parity` ([n-k][plen]), data piece j is share j of every
// stripe of the stripe-major segment `seg` (runs of ess bytes, k*ess apart).
// hashes: n*32 device bytes; ws: b3_segment_ws_bytes.
// hashes [nseg][n][32]: the data pieces of all nseg segments in one launch,
// the parity pieces in another; the hash rows of a segment are n*32 apart,
// so each launch writes into a [nseg][rows][32] staging area first.
}  // extern "C"
namespace uplink_ec {
namespace capi {
B3View data_view(const ec_ctx *c, const uint8_t *segs, size_t nseg, size_t nstripes) {
    const uint64_t plen = nstripes * (uint64_t)c->ess;
    return B3View{segs, (int64_t)c->ess, plen, (uint64_t)c->ess, (int64_t)c->k * c->ess, nseg * (uint64_t)c->k,
                  (uint64_t)c->k, (int64_t)(plen * c->k), 0};
}
B3View parity_view(const ec_ctx *c, const uint8_t *parity, size_t nseg, size_t nstripes) {
    const uint64_t plen = nstripes * (uint64_t)c->ess;
    return B3View{parity, (int64_t)plen, plen, plen, (int64_t)plen, nseg * (uint64_t)(c->n - c->k), 0, 0, 0};
}
size_t b3_segment_ws_bytes(const ec_ctx *c, size_t nseg, size_t nstripes) {
    B3View all = parity_view(c, nullptr, nseg, nstripes);
    all.npieces = nseg * (uint64_t)c->n;
    return align_up(b3_workspace_bytes(all), 256) + align_up(32 * nseg * (size_t)c->n, 256);
}
int hash_segments(const ec_ctx *c, const uint8_t *segs, const uint8_t *parity, size_t nseg, size_t nstripes,
                         uint8_t *hashes, uint8_t *ws, hipStream_t st) {
    const size_t n = c->n, k = c->k;
    uint8_t *stage = ws;  // [data: nseg*k*32][parity: nseg*(n-k)*32]
    uint8_t *tree = ws + align_up(32 * nseg * n, 256);
    B3View pv = parity_view(c, parity, nseg, nstripes);
    if (n == k) pv.npieces = 0;
    HIP_TRY(b3_launch2(data_view(c, segs, nseg, nstripes), pv, stage, tree, st));
    // interleave to [nseg][n][32]
    HIP_TRY(hipMemcpy2DAsync(hashes, 32 * n, stage, 32 * k, 32 * k, nseg, hipMemcpyDeviceToDevice, st));
    if (n > k)
        HIP_TRY(hipMemcpy2DAsync(hashes + 32 * k, 32 * n, stage + 32 * nseg * k, 32 * (n - k), 32 * (n - k), nseg,
                                 hipMemcpyDeviceToDevice, st));
    return EC_OK;
}
}  // namespace capi
}  // namespace uplink_ec
extern "C" {

// Host pipeline of the encode.  The three pipe streams take roles (H2D,
// compute, D2H) and every segment goes through in chunks of stripes, so the
// upload of chunk i+1, the encode of chunk i and the download of chunk i-1
// overlap, and PCIe carries both directions at once (it is full duplex:
// ~57 GB/s each way, ~97 GB/s both, tools/exp/pcie_probe.py).  Segments
// rotate over the three device slots; a slot is reused once its D2H is done.
static int encode_host(ec_ctx *c, const uint8_t *segs, size_t nseg, size_t nstripes, uint8_t *pieces,
                       uint8_t *hashes, int flags) {
    if (!c || !segs || !pieces) return EC_ERR_INVALID_ARG;
    if (nseg == 0 || nstripes == 0) return EC_OK;
    DeviceGuard dg(c->device);
    const size_t ess = c->ess, stripe = (size_t)c->k * ess, spad = nstripes * stripe;
    const bool parity_only = (flags & EC_FLAG_PARITY_ONLY) != 0;
    const int rows = parity_only ? c->n - c->k : c->n;
    const size_t plen = nstripes * ess, pbytes = (size_t)rows * plen;
    // device slot: pieces | hashes (n*32) | BLAKE3 workspace
    const size_t hash_at = align_up(pbytes, 256), ws_at = hash_at + align_up(32 * (size_t)c->n, 256);
    const size_t out_cap = hashes ? ws_at + b3_segment_ws_bytes(c, 1, nstripes) : std::max<size_t>(pbytes, 1);
    const size_t nch = std::min<size_t>(8, std::max<size_t>(1, nstripes / 256));
    const size_t chunk = (nstripes + nch - 1) / nch;
    std::lock_guard<std::mutex> g(c->pipe_mu);
    int rc = pipe_reserve(c, spad, out_cap);
    if (rc) return rc;
    hipStream_t h2d = c->pipe.st[0], comp = c->pipe.st[1], d2h = c->pipe.st[2];
    std::vector<hipEvent_t> ev(2 * nch + 1 + HostPipe::kSlots, nullptr);
    for (auto &e : ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = EC_ERR_DEVICE;
    hipEvent_t *ev_in = ev.data(), *ev_enc = ev.data() + nch, ev_hash = ev[2 * nch];
    hipEvent_t *slot_free = ev.data() + 2 * nch + 1;
    for (size_t sg = 0; sg < nseg && rc == EC_OK; sg++) {
        const int slot = (int)(sg % HostPipe::kSlots);
        uint8_t *d_in = c->pipe.d_in[slot], *d_out = c->pipe.d_out[slot];
        if (sg >= (size_t)HostPipe::kSlots && hipStreamWaitEvent(h2d, slot_free[slot], 0) != hipSuccess) {
            rc = EC_ERR_DEVICE;
            break;
        }
        for (size_t ch = 0; ch < nch && rc == EC_OK; ch++) {
            const size_t s0 = ch * chunk, s1 = std::min(nstripes, s0 + chunk);
            if (s0 >= s1) break;
            if (hipMemcpyAsync(d_in + s0 * stripe, segs + sg * spad + s0 * stripe, (s1 - s0) * stripe,
                               hipMemcpyHostToDevice, h2d) != hipSuccess ||
                hipEventRecord(ev_in[ch], h2d) != hipSuccess || hipStreamWaitEvent(comp, ev_in[ch], 0) != hipSuccess) {
                rc = EC_ERR_DEVICE;
                break;
            }
            if (rows > 0) rc = encode_range(c, d_in, 1, nstripes, s0, s1, d_out, flags, comp);
            if (rc) break;
            if (hipEventRecord(ev_enc[ch], comp) != hipSuccess || hipStreamWaitEvent(d2h, ev_enc[ch], 0) != hipSuccess) {
                rc = EC_ERR_DEVICE;
                break;
            }
            if (rows > 0 && hipMemcpy2DAsync(pieces + sg * pbytes + s0 * ess, plen, d_out + s0 * ess, plen,
                                             (s1 - s0) * ess, rows, hipMemcpyDeviceToHost, d2h) != hipSuccess)
                rc = EC_ERR_DEVICE;
        }
        if (rc == EC_OK && hashes) {
            const uint8_t *parity = d_out + (parity_only ? 0 : (size_t)c->k * plen);
            rc = hash_segments(c, d_in, parity, 1, nstripes, d_out + hash_at, d_out + ws_at, comp);
            if (rc == EC_OK &&
                (hipEventRecord(ev_hash, comp) != hipSuccess || hipStreamWaitEvent(d2h, ev_hash, 0) != hipSuccess ||
                 hipMemcpyAsync(hashes + sg * 32 * (size_t)c->n, d_out + hash_at, 32 * (size_t)c->n,
                                hipMemcpyDeviceToHost, d2h) != hipSuccess))
                rc = EC_ERR_DEVICE;
        }
        if (rc == EC_OK && hipEventRecord(slot_free[slot], d2h) != hipSuccess) rc = EC_ERR_DEVICE;
    }
    rc = pipe_drain(c, rc);
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

int ec_encode_segments_host(const ec_ctx *cc, const uint8_t *segs, size_t nseg, size_t nstripes, uint8_t *pieces,
                            int flags) {
    return encode_host(const_cast<ec_ctx *>(cc), segs, nseg, nstripes, pieces, nullptr, flags);
}

int ec_encode_segments_host_hashed(const ec_ctx *cc, const uint8_t *segs, size_t nseg, size_t nstripes,
                                   uint8_t *pieces, uint8_t *hashes, int flags) {
    if (!hashes) return EC_ERR_INVALID_ARG;
    return encode_host(const_cast<ec_ctx *>(cc), segs, nseg, nstripes, pieces, hashes, flags);
}

int ec_hash_segments(const ec_ctx *c, const uint8_t *segs, const uint8_t *parity, size_t nseg, size_t nstripes,
                     uint8_t *hashes, ec_stream stream) {
    if (!c || !segs || !hashes || (c->n > c->k && !parity)) return EC_ERR_INVALID_ARG;
    if (nseg == 0) return EC_OK;
    DeviceGuard dg(c->device);
    hipStream_t st = (hipStream_t)stream;
    void *ws = nullptr;
    HIP_TRY(hipMallocAsync(&ws, b3_segment_ws_bytes(c, nseg, nstripes), st));
    const int rc = hash_segments(c, segs, parity, nseg, nstripes, hashes, (uint8_t *)ws, st);
    (void)hipFreeAsync(ws, st);
    return rc;
}

int ec_blake3_pieces(const uint8_t *base, size_t npieces, long long piece_stride, size_t piece_len, size_t run,
                     long long run_stride, uint8_t *hashes, ec_stream stream) {
    if (!hashes || (!base && piece_len && npieces)) return EC_ERR_INVALID_ARG;
    if (npieces == 0) return EC_OK;
    hipStream_t st = (hipStream_t)stream;
    const B3View v{base, piece_stride, piece_len, run, run_stride, npieces, 0, 0, 0};
    const size_t ws_bytes = b3_workspace_bytes(v);
    void *ws = nullptr;
    if (ws_bytes) HIP_TRY(hipMallocAsync(&ws, ws_bytes, st));
    const hipError_t e = b3_launch(v, hashes, ws, st);
    if (ws) (void)hipFreeAsync(ws, st);
    return hip_fail(e);
}

int ec_blake3_host(const uint8_t *data, size_t npieces, long long stride, size_t piece_len, uint8_t *hashes) {
    if (!hashes || (!data && piece_len && npieces)) return EC_ERR_INVALID_ARG;
    if (npieces == 0) return EC_OK;
    const size_t span = (npieces - 1) * (size_t)stride + piece_len;
    hipStream_t st = nullptr;
    uint8_t *d = nullptr;
    int rc = EC_OK;
    do {
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        if (hipMalloc(&d, align_up(span, 256) + 32 * npieces) != hipSuccess) { rc = EC_ERR_DEVICE; d = nullptr; break; }
        uint8_t *dh = d + align_up(span, 256);
        if (span && hipMemcpyAsync(d, data, span, hipMemcpyHostToDevice, st) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        rc = ec_blake3_pieces(d, npieces, stride, piece_len, piece_len, stride, dh, st);
        if (rc) break;
        if (hipMemcpyAsync(hashes, dh, 32 * npieces, hipMemcpyDeviceToHost, st) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        if (hipStreamSynchronize(st) != hipSuccess) rc = EC_ERR_DEVICE;
    } while (0);
    if (st) (void)hipStreamSynchronize(st);
    if (d) (void)hipFree(d);
    if (st) (void)hipStreamDestroy(st);
    return rc;
}

int ec_rebuild_segments_host(const ec_ctx *cc, int nshares, const int *nums, const uint8_t *const *pieces,
                             size_t nstripes, size_t nseg, long long piece_seg_stride, uint8_t *out) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c || !nums || !pieces || !out) return EC_ERR_INVALID_ARG;
    if (nshares < c->k) return EC_ERR_NOT_ENOUGH_SHARES;
    if (nseg == 0 || nstripes == 0) return EC_OK;
    DeviceGuard dg(c->device);
    std::vector<int> order, ids;
    int rc = choose_shares(c, nshares, nums, order, ids);
    if (rc) return rc;
    const size_t ess = c->ess, plen = nstripes * ess, stripe = (size_t)c->k * ess, spad = nstripes * stripe;
    // The k chosen pieces usually sit at one stride in host memory (one buffer per segment): then
    // each chunk is one 2D copy.  Otherwise every piece is its own copy per chunk, and chunks are
    // kept >= 1 MiB per piece so the per-copy cost stays small.
    int64_t pstride = 0;
    bool strided = c->k > 1;
    if (strided) {
        pstride = pieces[order[1]] - pieces[order[0]];
        for (int i = 2; i < c->k && strided; i++) strided = pieces[order[i]] - pieces[order[i - 1]] == pstride;
        strided = strided && pstride >= (int64_t)plen;
    }
    const size_t nch = strided ? std::min<size_t>(8, std::max<size_t>(1, nstripes / 256))
                               : std::min<size_t>(8, std::max<size_t>(1, plen >> 20));
    const size_t chunk = (nstripes + nch - 1) / nch;
    std::lock_guard<std::mutex> g(c->pipe_mu);
    rc = pipe_reserve(c, plen * c->k, spad);
    if (rc) return rc;
    hipStream_t h2d = c->pipe.st[0], comp = c->pipe.st[1], d2h = c->pipe.st[2];
    std::vector<hipEvent_t> ev(2 * nch + HostPipe::kSlots, nullptr);
    for (auto &e : ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = EC_ERR_DEVICE;
    hipEvent_t *ev_in = ev.data(), *ev_out = ev.data() + nch, *slot_free = ev.data() + 2 * nch;
    std::vector<int> knums(c->k);
    for (int i = 0; i < c->k; i++) knums[i] = ids[i];
    std::vector<const uint8_t *> dptr(c->k);
    for (size_t sg = 0; sg < nseg && rc == EC_OK; sg++) {
        const int slot = (int)(sg % HostPipe::kSlots);
        uint8_t *d_in = c->pipe.d_in[slot], *d_out = c->pipe.d_out[slot];
        if (sg >= (size_t)HostPipe::kSlots && hipStreamWaitEvent(h2d, slot_free[slot], 0) != hipSuccess) {
            rc = EC_ERR_DEVICE;
            break;
        }
        for (size_t ch = 0; ch < nch && rc == EC_OK; ch++) {
            const size_t s0 = ch * chunk, s1 = std::min(nstripes, s0 + chunk);
            if (s0 >= s1) break;
            for (int i = 0; i < c->k; i++) dptr[i] = d_in + plen * i + s0 * ess;
            if (strided) {
                if (hipMemcpy2DAsync(d_in + s0 * ess, plen, pieces[order[0]] + (int64_t)sg * piece_seg_stride + s0 * ess,
                                     (size_t)pstride, (s1 - s0) * ess, c->k, hipMemcpyHostToDevice, h2d) != hipSuccess)
                    rc = EC_ERR_DEVICE;
            } else {
                for (int i = 0; i < c->k && rc == EC_OK; i++) {
                    const uint8_t *src = pieces[order[i]] + (int64_t)sg * piece_seg_stride + s0 * ess;
                    if (hipMemcpyAsync(d_in + plen * i + s0 * ess, src, (s1 - s0) * ess, hipMemcpyHostToDevice, h2d) !=
                        hipSuccess)
                        rc = EC_ERR_DEVICE;
                }
            }
            if (rc || hipEventRecord(ev_in[ch], h2d) != hipSuccess || hipStreamWaitEvent(comp, ev_in[ch], 0) != hipSuccess) {
                rc = rc ? rc : EC_ERR_DEVICE;
                break;
            }
            rc = rebuild_device(c, c->k, knums.data(), dptr.data(), c->ess, (int64_t)(s1 - s0), 1, 0, 0,
                                d_out + s0 * stripe, comp);
            if (rc) break;
            if (hipEventRecord(ev_out[ch], comp) != hipSuccess || hipStreamWaitEvent(d2h, ev_out[ch], 0) != hipSuccess ||
                hipMemcpyAsync(out + sg * spad + s0 * stripe, d_out + s0 * stripe, (s1 - s0) * stripe,
                               hipMemcpyDeviceToHost, d2h) != hipSuccess)
                rc = EC_ERR_DEVICE;
        }
        if (rc == EC_OK && hipEventRecord(slot_free[slot], d2h) != hipSuccess) rc = EC_ERR_DEVICE;
    }
    rc = pipe_drain(c, rc);
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

// expected[r] = the share numbered nums[outs[r]], re-encoded from the k shares at positions
// basis[0..k) of the device share slots (rows `slot` apart); expected rows `slot` apart
static int reencode(ec_ctx *c, const uint8_t *d, size_t slot, size_t len, const int *nums, const int *basis,
                    const int *outs, int nout, uint8_t *expected, hipStream_t st) {
    const int k = c->k;
    // plan key: -1, the basis share numbers, -2, the re-encoded share numbers
    std::vector<int> key{-1};
    for (int i = 0; i < k; i++) key.push_back(nums[basis[i]]);
    key.push_back(-2);
    for (int r = 0; r < nout; r++) key.push_back(nums[outs[r]]);
    PlanPtr plan;
    int rc = cached_plan(c, key, [&](std::vector<uint8_t> &M, int &rows, std::vector<int> &) {
        std::vector<uint8_t> m((size_t)k * k);
        for (int i = 0; i < k; i++) memcpy(&m[(size_t)i * k], &c->G[(size_t)nums[basis[i]] * k], k);
        if (!gf_invert(m.data(), k)) return EC_ERR_SINGULAR;
        rows = nout;
        M.assign((size_t)std::max(nout, 1) * k, 0);
        for (int r = 0; r < nout; r++)
            for (int col = 0; col < k; col++) {
                uint8_t acc = 0;
                for (int t = 0; t < k; t++) acc ^= gf_mul(c->G[(size_t)nums[outs[r]] * k + t], m[(size_t)t * k + col]);
                M[(size_t)r * k + col] = acc;
            }
        return EC_OK;
    }, &plan);
    if (rc) return rc;
    RsArgs a{};
    a.in_base = d;
    a.out_base = expected;
    a.in_stripe_stride = (int64_t)len;
    a.out_stripe_stride = (int64_t)len;
    for (int j = 0; j < k; j++) {
        a.in_off[j] = (int64_t)slot * basis[j];
        a.copy_off[j] = -1;
    }
    std::vector<int64_t> out_off(std::max(nout, 1));
    for (int r = 0; r < nout; r++) out_off[r] = (int64_t)slot * r;
    fill_geometry(a, (int)len, 1, 1);
    const bool bits = (len % 16) == 0;
    if (!bits) a.cps = 1;
    return run_matmul(c, a, out_off.data(), *plan, 1, bits, st);
}

// Where the Correct step keeps its data in a device workspace of ns share
// slots `slot` bytes apart (ec_decode, and ec_decode_segments' error path).
struct CorrectLayout {
    size_t slot, exp_at, flags_at, cols_at, nums_at, stat_at, out_at, samp_at, bytes;
    static constexpr int kSample = 64;  // flagged columns decoded first to locate bad shares
    CorrectLayout(size_t share_len, int nshares, int k, size_t out_bytes) {
        slot = (share_len + 15) & ~(size_t)15;
        const int extra = nshares - k;
        exp_at = slot * nshares;
        flags_at = exp_at + slot * (size_t)extra;
        cols_at = (flags_at + slot + 15) & ~(size_t)15;
        nums_at = cols_at + share_len * 8;
        stat_at = nums_at + 4 * 256;
        out_at = (stat_at + share_len * 4 + 15) & ~(size_t)15;
        samp_at = (out_at + out_bytes + 15) & ~(size_t)15;  // sample cols, status, changed, row lists
        bytes = samp_at + kSample * (8 + 4 + (size_t)nshares) + 8 * (size_t)nshares + 64;
    }
};

// FEC.Correct on the nshares shares in the workspace (slots L.slot apart, sorted
// by number): re-encode the shares beyond the first k from the first k and flag
// the columns where any differs; correct those (a bad piece's columns by the
// fast path below, the rest by Berlekamp-Welch), in place.  *changed: whether
// any column was flagged (the shares were rewritten).
static int correct_device(ec_ctx *c, uint8_t *d, const CorrectLayout &L, size_t share_len, const int *nums,
                          int nshares, hipStream_t st, bool *changed) {
    const int k = c->k, extra = nshares - k;
    constexpr int kSample = CorrectLayout::kSample;
    const size_t slot = L.slot;
    *changed = false;
    if (extra <= 0 || share_len == 0) return EC_OK;
    auto bw_columns = [&](const std::vector<int64_t> &cl) -> int {  // Berlekamp-Welch on columns, in place
        if (cl.empty()) return EC_OK;
        if (hipMemcpyAsync(d + L.cols_at, cl.data(), cl.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
            launch_berlekamp_welch(d, slot, (int64_t)share_len, (const int *)(d + L.nums_at), k, c->n, nshares,
                                   (const int64_t *)(d + L.cols_at), (int)cl.size(), (int *)(d + L.stat_at), st) !=
                hipSuccess)
            return EC_ERR_DEVICE;
        std::vector<int> status(cl.size());
        if (hipMemcpyAsync(status.data(), d + L.stat_at, 4 * cl.size(), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return EC_ERR_DEVICE;
        for (int s2 : status) {
            if (s2 == -6) return EC_ERR_NOT_ENOUGH_SHARES;
            if (s2 == -7) return EC_ERR_TOO_MANY_ERRORS;
            if (s2 != 0) return EC_ERR_UNSUPPORTED;
        }
        return EC_OK;
    };
    std::vector<int> basis(k), rest(extra);
    for (int i = 0; i < k; i++) basis[i] = i;
    for (int r = 0; r < extra; r++) rest[r] = k + r;
    int rc = reencode(c, d, slot, share_len, nums, basis.data(), rest.data(), extra, d + L.exp_at, st);
    if (rc) return rc;
    if (launch_flag_columns(d, slot, d + L.exp_at, slot, k, nshares, share_len, d + L.flags_at, st) != hipSuccess)
        return EC_ERR_DEVICE;
    std::vector<uint8_t> flags(share_len);
    if (hipMemcpyAsync(flags.data(), d + L.flags_at, share_len, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(d + L.nums_at, nums, 4 * (size_t)nshares, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return EC_ERR_DEVICE;
    std::vector<int64_t> cols;
    for (size_t col = 0; col < share_len; col++)
        if (flags[col]) cols.push_back((int64_t)col);
    if (cols.empty()) return EC_OK;
    *changed = true;
    // Fast path for errors confined to a few shares (a bad piece): decode a sample of the
    // flagged columns, take the shares BW rewrote there as the bad set B, and if
    // |B| <= e check every column on the other shares alone.  Where they agree, the
    // codeword they define is within e of what was received, so it is the unique BW
    // answer: B is rewritten from them.  Only columns where they disagree go to BW.
    const int e = extra / 2;
    if (e >= 1 && cols.size() > (size_t)4 * kSample) {
        std::vector<int64_t> samp(kSample);
        for (int i = 0; i < kSample; i++) samp[i] = cols[(size_t)i * cols.size() / kSample];
        uint8_t *d_changed = d + L.samp_at + kSample * 12;
        if (hipMemcpyAsync(d + L.samp_at, samp.data(), kSample * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
            launch_berlekamp_welch(d, slot, (int64_t)share_len, (const int *)(d + L.nums_at), k, c->n, nshares,
                                   (const int64_t *)(d + L.samp_at), kSample, (int *)(d + L.samp_at + kSample * 8),
                                   st, d_changed) != hipSuccess)
            return EC_ERR_DEVICE;
        std::vector<int> sstat(kSample);
        std::vector<uint8_t> chg((size_t)kSample * nshares);
        if (hipMemcpyAsync(sstat.data(), d + L.samp_at + kSample * 8, 4 * kSample, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(chg.data(), d_changed, chg.size(), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return EC_ERR_DEVICE;
        bool sample_ok = true;
        for (int s2 : sstat) sample_ok = sample_ok && s2 == 0;
        std::vector<int> bad, good;
        for (int i = 0; i < nshares; i++) {
            bool b = false;
            for (int t = 0; t < kSample && sample_ok; t++) b = b || chg[(size_t)t * nshares + i];
            (b ? bad : good).push_back(i);
        }
        if (sample_ok && !bad.empty() && (int)bad.size() <= e && (int)good.size() >= k) {
            // expected rows: the other good shares, then the bad ones, from the first k good
            std::vector<int> outs(good.begin() + k, good.end());
            const int ncheck = (int)outs.size();
            outs.insert(outs.end(), bad.begin(), bad.end());
            int *d_rows = (int *)(d_changed + chg.size() + 16 - (chg.size() % 16));
            rc = reencode(c, d, slot, share_len, nums, good.data(), outs.data(), (int)outs.size(), d + L.exp_at, st);
            if (rc) return rc;
            if (hipMemcpyAsync(d_rows, outs.data(), 4 * outs.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
                launch_flag_rows(d, slot, d_rows, ncheck, d + L.exp_at, slot, share_len, d + L.flags_at, st) != hipSuccess ||
                hipMemcpyAsync(flags.data(), d + L.flags_at, share_len, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return EC_ERR_DEVICE;
            std::vector<int64_t> rest_cols;
            for (size_t col = 0; col < share_len; col++)
                if (flags[col]) rest_cols.push_back((int64_t)col);
            // rewrite the bad shares where the good ones agree, then BW the rest on the
            // received data (the sample columns are already decoded: their good
            // shares agree now)
            if (launch_put_rows(d, slot, d_rows + ncheck, (int)bad.size(), d + L.exp_at + slot * ncheck, slot,
                                share_len, d + L.flags_at, st) != hipSuccess)
                return EC_ERR_DEVICE;
            return bw_columns(rest_cols);
        }
    }
    return bw_columns(cols);
}

int ec_decode(const ec_ctx *cc, int nshares, int *nums, uint8_t **shares, size_t share_len, uint8_t *out) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c || (nshares > 0 && (!nums || !shares))) return EC_ERR_INVALID_ARG;
    const int k = c->k;
    if (nshares < k) return EC_ERR_NOT_ENOUGH_SHARES;
    DeviceGuard dg(c->device);
    sort_shares_inplace(nshares, nums, (const uint8_t **)shares);
    if (share_len == 0) return EC_OK;
    if (!out) return EC_ERR_INVALID_ARG;
    for (int i = 0; i < nshares; i++)
        if (nums[i] < 0 || nums[i] >= c->n) return EC_ERR_INVALID_SHARE;
    if (k > kMaxOps) return EC_ERR_UNSUPPORTED;
    const CorrectLayout L(share_len, nshares, k, share_len * k);
    Workspace *w = acquire_ws(c, L.bytes);
    if (!w->d_buf || !w->stream) { release_ws(c, w); return EC_ERR_DEVICE; }
    int rc = EC_OK;
    uint8_t *d = w->d_buf;
    hipStream_t st = w->stream;
    do {
        for (int i = 0; i < nshares; i++)
            if (hipMemcpyAsync(d + L.slot * i, shares[i], share_len, hipMemcpyHostToDevice, st) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        if (rc) break;
        bool changed = false;
        rc = correct_device(c, d, L, share_len, nums, nshares, st, &changed);
        if (rc) break;
        if (changed) {  // infectious corrects share.Data in place
            for (int i = 0; i < nshares; i++)
                if (hipMemcpyAsync(shares[i], d + L.slot * i, share_len, hipMemcpyDeviceToHost, st) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
            if (rc) break;
        }
        std::vector<const uint8_t *> dptr(nshares);
        for (int i = 0; i < nshares; i++) dptr[i] = d + L.slot * i;
        rc = rebuild_device(c, nshares, nums, dptr.data(), (int)share_len, 1, 1, 0, 0, d + L.out_at, st);
        if (rc) break;
        if (hipMemcpyAsync(out, d + L.out_at, share_len * k, hipMemcpyDeviceToHost, st) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        if (hipStreamSynchronize(st) != hipSuccess) rc = EC_ERR_DEVICE;
    } while (0);
    if (rc) (void)hipStreamSynchronize(st);
    release_ws(c, w);
    return rc;
}

// Syndrome rows of the sorted share set: row r = G_{k+r} G_B^-1 over the first k
// shares (B) plus the share k+r itself, zero on every codeword.
static int syndrome_plan(ec_ctx *c, const std::vector<int> &nums, PlanPtr *out) {
    const int k = c->k, ns = (int)nums.size(), extra = ns - k;
    std::vector<int> key{-3};
    key.insert(key.end(), nums.begin(), nums.end());
    return cached_plan(c, key, [&](std::vector<uint8_t> &M, int &rows, std::vector<int> &) {
        std::vector<uint8_t> m((size_t)k * k);
        for (int i = 0; i < k; i++) memcpy(&m[(size_t)i * k], &c->G[(size_t)nums[i] * k], k);
        if (!gf_invert(m.data(), k)) return EC_ERR_SINGULAR;
        rows = extra;
        M.assign((size_t)std::max(extra, 1) * ns, 0);
        for (int r = 0; r < extra; r++) {
            for (int b = 0; b < k; b++) {
                uint8_t acc = 0;
                for (int t = 0; t < k; t++) acc ^= gf_mul(c->G[(size_t)nums[k + r] * k + t], m[(size_t)t * k + b]);
                M[(size_t)r * ns + b] = acc;
            }
            M[(size_t)r * ns + k + r] = 1;
        }
        return EC_OK;
    }, out, ns);
}

// Fused Decode plan over the sorted share set (nums, all nshares of them as
// inputs): first the rows of Rebuild -- the data shares infectious' share
// choice leaves missing, from the shares it chooses (choose_shares) -- then one
// syndrome row per share it does not choose: that share minus its value
// interpolated through the chosen ones.  One launch reads every share once,
// stores the rebuilt rows (the present data shares are copied through) and
// checks the syndrome rows for zero; *nrebuild = the number of rebuilt rows.
// (Whether every share agrees with one codeword does not depend on which k
// shares the syndromes are taken against; against the chosen ones, only those
// k columns carry general coefficients -- every other column a single 1 -- so
// each wave builds the 4-plane combinations of k inputs, not of the union of
// two bases: Decode at k+20 (~11 more such inputs) 42.5 -> see DESIGN.md §4e.)
static int fused_decode_plan(ec_ctx *c, const std::vector<int> &nums, PlanPtr *out, std::vector<int> &missing_out) {
    const int k = c->k, ns = (int)nums.size(), extra = ns - k;
    std::vector<int> order, ids;
    int rc = choose_shares(c, ns, nums.data(), order, ids);
    if (rc) return rc;
    std::vector<int> key{-4};
    key.insert(key.end(), nums.begin(), nums.end());
    rc = cached_plan(c, key, [&](std::vector<uint8_t> &M, int &rows, std::vector<int> &missing) {
        // Rebuild rows over the chosen shares (their positions in the sorted list: order)
        std::vector<uint8_t> m((size_t)k * k, 0);
        for (int i = 0; i < k; i++) {
            if (ids[i] < k) m[(size_t)i * k + i] = 1;
            else memcpy(&m[(size_t)i * k], &c->G[(size_t)ids[i] * k], k);
        }
        if (!gf_invert(m.data(), k)) return EC_ERR_SINGULAR;
        for (int i = 0; i < k; i++)
            if (ids[i] >= k) missing.push_back(i);
        const int nreb = (int)missing.size();
        rows = nreb + extra;
        M.assign((size_t)std::max(rows, 1) * ns, 0);
        for (int r = 0; r < nreb; r++)
            for (int i = 0; i < k; i++) M[(size_t)r * ns + order[i]] = m[(size_t)missing[r] * k + i];
        // syndrome rows: share u (not chosen) minus G_u (G_chosen)^-1 applied to the chosen shares
        std::vector<char> chosen(ns, 0);
        for (int i = 0; i < k; i++) chosen[order[i]] = 1;
        int r = nreb;
        for (int u = 0; u < ns; u++) {
            if (chosen[u]) continue;
            uint8_t *row = &M[(size_t)r++ * ns];
            for (int i = 0; i < k; i++) {
                uint8_t acc = 0;
                for (int t = 0; t < k; t++) acc ^= gf_mul(c->G[(size_t)nums[u] * k + t], m[(size_t)t * k + i]);
                row[order[i]] = acc;
            }
            row[u] = 1;
        }
        return EC_OK;
    }, out, ns);
    if (rc == EC_OK) missing_out = (*out)->missing;
    return rc;
}

int ec_decode_segments_batched(const ec_ctx *cc, int nshares, const int *nums_in, uint8_t *const *pieces_in,
                               size_t nstripes, size_t nseg, long long piece_seg_stride, long long out_seg_stride,
                               uint8_t *out, ec_stream stream) {
    ec_ctx *c = const_cast<ec_ctx *>(cc);
    if (!c || (nshares > 0 && (!nums_in || !pieces_in))) return EC_ERR_INVALID_ARG;
    const int k = c->k, ess = c->ess;
    if (nshares < k) return EC_ERR_NOT_ENOUGH_SHARES;
    for (int i = 0; i < nshares; i++)
        if (nums_in[i] < 0 || nums_in[i] >= c->n) return EC_ERR_INVALID_SHARE;
    if (k > kMaxOps) return EC_ERR_UNSUPPORTED;
    if (nstripes == 0 || nseg == 0) return EC_OK;
    if (!out) return EC_ERR_INVALID_ARG;
    DeviceGuard dg(c->device);
    hipStream_t s = (hipStream_t)stream;
    // the shares in number order, as infectious sorts its []Share (the caller's arrays stay as they are)
    std::vector<int> ord(nshares);
    for (int i = 0; i < nshares; i++) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return nums_in[x] < nums_in[y]; });
    // a launch takes at most kMaxOps inputs.  Of more shares (a wide code, n > 128) the first
    // kMaxOps in number order go through the one-pass check + rebuild, and the syndromes of the
    // others are checked in further launches of kMaxOps - k of them at a time against the same
    // basis (the first k); a segment with errors is corrected over all of them, as infectious'
    // Correct uses every share it is given (rs.go:32-38)
    const int ns_all = nshares;
    std::vector<int> nums_all(ns_all);
    std::vector<uint8_t *> pcs_all(ns_all);
    for (int i = 0; i < ns_all; i++) {
        nums_all[i] = nums_in[ord[i]];
        pcs_all[i] = pieces_in[ord[i]];
    }
    nshares = std::min(nshares, kMaxOps);
    std::vector<int> nums(nums_all.begin(), nums_all.begin() + nshares);
    std::vector<uint8_t *> pcs(pcs_all.begin(), pcs_all.begin() + nshares);
    const int extra = nshares - k;
    const size_t piece_len = nstripes * (size_t)ess;
    bool bits = ess % 16 == 0 && aligned16(out);
    for (auto p : pcs_all) bits = bits && aligned16(p);
    Workspace *w = nullptr;
    int rc = EC_OK;
    uint32_t nbad = bits ? 0u : 1u;  // no bit-sliced check: take the workspace path
    std::vector<const uint8_t *> cp(pcs.begin(), pcs.end());
    bool fused = false;
    if (extra > 0 && bits) {
        // Decode, clean case, in one pass over the shares: the rebuilt data rows
        // stored, the syndrome rows checked for zero inside the kernel (a segment
        // with errors is redone below, Correct then Rebuild, over this output)
        PlanPtr plan;
        std::vector<int> missing;
        rc = fused_decode_plan(c, nums, &plan, missing);
        if (rc == EC_OK && plan->rows <= kMaxOps) {
            w = acquire_ws(c, 16);
            if (!w->d_buf) { release_ws(c, w); return EC_ERR_DEVICE; }
            RsArgs a{};
            const uint8_t *base = pcs[0];
            for (auto p : pcs) base = std::min<const uint8_t *>(base, p);
            a.in_base = base;
            a.out_base = out;
            a.in_stripe_stride = ess;
            a.out_stripe_stride = (int64_t)k * ess;
            a.in_seg_stride = piece_seg_stride;
            a.out_seg_stride = out_seg_stride;
            for (int i = 0; i < nshares; i++) {
                a.in_off[i] = pcs[i] - base;
                a.copy_off[i] = nums[i] < k ? (int64_t)nums[i] * ess : -1;
            }
            a.zero_check = (uint32_t *)w->d_buf;
            a.nstore = (int32_t)missing.size();
            std::vector<int64_t> out_off(std::max(plan->rows, 1), 0);
            for (size_t r = 0; r < missing.size(); r++) out_off[r] = (int64_t)missing[r] * ess;
            fill_geometry(a, ess, (int64_t)nstripes, (int64_t)nseg);
            if (hipMemsetAsync(w->d_buf, 0, 4, s) != hipSuccess) rc = EC_ERR_DEVICE;
            if (!rc) rc = run_matmul(c, a, out_off.data(), *plan, (int64_t)nseg, true, s);
            if (!rc && hipMemcpyAsync(&nbad, w->d_buf, 4, hipMemcpyDeviceToHost, s) != hipSuccess) rc = EC_ERR_DEVICE;
            fused = true;
        }
    }
    if (!rc && !fused && extra > 0 && bits) {
        // (a share set whose fused plan has more than kMaxOps rows) the syndrome rows
        // checked for zero inside the kernel (nothing stored); then Rebuild
        w = acquire_ws(c, 16);
        if (!w->d_buf) { release_ws(c, w); return EC_ERR_DEVICE; }
        PlanPtr plan;
        rc = syndrome_plan(c, nums, &plan);
        if (rc) { release_ws(c, w); return rc; }
        RsArgs a{};
        const uint8_t *base = pcs[0];
        for (auto p : pcs) base = std::min<const uint8_t *>(base, p);
        a.in_base = base;
        a.out_base = nullptr;
        a.in_stripe_stride = ess;
        a.out_stripe_stride = ess;
        for (int i = 0; i < nshares; i++) {
            a.in_off[i] = pcs[i] - base;
            a.copy_off[i] = -1;
        }
        a.in_seg_stride = piece_seg_stride;
        a.zero_check = (uint32_t *)w->d_buf;
        std::vector<int64_t> out_off(std::max(extra, 1), 0);
        fill_geometry(a, ess, (int64_t)nstripes, (int64_t)nseg);
        if (hipMemsetAsync(w->d_buf, 0, 4, s) != hipSuccess) rc = EC_ERR_DEVICE;
        if (!rc) rc = run_matmul(c, a, out_off.data(), *plan, (int64_t)nseg, true, s);
        if (!rc && hipMemcpyAsync(&nbad, w->d_buf, 4, hipMemcpyDeviceToHost, s) != hipSuccess) rc = EC_ERR_DEVICE;
    }
    if (!rc && !fused)
        rc = rebuild_device(c, nshares, nums.data(), cp.data(), ess, (int64_t)nstripes, (int64_t)nseg,
                            piece_seg_stride, out_seg_stride, out, s);
    // the shares past the first kMaxOps: their syndromes, a block of kMaxOps - k at a time
    if (ns_all > nshares && k >= kMaxOps) nbad = 1;  // (no room for a syndrome row in a launch: Correct checks)
    for (int lo = nshares; !rc && bits && k < kMaxOps && lo < ns_all; lo += kMaxOps - k) {
        const int hi = std::min(ns_all, lo + (kMaxOps - k));
        if (!w) {
            w = acquire_ws(c, 16);
            if (!w->d_buf) { release_ws(c, w); return EC_ERR_DEVICE; }
            if (hipMemsetAsync(w->d_buf, 0, 4, s) != hipSuccess) rc = EC_ERR_DEVICE;
        }
        std::vector<int> sub(nums_all.begin(), nums_all.begin() + k);
        std::vector<uint8_t *> sp(pcs_all.begin(), pcs_all.begin() + k);
        sub.insert(sub.end(), nums_all.begin() + lo, nums_all.begin() + hi);
        sp.insert(sp.end(), pcs_all.begin() + lo, pcs_all.begin() + hi);
        PlanPtr plan;
        if (!rc) rc = syndrome_plan(c, sub, &plan);
        if (rc) break;
        RsArgs a{};
        const uint8_t *base = sp[0];
        for (auto p : sp) base = std::min<const uint8_t *>(base, p);
        a.in_base = base;
        a.in_stripe_stride = ess;
        a.out_stripe_stride = ess;
        for (size_t i = 0; i < sp.size(); i++) {
            a.in_off[i] = sp[i] - base;
            a.copy_off[i] = -1;
        }
        a.in_seg_stride = piece_seg_stride;
        a.zero_check = (uint32_t *)w->d_buf;
        std::vector<int64_t> out_off(std::max(hi - lo, 1), 0);
        fill_geometry(a, ess, (int64_t)nstripes, (int64_t)nseg);
        rc = run_matmul(c, a, out_off.data(), *plan, (int64_t)nseg, true, s);
        if (!rc && hipMemcpyAsync(&nbad, w->d_buf, 4, hipMemcpyDeviceToHost, s) != hipSuccess) rc = EC_ERR_DEVICE;
    }
    if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = EC_ERR_DEVICE;  // returns when done (header)
    if (w) {  // (released before the error path takes a workspace of its own)
        if (rc) (void)hipStreamSynchronize(s);
        release_ws(c, w);
    }
    if (ns_all > k && !rc) {
        std::vector<const uint8_t *> cpa(ns_all);
        for (size_t g = 0; g < nseg && nbad != 0 && !rc; g++) {
            // errors (or no bit-sliced check): segment by segment, Correct over every share in
            // a workspace, write the corrected shares back into the caller's pieces (infectious
            // corrects share.Data in place), Rebuild again from them
            for (int i = 0; i < ns_all; i++) {
                pcs_all[i] = pieces_in[ord[i]] + (int64_t)g * piece_seg_stride;
                cpa[i] = pcs_all[i];
            }
            uint8_t *gout = out + (int64_t)g * out_seg_stride;
            const CorrectLayout L(piece_len, ns_all, k, 0);
            Workspace *cw = acquire_ws(c, L.bytes);
            if (!cw->d_buf || !cw->stream) rc = EC_ERR_DEVICE;
            hipStream_t st = cw->stream;
            for (int i = 0; i < ns_all && !rc; i++)
                if (hipMemcpyAsync(cw->d_buf + L.slot * i, pcs_all[i], piece_len, hipMemcpyDeviceToDevice, st) !=
                    hipSuccess)
                    rc = EC_ERR_DEVICE;
            bool changed = false;
            if (!rc) rc = correct_device(c, cw->d_buf, L, piece_len, nums_all.data(), ns_all, st, &changed);
            for (int i = 0; i < ns_all && !rc && changed; i++)
                if (hipMemcpyAsync(pcs_all[i], cw->d_buf + L.slot * i, piece_len, hipMemcpyDeviceToDevice, st) !=
                    hipSuccess)
                    rc = EC_ERR_DEVICE;
            if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = EC_ERR_DEVICE;
            if (cw->stream) (void)hipStreamSynchronize(st);
            release_ws(c, cw);
            if (!rc && changed)
                rc = rebuild_device(c, ns_all, nums_all.data(), cpa.data(), ess, (int64_t)nstripes, 1, 0, 0, gout, s);
            if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = EC_ERR_DEVICE;
        }
    }
    return rc;
}

int ec_decode_segments(const ec_ctx *c, int nshares, const int *nums, uint8_t *const *pieces, size_t nstripes,
                       uint8_t *out, ec_stream stream) {
    return ec_decode_segments_batched(c, nshares, nums, pieces, nstripes, 1, 0, 0, out, stream);
}

}  // extern "C"
