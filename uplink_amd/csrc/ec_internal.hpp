// Internal header of the C-ABI (ec_capi.cpp, ec_sets.cpp, ec_upload.cpp): the
// context and its parts, and the helpers the three files share.  Not installed;
// include/uplink_ec.h is the interface.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <list>
#include <memory>
#include <deque>
#include <atomic>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "../../include/uplink_ec.h"
#include "blake3.hpp"
#include "ec_log.hpp"
#include "gf256.hpp"
#include "rs_correct.hpp"
#include "rs_kernels.hpp"
#include "rs_sets.hpp"
#include "rs_sl.hpp"


#pragma GCC visibility push(hidden)  // (internal to the library: not in its dynamic symbol table)
namespace uplink_ec {
namespace capi {


// A runtime matrix M (rows x nin) uploaded for the generic kernels: the
// coefficients coef[j][r] = M[r][j] and, for the bit-sliced kernel, the
// jump-table leaf addresses of every block of up to kMaxOps rows
// (launch_jt_targets).  Plans are built once -- synchronously, on the
// context's own setup stream -- and reused by every launch of that matrix, so
// no launch allocates memory or prepares tables in stream order.
//
// Plans of at most kMaxOps rows can also carry the matrix as straight-line
// code (rs_sl.hpp): a module made from the template code object on the first
// launch that wants it, and the absolute addresses of its segments.
// Device memory for the plans' small tables (coefficients, leaf addresses,
// segment addresses), carved from 2-MiB chunks in power-of-two classes and
// recycled, so that making or evicting a plan costs no hipMalloc / hipFree
// (a fresh share set per segment is the download path's common case).  The
// chunks go back to HIP when the context and every plan are gone.
struct DevArena {
    static constexpr size_t kChunk = 2u << 20, kMinClass = 256;
    std::mutex mu;
    std::vector<void *> chunks;
    uint8_t *cur = nullptr;
    size_t left = 0;
    std::vector<std::vector<uint8_t *>> free_by_class = std::vector<std::vector<uint8_t *>>(32);
    static int cls(size_t n) {
        int c = 0;
        while ((kMinClass << c) < n) c++;
        return c;
    }
    uint8_t *alloc(size_t n) {
        const int c = cls(n);
        const size_t sz = kMinClass << c;
        std::lock_guard<std::mutex> g(mu);
        if (!free_by_class[c].empty()) {
            uint8_t *p = free_by_class[c].back();
            free_by_class[c].pop_back();
            return p;
        }
        if (sz > kChunk) {  // (no plan table is this large; served directly)
            void *p = nullptr;
            if (hipMalloc(&p, sz) != hipSuccess) return nullptr;
            chunks.push_back(p);
            return (uint8_t *)p;
        }
        if (left < sz) {
            void *p = nullptr;
            if (hipMalloc(&p, kChunk) != hipSuccess) return nullptr;
            chunks.push_back(p);
            cur = (uint8_t *)p;
            left = kChunk;
        }
        uint8_t *p = cur;
        cur += sz;
        left -= sz;
        return p;
    }
    void release(uint8_t *p, size_t n) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu);
        free_by_class[cls(n)].push_back(p);
    }
    ~DevArena() {
        for (void *p : chunks) (void)hipFree(p);
    }
};

// Completion marks of a context's runtime-matrix launches, per caller stream.
// Each launch gets the next sequence number of its stream; an event is
// recorded behind every kEvery-th launch only (a marker on the stream costs
// microseconds per launch).  Launch q on stream s is known complete once an
// event recorded at or after it has completed.  Events are recorded only at
// launch time, on the stream being launched on, and queried afterwards (never
// recorded on a stream the caller may have destroyed since).
struct StreamMarks {
    static constexpr int kEvery = 8;
    static constexpr size_t kMaxStreams = 32;
    struct Mark {
        hipStream_t s = nullptr;
        uint64_t issued = 0, ev_seq = 0;
        int since = 0;
        hipEvent_t ev = nullptr;
    };
    std::mutex mu;
    std::deque<Mark> marks;  // most recently used streams last
    // note a launch just queued on s; returns its sequence number (0: untracked)
    uint64_t launched(hipStream_t s) {
        std::lock_guard<std::mutex> g(mu);
        Mark *m = nullptr;
        for (auto it = marks.begin(); it != marks.end(); ++it)
            if (it->s == s) {
                if (std::next(it) != marks.end()) {  // most recently used last: eviction takes the idlest
                    Mark keep = *it;
                    marks.erase(it);
                    marks.push_back(keep);
                }
                m = &marks.back();
                break;
            }
        if (!m) {
            if (marks.size() >= kMaxStreams) {  // the least recently used stream's marks go
                if (marks.front().ev) (void)hipEventDestroy(marks.front().ev);
                marks.pop_front();
            }
            marks.emplace_back();
            m = &marks.back();
            m->s = s;
            if (hipEventCreateWithFlags(&m->ev, hipEventDisableTiming) != hipSuccess) m->ev = nullptr;
        }
        const uint64_t q = ++m->issued;
        if (++m->since >= kEvery && m->ev && hipEventRecord(m->ev, s) == hipSuccess) {
            m->since = 0;
            m->ev_seq = q;
        }
        return q;
    }
    bool done(hipStream_t s, uint64_t q) {
        std::lock_guard<std::mutex> g(mu);
        for (auto &x : marks)
            if (x.s == s) return q != 0 && x.ev && x.ev_seq >= q && hipEventQuery(x.ev) == hipSuccess;
        return false;
    }
    ~StreamMarks() {
        for (auto &x : marks)
            if (x.ev) (void)hipEventSynchronize(x.ev), (void)hipEventDestroy(x.ev);
    }
};

struct MatPlan {
    std::shared_ptr<DevArena> arena;  // where d_coef, d_tgt and d_sl live
    std::shared_ptr<StreamMarks> marks;  // the context's completion marks
    size_t coef_bytes = 0, sl_bytes = 0;
    std::vector<size_t> tgt_bytes;
    std::atomic<int> launches{0};     // launches made with this plan (straight-line code from the second on)
    std::vector<int> key;          // what the matrix is (decode: chosen share ids; see plan keys below)
    std::vector<int> missing;      // decode plans: the data positions rebuilt, in row order
    int rows = 0, nin = 0, coef_ld = 0;
    uint8_t *d_coef = nullptr;     // [j][r], ld = coef_ld
    std::vector<uint64_t *> d_tgt; // leaf addresses per block of kMaxOps rows
    std::vector<uint8_t> M;        // rows x nin, row-major (for the straight-line code)
    std::mutex sl_mu;
    bool sl_tried = false;
    std::atomic<bool> sl_ready{false};  // d_sl is set (launch paths read this, not d_sl, without sl_mu)
    hipModule_t sl_mod = nullptr;
    uint64_t *d_sl = nullptr;      // segment addresses [pass][chunk][group]
    // The plan's launches, as (stream, sequence number) of the context's
    // completion marks: the latest per stream.  A plan is destroyed only when
    // every one of them is known complete (evicted plans wait in the context's
    // graveyard for that); if not -- its last reference went elsewhere, or the
    // marks were dropped -- the destructor synchronises the device instead.
    std::mutex use_mu;
    std::vector<std::pair<hipStream_t, uint64_t>> uses;
    void note_use(hipStream_t s) {
        const uint64_t q = marks ? marks->launched(s) : 0;
        std::lock_guard<std::mutex> g(use_mu);
        for (auto &u : uses)
            if (u.first == s) {
                u.second = q;
                return;
            }
        uses.emplace_back(s, q);
    }
    bool idle() {
        std::lock_guard<std::mutex> g(use_mu);
        for (auto &u : uses)
            if (!marks || !marks->done(u.first, u.second)) return false;
        return true;
    }
    ~MatPlan() {
        if (!uses.empty() && !idle()) (void)hipDeviceSynchronize();
        if (arena) {
            arena->release(d_coef, coef_bytes);
            for (size_t i = 0; i < d_tgt.size(); i++) arena->release((uint8_t *)d_tgt[i], tgt_bytes[i]);
            arena->release((uint8_t *)d_sl, sl_bytes);
        }
        if (sl_mod) (void)hipModuleUnload(sl_mod);
    }
};
using PlanPtr = std::shared_ptr<MatPlan>;

struct Workspace {
    uint8_t *d_buf = nullptr;
    size_t cap = 0;
    uint8_t *h_buf = nullptr;  // pinned staging for the per-stripe calls' host buffers
    size_t h_cap = 0;
    hipStream_t stream = nullptr;
};

// A caller waiting for a workspace (acquire_ws).
struct WsWaiter {
    std::condition_variable cv;
    Workspace *w = nullptr;
};

// EncodeSingle requests waiting for a batched launch (ec_encode_single).
struct SingleReq {
    const uint8_t *in;
    size_t bs;
    uint8_t *out;
    int num;
    int rc = EC_OK;
    bool taken = false;  // in a batch a leader is running
    bool done = false;
    std::condition_variable cv;  // this caller's wake-up (done, or its turn to lead)
};

// Every export that takes a context runs on the context's device and
// restores the caller's current device on return (a Go caller's goroutine
// may move between OS threads, each with its own current device).
struct DeviceGuard {
    int prev = -1;
    bool switched = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) switched = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (switched) (void)hipSetDevice(prev);
    }
};



struct HostPipe {
    static constexpr int kSlots = 3;
    hipStream_t st[kSlots] = {};
    uint8_t *d_in[kSlots] = {};
    uint8_t *d_out[kSlots] = {};
    size_t in_cap = 0, out_cap = 0;
};

// Device side of one streamed upload (ec_upload_begin): the segment, its
// pieces and the four role streams (H2D, encode, D2H, piece hashes).  Kept in
// a per-context pool between uploads; one upload owns a slot from begin to end.
struct UploadSlot {
    hipStream_t st[4] = {};
    uint8_t *d_in = nullptr, *d_out = nullptr;
    size_t in_cap = 0, out_cap = 0;
    uint8_t *d_hash = nullptr;   // EC_FLAG_HASH_PIECES: chunk CVs | hashes | fold scratch
    size_t hash_cap = 0;
    uint8_t *h_hash = nullptr;   // pinned, n*32 bytes: the hashes as they come back
    size_t h_hash_cap = 0;
    std::vector<hipEvent_t> ev;  // [in ch][enc ch][d2h ch][hashes] of the current upload
    ~UploadSlot() {  // (also on an error path of ec_upload_begin: nothing of it is left behind)
        for (auto st : this->st)
            if (st) (void)hipStreamSynchronize(st), (void)hipStreamDestroy(st);
        for (auto e : ev)
            if (e) (void)hipEventDestroy(e);
        if (d_in) (void)hipFree(d_in);
        if (d_out) (void)hipFree(d_out);
        if (d_hash) (void)hipFree(d_hash);
        if (h_hash) (void)hipHostFree(h_hash);
    }
};

// One slot of a context's share-set calls (rs_sets.hpp): the pinned staging
// the host writes, the device descriptors and leaf tables rs_sets_prep makes
// from it, and the words the launches report through.  A call takes a slot
// whose previous call has finished on the GPU -- its last workgroup stores the
// call's sequence number into *h_done (pinned) -- so neither the host's writes
// nor the prep kernel's ever overtake a launch still reading the slot, and no
// event, marker or synchronisation is put on the caller's stream.
struct SetsSlot {
    SetStage *h_stage = nullptr;  // pinned, stage_cap entries (host-cached unless the zero-copy form)
    SetStage *d_stage = nullptr;  // device copy of it (the DMA form: one hipMemcpyAsync per call)
    size_t stage_cap = 0;
    SetDesc *d_desc = nullptr;    // device, stage_cap entries
    uint64_t *d_tgt = nullptr;    // device leaf tables, tgt_cap words
    size_t tgt_cap = 0;
    uint32_t *d_words = nullptr;  // device: [0] done counter, [1 + g] segment g's syndrome count (stage_cap + 1)
    uint32_t *h_words = nullptr;  // pinned: [0] done sequence number, [1 + g] syndrome counts read back (Decode)
    size_t words_cap = 0;         // entries of h_words
    uint32_t seq = 0;             // of the slot's latest call
    bool busy = false;            // a caller is filling or launching it
    bool dead = false;            // a launch failed after the prep and the device did not recover: never reused
    // buffers a slot outgrew: freed with the slot (ec_destroy), never on the call
    // path, where hipFree / hipHostFree would synchronise the whole device
    std::vector<void *> old_dev, old_host;
    ~SetsSlot() {
        if (h_stage) (void)hipHostFree(h_stage);
        if (d_stage) (void)hipFree(d_stage);
        if (d_desc) (void)hipFree(d_desc);
        if (d_tgt) (void)hipFree(d_tgt);
        if (d_words) (void)hipFree(d_words);
        if (h_words) (void)hipHostFree(h_words);
        for (void *p : old_dev) (void)hipFree(p);
        for (void *p : old_host) (void)hipHostFree(p);
    }
    bool idle() const { return !busy && !dead && __atomic_load_n(h_words, __ATOMIC_ACQUIRE) == seq; }
};

struct SetsRing {
    static constexpr size_t kMaxSlots = 16;  // live calls in flight per context before a caller waits
    // segments and leaf-table words a new slot is sized for (a pass of sets_export,
    // kPass segments of up to 128 inputs): a slot grows -- geometrically -- only for
    // larger ec_rebuild_segments_batched calls
    static constexpr size_t kInitSegs = 64, kInitTgtWords = (size_t)64 * 1024;
    // a caller waits at most this long for a slot (calls in flight that never
    // complete, e.g. a stream whose work never runs): then EC_ERR_DEVICE
    static constexpr int kAcquireTimeoutMs = 30000;
    std::mutex mu;
    std::vector<std::unique_ptr<SetsSlot>> slots;
};

// Background maker of decode plans' straight-line code (DESIGN.md §4
// "Straight-line rebuild bodies"): code generation and hipModuleLoadData take
// ~0.4 ms per share set, so a batched rebuild never waits for them.  A launch
// whose share set has no ready code runs the share-set path (jump-table body,
// rs_sets.hpp) and queues the set here; later launches of the set take the
// generated code once it has landed.
struct SlBuilder {
    std::mutex mu;
    std::condition_variable cv;      // work queued / stop (worker), a set finished (waiters)
    std::deque<std::vector<int>> q;  // share sets (chosen ids) to build
    std::set<std::vector<int>> pending;
    std::thread th;
    bool stop = false;
};

// Work counters of the compile-time encoder's launches (RsArgs::queue): a
// ring of counter pairs (tile counter, workgroups done), zeroed once when the
// ring is made.  The last workgroup of a launch puts its pair back to zero
// (rs_encoder.hpp), so a launch needs no memset before it, and then stores the
// launch's sequence number into the slot's completion word in pinned host
// memory.  A slot serves one launch at a time: it goes to a launch on the
// stream its previous launch ran on (stream order), or to any stream once its
// completion word shows that its latest launch has finished; with no such
// slot the launch assigns its tiles statically (identical results).  No launch
// waits on another stream and none needs an event or marker on its stream, so
// a stream that launches a few times and goes away leaves its slot to the
// others.
struct QueueRing {
    static constexpr int kSlots = 32;
    static constexpr int kStride = 64;  // words per slot: the counter pair (kQueueDoneWord), a slot per 256 bytes
    std::mutex mu;
    uint32_t *d = nullptr;
    uint32_t *h_done = nullptr;         // pinned, coherent: [slot] sequence number of its latest finished launch
    uint32_t seq[kSlots] = {};          // [slot] sequence number of its latest launch
    hipStream_t owner[kSlots] = {};     // stream of the slot's last launch
    bool used[kSlots] = {}, busy[kSlots] = {};
    bool done(int i) const { return __atomic_load_n(h_done + i, __ATOMIC_ACQUIRE) == seq[i]; }
};

}  // namespace capi
}  // namespace uplink_ec

using namespace uplink_ec;
using namespace uplink_ec::capi;

struct ec_ctx {
    int k = 0, n = 0, ess = 0, device = 0;
    QueueRing qring;
    std::atomic<uint64_t> q_taken{0}, q_static{0};  // encoder launches with a counter slot / static tiles
    std::mutex pipe_mu;  // one host pipeline at a time per context
    HostPipe pipe;
    std::mutex upload_mu;
    std::vector<std::unique_ptr<UploadSlot>> upload_free;  // idle streamed-upload slots
    std::vector<uint8_t> G;        // n x k
    hipStream_t setup = nullptr;   // plan uploads (synchronous, never a caller's stream)
    std::shared_ptr<DevArena> arena = std::make_shared<DevArena>();
    std::shared_ptr<StreamMarks> marks = std::make_shared<StreamMarks>();
    std::vector<PlanPtr> graveyard;  // evicted plans whose launches may still run (under mu)
    std::mutex setup_mu;
    std::mutex mu;
    std::list<PlanPtr> plans;      // decode / re-encode plans, MRU first
    PlanPtr enc_parity;            // rows k..n-1 of G
    std::vector<PlanPtr> enc_row;  // row num of G (EncodeSingle)
    std::vector<Workspace *> free_ws;
    std::vector<std::unique_ptr<Workspace>> all_ws;
    std::deque<WsWaiter *> ws_waiters;  // callers waiting for a workspace, first come first served
    uint32_t *d_chk = nullptr;     // checked build: the kernels' violation word
    int body = EC_BODY_AUTO;       // ec_set_body
    int last_body = EC_BODY_AUTO;  // ec_last_body
    // EncodeSingle coalescing (group commit): callers queue; up to
    // kSingleLeaders of them at a time each run everything queued as one batch
    std::mutex single_mu;
    std::deque<SingleReq *> single_q;
    int single_leaders = 0;
    // fault injection for tests only (UPLINK_EC_FAULT_SINGLE="max=M,num=J" read
    // at ec_create): EncodeSingle batches of more than M requests find no
    // staging, nor does a one-request batch for share J
    int fault_max_batch = 0, fault_fail_num = -1;
    // share-set calls (ec_*_segments_sets, and fresh share sets of the batched rebuild)
    uint64_t jt_base = 0;          // address of the jump table's leaf 0 on this device
    // one launch per share-set call on the widest class's waves, instead of one per wave-count
    // class: 951.2 vs 982.6 us per 32 fresh-set segments on one box (profiles/r05/d/bench_sets*.json);
    // UPLINK_EC_SETS_MERGE=0 at ec_create for the per-class launches (A/B)
    bool sets_merge = true;
    // the per-segment staging is read by the prep kernel straight from coherent pinned memory, or
    // -- UPLINK_EC_SETS_STAGE_DMA=1 -- reaches the GPU by one DMA into device memory per call (host
    // writes to cached pinned memory; the stream then waits ~20 us for the copy engine between
    // calls, profiles/r05/g)
    bool sets_stage_dma = false;
    // a one-segment Rebuild share-set call as one launch, its rows solved on the host and passed
    // in the launch's arguments (rs_sets_one), instead of rs_sets_prep1 + rs_matmul_sets;
    // UPLINK_EC_SETS_ONE=0 at ec_create for the two launches (A/B)
    bool sets_one = true;
    SetsRing sets;
    SlBuilder slb;
};

#define HIP_TRY(x)                                   \
    do {                                             \
        hipError_t e_ = (x);                         \
        if (e_ != hipSuccess) return hip_fail(e_);   \
    } while (0)

namespace uplink_ec {
namespace capi {

// Launches of at least this many tiles use a plan's straight-line code under
// EC_BODY_AUTO: its module costs a code generation and a module load once per
// plan, which only pays over many stripes.
constexpr int64_t kSlMinTiles = 64;
// Launches of at least this many tiles start the run-time compilation of their
// code's encoder when the library has none built in (rs_encoder_registry.cpp):
// a compile takes seconds of host CPU, per-stripe calls (1 tile) never start
// one, and a process that started one waits for it at exit.
constexpr int64_t kJitMinTiles = 256;

// ec_capi.cpp
int hip_fail(hipError_t e);
bool aligned16(const void *p);
int after_launch(uint32_t *chk, hipStream_t s);
// infectious Rebuild share choice: sort by number, then for i in 0..k-1 take
// the front share if its number == i else take from the back.
int choose_shares(const ec_ctx *c, int nshares, const int *nums, std::vector<int> &order_out,
                  std::vector<int> &ids_out);
int get_plan(ec_ctx *c, const std::vector<int> &ids, PlanPtr *out);
void ensure_sl(ec_ctx *c, MatPlan &plan);
int rebuild_with_plan(ec_ctx *c, MatPlan &plan, const std::vector<int> &order, const std::vector<int> &ids,
                      const uint8_t *const *pieces, int ess, int64_t nstripes, int64_t nseg, int64_t piece_seg_stride,
                      int64_t out_seg_stride, uint8_t *out, hipStream_t s);
int rebuild_device(ec_ctx *c, int nshares, const int *nums, const uint8_t *const *pieces, int ess, int64_t nstripes,
                   int64_t nseg, int64_t piece_seg_stride, int64_t out_seg_stride, uint8_t *out, hipStream_t s);
// shape_probe: run the encoder's no-arithmetic form instead (ec_encode_shape_probe)
int encode_range(ec_ctx *c, const uint8_t *segs, size_t nseg, size_t nstripes, size_t s0, size_t s1,
                 uint8_t *pieces, int flags, hipStream_t s, bool shape_probe = false);
size_t align_up(size_t x, size_t a);
B3View data_view(const ec_ctx *c, const uint8_t *segs, size_t nseg, size_t nstripes);
B3View parity_view(const ec_ctx *c, const uint8_t *parity, size_t nseg, size_t nstripes);
size_t b3_segment_ws_bytes(const ec_ctx *c, size_t nseg, size_t nstripes);
int hash_segments(const ec_ctx *c, const uint8_t *segs, const uint8_t *parity, size_t nseg, size_t nstripes,
                  uint8_t *hashes, uint8_t *ws, hipStream_t st);

// ec_sets.cpp
void stop_builder(ec_ctx *c);  // stop and join the context's straight-line builder (ec_destroy)

}  // namespace capi
}  // namespace uplink_ec
#pragma GCC visibility pop
