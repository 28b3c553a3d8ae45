// fsx_api.hip — the C ABI of libfsx_hip.so (include/fsx_hip.h).
//
// Host side of the drop-in boundary: context, device memory, map syscalls and the
// batch entry points that replace the XDP program fsx() (src/fsx_kern.c:96-347)
// and its five maps (src/fsx_kern.c:56-94). No torch types; plain pointers/sizes;
// 0 or -errno; nothing throws across the boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <vector>

#include "../../include/fsx_hip.h"
#include "fsx_internal.h"
#include "fsx_shard.h"

using namespace fsx;

namespace {
constexpr int kMaxEv = 32;   // events per batch (one per kernel)
constexpr int kRing = 64;    // batches of events in flight before a drain
constexpr int kMaxNames = 48;
constexpr uint64_t kMaxBatchLimit = 0x7FFFFFFFull;
}  // namespace

struct fsx_ctx {
    fsx_config cfg{};
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    Slot *table = nullptr;
    uint64_t slots = 0;
    uint64_t id_slots = 0;       // per-batch id table (flow-only batches; FSX_FLAG_OVERFLOW_ADMIT)
    uint64_t tr_slots = 0;       // FSX_FLAG_OVERFLOW_ADMIT: transient slots after the table
    TableState *tstate = nullptr;
    BatchState *bs = nullptr;
    Scratch sc{};
    Limits lim{};
    // host-pointer staging
    uint8_t *d_hdr = nullptr;
    uint32_t *d_len = nullptr;
    uint64_t *d_ts = nullptr;
    uint8_t *d_verdict = nullptr;
    uint64_t stage_cap = 0;
    // scoring staging
    float *d_feat = nullptr;
    float *d_prob = nullptr;
    uint8_t *d_dec = nullptr;
    uint64_t score_cap = 0;
    uint32_t id_gen = 0;       // batch generation: per-batch id table, born stamps
    // persistent source index (TableIndex): heads + IPv6 key words, epoch
    unsigned long long *idx_heads = nullptr;
    uint32_t *idx_k6 = nullptr;
    uint32_t idx_epoch = 1;
    void *idx_mir = nullptr;     // IPv4 mirror of the heads (fsx_internal.h mir_entry; FSX_NO_MIRROR=1: off)
    uint32_t idx_shift = 0;      // log2(slots)
    uint32_t pending_born = 0;  // generation of the in-flight limiter batch (rollback)
    // FSX_FLAG_EVICT_IDLE: survivors' copy (grown on demand), sources evicted before the
    // last limiter batch
    Slot *evict_buf = nullptr;
    uint64_t evict_cap = 0;
    uint64_t last_evicted = 0;
    // FSX_FLAG_EVICT_IDLE: an upper bound on the tracked sources (the last count read plus
    // the packets of every batch since); ~0 = unknown (map imports, reset)
    uint64_t count_bound = ~0ull;
    // the last checked limiter batch inserted more new sources than half its IP packets: the
    // next batches take the home-ordered inserts (FSX_FLAG_ORDERED_INSERTS: always)
    bool flood_hint = false;
    bool light_dom = false;   // the last checked batch: >= 90 % of its IP packets light (Limits::light_dom)
    // sharding: per (owner, tile) counts of fsx_shard_pack_device, blocklist replica
    uint32_t *d_shard_cnt = nullptr;
    uint64_t shard_cnt_cap = 0;
    uint32_t *d_rec_len = nullptr;       // record mode: len / ts written by k_parse
    uint64_t *d_rec_ts = nullptr;
    uint64_t rec_cap = 0;
    unsigned long long *d_shard_stat = nullptr;   // per (tile, owner) look-back words (k_shard_place16)
    uint32_t *d_shard_ticket = nullptr;
    uint8_t *d_shard_own = nullptr;      // per packet owner (k_shard_parse)
    void *d_shard_crec = nullptr;        // per packet 16-byte record in arrival order
    uint64_t shard_scr_cap = 0;
    ShardBlock *d_rep = nullptr;
    uint64_t rep_slots = 0;
    bool rep_valid = false;
    // sliding-window history (limiter == FSX_LIMIT_SLIDING_WINDOW only)
    HistBufs hist{};
    // per-source flow accumulators
    void *d_flow_acc = nullptr;
    uint64_t flow_acc_cap = 0;
    // fsx_flows_begin .. fsx_flows_end: per table slot sums carried across calls
    void *d_slot_acc = nullptr;
    unsigned long long *d_flow_rows = nullptr;
    uint32_t flow_epoch = 0;
    bool flow_accum = false;
    // prefix blocklists (FSX_MAP_IPV4_PREFIX / _IPV6_PREFIX): the host copy is the map;
    // the device probe table is rebuilt from it before the next batch after a change
    std::map<std::array<uint32_t, 5>, uint64_t> rules;   // {family << 8 | len, addr words}
    uint32_t rule_cnt[2]{};
    uint32_t rule_len_cnt[2][129]{};
    bool rules_dirty = false;
    RuleSlot *d_rule_slot = nullptr;
    uint8_t *d_rule_lens = nullptr;
    uint32_t *d_rule_filter = nullptr;
    uint64_t rule_cap = 0;
    RuleSet rs{};
    // small device scratch for map ops
    int32_t *d_res = nullptr;
    uint64_t *d_val = nullptr;
    // model
    bool model_loaded = false;
    int8_t w[8]{};
    float inv_in = 0, bias_over_ats = 0, mult = 0;
    int32_t zp_in = 0, zp_out = 0;
    uint8_t lut[256]{};
    // timing
    bool timing = false;
    bool ev_ready = false;
    hipEvent_t ev[kRing][kMaxEv]{};
    const char *ev_names[kRing][kMaxEv]{};
    int ev_prev[kRing][kMaxEv]{};
    int ev_used[kRing]{};
    // second stream: flow features beside the limiter (fork / join events)
    hipStream_t aux_stream = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    hipEvent_t wait_ev = nullptr;     // fsx_stream_wait_batches
    hipStream_t walk_stream = nullptr;   // third stream: long-segment walker
    hipEvent_t walk_fork_ev = nullptr, walk_join_ev = nullptr;
    hipEvent_t heavy_fork_ev = nullptr, heavy_flow_ev = nullptr;   // heavy work after the sort
    int ring_n = 0;
    const char *acc_name[kMaxNames]{};
    double acc_ms[kMaxNames]{};
    uint64_t acc_cnt[kMaxNames]{};
    int acc_n = 0;
    uint64_t acc_batches = 0;
    bool pending = false;
    // batch pipelining (fsx_set_pipeline): two sets of the front buffers (sort arrays,
    // BatchState), the batch of each set still in flight, the tail-done event per set
    struct FrontBufs {
        uint64_t *packed[2], *pay[2];
        uint32_t *hist, *sort_ctl, *gbase;
        HeavySet *heavy;
        uint32_t *chunk_cnt;
        void *hrec;
        BatchState *bs;
    };
    int pipe = 0;                     // fsx_set_pipeline mode (2: never split front / tail)
    static constexpr int kSets = 3;   // front buffer sets: batch k waits only for batch k - 3
    FrontBufs fb[kSets]{};
    int par = 0;                      // set of the last pipelined batch
    bool fl_on[kSets]{};              // a pipelined batch of set p is in flight
    uint32_t fl_born[kSets]{};
    hipEvent_t tail_done[kSets]{};
    hipEvent_t front_done = nullptr;  // after the last pipelined batch's sort
    hipEvent_t parse_done = nullptr;  // after the current pipelined batch's parse
    hipEvent_t pro_wait = nullptr, pro_done = nullptr;   // early prologue (PipeSplit)
    // context-stream work other than a split batch's front was enqueued since pro_wait was
    // last recorded (every other entry point goes through sel()): the next early prologue
    // waits for all of it
    bool pro_fence = true;
    TailArgs tail_args{};             // the last pipelined batch's tail, not yet enqueued
    bool tail_pending = false;
    int tail_par = 0;
    int tail_prev = -1;               // set of the last tail enqueued (its completion: tail_done)
    bool tail_join = false;           // the last pipelined batch's tail is not joined into stream
    // fsx_reset between pipelined batches (fixed window / token bucket): a second table set
    // (slots, scalars, index) is swapped in and cleared on the device after the last tail
    // that used it, so the reset neither waits on the host nor orders the next front after
    // the last tail (DESIGN.md §3 "Pipelined resets"); FSX_RESET_SYNC=1: the synchronous reset
    struct TableSet {
        Slot *table = nullptr;
        TableState *tstate = nullptr;
        unsigned long long *heads = nullptr;
        uint32_t *k6 = nullptr;
        void *mir = nullptr;
        uint32_t epoch = 1;
    };
    TableSet spare{};
    // the spare's last users: the walk / aux streams after its tails (and after the deferred
    // tail too, when it is enqueued), the context stream after its fronts
    hipEvent_t spare_free[3]{};
    bool spare_tail = false;
    hipStream_t clr_stream = nullptr; // the swapped-in set is cleared here, beside the last front
    hipEvent_t clr_done = nullptr;
    bool spare_dirty = false;         // the spare holds lines of table generations that come round again
    uint32_t tgen = 0;                // table generation: one per pipelined reset
    uint32_t fl_tgen[kSets]{};
    bool fresh_tables = false;        // the next pipelined batch starts a table generation
    // record mode, pipelined: the records' len / ts per front set (a split tail reads its
    // batch's while the next front writes its own); max_batch each, allocated on first use
    uint32_t *rec_len_set[kSets]{};
    uint64_t *rec_ts_set[kSets]{};
    char err[512]{};
};

static int set_err(fsx_ctx *c, int code, const char *fmt, ...) {
    if (c) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(c->err, sizeof(c->err), fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(c, x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
            return set_err((c), -EIO, "%s failed: %s", #x, hipGetErrorString(e_));     \
    } while (0)

static uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

static void free_scratch(fsx_ctx *c) {
    Scratch &s = c->sc;
    hipFree(s.packed[0]); hipFree(s.packed[1]); hipFree(s.pay[0]); hipFree(s.pay[1]); hipFree(s.marks); hipFree(s.headf);
    hipFree(s.seg_start); hipFree(s.seg_slot); hipFree(s.seg_lo); hipFree(s.seg_len); hipFree(s.hist);
    hipFree(s.tile_aux); hipFree(s.tile_last); hipFree(s.id_tab);
    hipFree(s.seg_order); hipFree(s.seg_cls); hipFree(s.sub_cnt); hipFree(s.flow_first); hipFree(s.flow_last);
    hipFree(s.span_list); hipFree(s.sort_ctl); hipFree(s.gbase); hipFree(s.status);
    hipFree(s.lim_tiles); hipFree(s.sw_seg); hipFree(s.sketch); hipFree(s.heavy);
    hipFree(s.drop_list); hipFree(s.drop_cur); hipFree(s.heavy_flow);
    hipFree(s.chunk_cnt); hipFree(s.hrec); hipFree(s.hflow); hipFree(s.tbh); hipFree(s.dig);
    hipFree(s.admit_rank); hipFree(s.admit_cnt);
    s = Scratch{};
}

static int alloc_scratch(fsx_ctx *c, uint64_t cap) {
    if (cap <= c->sc.cap) return 0;
    free_scratch(c);
    Scratch &s = c->sc;
    const uint64_t ntiles = cap / kTile + 2;
    HIPCHK(c, hipMalloc(&s.packed[0], cap * 8));
    HIPCHK(c, hipMalloc(&s.packed[1], cap * 8));
    HIPCHK(c, hipMalloc(&s.pay[0], cap * 8));
    HIPCHK(c, hipMalloc(&s.pay[1], cap * 8));
    HIPCHK(c, hipMalloc(&s.marks, cap + 16));
    HIPCHK(c, hipMalloc(&s.dig, 2 * cap + 32));   // (16-bit words for 9-bit digits)
    HIPCHK(c, hipMalloc(&s.headf, cap + 16));
    HIPCHK(c, hipMalloc(&s.seg_start, (cap + 1) * 4));
    HIPCHK(c, hipMalloc(&s.seg_slot, cap * 4));
    HIPCHK(c, hipMalloc(&s.seg_lo, (cap + 1) * 4));
    HIPCHK(c, hipMalloc(&s.seg_len, (cap + 1) * 4));
    // (two regions: pass 0's 256 rows and the light passes' 512 — 9-bit digits —,
    // launch_verdict_pipeline)
    HIPCHK(c, hipMalloc(&s.hist, 256ull * std::max<uint64_t>(kSortMaxBlocks, 3 * (cap / kSortTile + 2)) * 4));
    HIPCHK(c, hipMalloc(&s.tile_aux, ntiles * 4));
    HIPCHK(c, hipMalloc(&s.tile_last, ntiles));
    // (s.id_tab, the per-batch id table of flow-only batches, is allocated on first use:
    // slots * 32 bytes, 16 GiB for a 2^28-source context that never needs it)
    c->id_gen = 0;
    HIPCHK(c, hipMalloc(&s.seg_order, (cap + 1) * 4));
    HIPCHK(c, hipMalloc(&s.seg_cls, kSegClassWords * 4));
    HIPCHK(c, hipMalloc(&s.sub_cnt, (cap / 1024 + 8) * 4));
    HIPCHK(c, hipMalloc(&s.flow_first, (cap / 1024 + 8) * flow_acc_bytes()));
    HIPCHK(c, hipMalloc(&s.flow_last, (cap / 1024 + 8) * flow_acc_bytes()));
    HIPCHK(c, hipMalloc(&s.span_list, (cap / 1024 + 8) * 4));
    HIPCHK(c, hipMalloc(&s.sort_ctl, kSortCtlWords * 4));
    HIPCHK(c, hipMalloc(&s.gbase, 1536 * 4));   // (+ the 9-bit passes' 512 bases)
    HIPCHK(c, hipMalloc(&s.status, (cap / kSortTile + 2) * 256 * 8));
    HIPCHK(c, hipMemset(s.status, 0, (cap / kSortTile + 2) * 256 * 8));
    s.lim_tiles_n = cap / kTile + 2;
    HIPCHK(c, hipMalloc(&s.lim_tiles, s.lim_tiles_n * 4 * 8));
    if (c->cfg.limiter == FSX_LIMIT_SLIDING_WINDOW) HIPCHK(c, hipMalloc(&s.sw_seg, cap * sizeof(SwSeg)));
    const uint64_t nchunks = (cap + kVChunk - 1) / kVChunk;
    HIPCHK(c, hipMalloc(&s.drop_list, nchunks * kVChunk * 4));
    HIPCHK(c, hipMalloc(&s.drop_cur, nchunks * 4));
    HIPCHK(c, hipMemset(s.drop_cur, 0, nchunks * 4));
    HIPCHK(c, hipMalloc(&s.sketch, 4 * kSketch * 4));
    HIPCHK(c, hipMemset(s.sketch, 0, 4 * kSketch * 4));
    HIPCHK(c, hipMalloc(&s.heavy, sizeof(HeavySet)));
    HIPCHK(c, hipMemset(s.heavy, 0, sizeof(HeavySet)));
    HIPCHK(c, hipMalloc(&s.heavy_flow, heavy_flow_bytes(cap)));
    HIPCHK(c, hipMalloc(&s.chunk_cnt, chunk_cnt_bytes(cap)));
    HIPCHK(c, hipMalloc(&s.hrec, heavy_rec_bytes(cap)));
    HIPCHK(c, hipMalloc(&s.hflow, hflow_bytes(cap)));
    if (c->cfg.limiter == FSX_LIMIT_TOKEN_BUCKET) HIPCHK(c, hipMalloc(&s.tbh, tb_heavy_bytes(cap)));
    s.cap = cap;
    return 0;
}

extern "C" {

int fsx_abi_version(void) { return FSX_ABI_VERSION; }

void fsx_config_default(fsx_config *cfg) {
    if (!cfg) return;
    memset(cfg, 0, sizeof(*cfg));
    cfg->pps_threshold = 1000;          // src/fsx_kern.c:309
    cfg->bps_threshold = 125000000;     // src/fsx_kern.c:310
    cfg->window_ns = 1000000000ull;     // src/fsx_kern.c:245
    cfg->block_ns = 10ull * 1000000000ull;  // src/fsx_kern.c:308,317
    cfg->max_entries = 100000;          // MAX_TRACK_IPS, src/fsx_struct.h:7
    cfg->max_batch = 1u << 20;
    cfg->tb_rate = 1000;
    cfg->tb_burst = 1000;
    cfg->hash_seed = 0x5EED0F5A0ull;
    cfg->limiter = FSX_LIMIT_FIXED_WINDOW;
    cfg->device = 0;
}

const char *fsx_last_error(const fsx_ctx *ctx) { return ctx ? ctx->err : "null context"; }

// The deferred tail of the last pipelined batch onto the walker stream (and the flows on the
// aux stream), after event `after` on the context stream.
// A tail whose flows run on the aux stream ends there (the aux stream waits for the
// walker stream's verdict apply): the walker stream is free for the next batch's early
// prologue at once, and the next tail starts after this one's flows (tail_done), which
// share the segment arrays with it.
static hipError_t flush_tail(fsx_ctx *c, hipEvent_t after) {
    if (!c->tail_pending) return hipSuccess;
    c->tail_pending = false;
    hipError_t e;
    if ((e = hipStreamWaitEvent(c->walk_stream, after, 0)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(c->aux_stream, after, 0)) != hipSuccess) return e;
    if (c->tail_prev >= 0 && (e = hipStreamWaitEvent(c->walk_stream, c->tail_done[c->tail_prev], 0)) != hipSuccess)
        return e;
    if ((e = launch_tail(c->tail_args)) != hipSuccess) return e;
    c->tail_prev = c->tail_par;
    if (c->spare_tail) {   // (the tail of the last batch before a pipelined reset: the spare's last user)
        c->spare_tail = false;
        if ((e = hipEventRecord(c->spare_free[0], c->walk_stream)) != hipSuccess) return e;
        if ((e = hipEventRecord(c->spare_free[1], c->aux_stream)) != hipSuccess) return e;
    }
    static const bool end_aux = getenv("FSX_TAIL_END_AUX") != nullptr;
    return hipEventRecord(c->tail_done[c->tail_par], c->tail_args.fork && end_aux ? c->aux_stream : c->walk_stream);
}

// PipeSplit::on_parse: the previous batch's tail goes in beside this batch's parse (before it by default).
static hipError_t pipe_on_parse(void *p, hipEvent_t recorded) {
    fsx_ctx *c = static_cast<fsx_ctx *>(p);
    if (!c->tail_pending) return hipSuccess;
    if (recorded) return flush_tail(c, recorded);
    hipError_t e = hipEventRecord(c->parse_done, c->stream);
    return e != hipSuccess ? e : flush_tail(c, c->parse_done);
}

// Every entry point except the batch calls: the last pipelined batch's tail is enqueued and
// the context stream continues after it (the tail runs on its own streams).
static int sel(fsx_ctx *c) {
    HIPCHK(c, hipSetDevice(c->device));
    c->pro_fence = true;
    if (c->tail_pending) {
        hipError_t e = flush_tail(c, c->front_done);
        if (e != hipSuccess) return set_err(c, -EIO, "pipelined tail: %s", hipGetErrorString(e));
    }
    if (c->tail_join) {
        c->tail_join = false;
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->tail_done[c->par], 0));
    }
    return 0;
}

static bool pipe_busy(const fsx_ctx *c) {
    for (int p = 0; p < fsx_ctx::kSets; ++p)
        if (c->fl_on[p]) return true;
    return false;
}
static bool busy(const fsx_ctx *c) { return c->pending || pipe_busy(c); }

// The front buffers of set p become the context's current sort arrays and BatchState.
static void use_front(fsx_ctx *c, int p) {
    const fsx_ctx::FrontBufs &f = c->fb[p];
    for (int b = 0; b < 2; ++b) { c->sc.packed[b] = f.packed[b]; c->sc.pay[b] = f.pay[b]; }
    c->sc.hist = f.hist;
    c->sc.sort_ctl = f.sort_ctl;
    c->sc.gbase = f.gbase;
    c->sc.heavy = f.heavy;
    c->sc.chunk_cnt = f.chunk_cnt;
    c->sc.hrec = f.hrec;
    c->bs = f.bs;
}

static void free_front(fsx_ctx::FrontBufs &f) {
    for (int b = 0; b < 2; ++b) { hipFree(f.packed[b]); hipFree(f.pay[b]); }
    hipFree(f.hist); hipFree(f.sort_ctl); hipFree(f.gbase); hipFree(f.heavy); hipFree(f.bs);
    hipFree(f.chunk_cnt); hipFree(f.hrec);
    f = fsx_ctx::FrontBufs{};
}

void fsx_close(fsx_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    sel(c);   // (a pipelined batch's deferred tail)
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->walk_stream) hipStreamSynchronize(c->walk_stream);
    if (c->aux_stream) hipStreamSynchronize(c->aux_stream);
    if (c->fb[0].bs) use_front(c, 0);   // (set 0 owns what free_scratch frees)
    for (int p = 1; p < fsx_ctx::kSets; ++p)
        if (c->fb[p].bs) free_front(c->fb[p]);
    for (int p = 0; p < fsx_ctx::kSets; ++p) if (c->tail_done[p]) hipEventDestroy(c->tail_done[p]);
    if (c->front_done) hipEventDestroy(c->front_done);
    if (c->parse_done) hipEventDestroy(c->parse_done);
    if (c->pro_wait) hipEventDestroy(c->pro_wait);
    if (c->pro_done) hipEventDestroy(c->pro_done);
    free_scratch(c);
    hipFree(c->table); hipFree(c->tstate); hipFree(c->bs);
    hipFree(c->d_hdr); hipFree(c->d_len); hipFree(c->d_ts); hipFree(c->d_verdict);
    hipFree(c->d_feat); hipFree(c->d_prob); hipFree(c->d_dec); hipFree(c->d_flow_acc);
    hipFree(c->d_slot_acc); hipFree(c->d_flow_rows);
    hipFree(c->d_res); hipFree(c->d_val);
    for (int b = 0; b < 2; ++b) { hipFree(c->hist.t[b]); hipFree(c->hist.l[b]); }
    hipFree(c->hist.tile_cnt); hipFree(c->hist.tile_off); hipFree(c->hist.total);
    hipFree(c->d_shard_cnt); hipFree(c->d_rep); hipFree(c->d_shard_own); hipFree(c->d_shard_crec);
    hipFree(c->d_shard_stat); hipFree(c->d_shard_ticket);
    hipFree(c->d_rec_len); hipFree(c->d_rec_ts);
    for (int p = 0; p < fsx_ctx::kSets; ++p) { hipFree(c->rec_len_set[p]); hipFree(c->rec_ts_set[p]); }
    hipFree(c->spare.table); hipFree(c->spare.tstate); hipFree(c->spare.heads); hipFree(c->spare.k6);
    hipFree(c->spare.mir);
    for (int k = 0; k < 3; ++k) if (c->spare_free[k]) hipEventDestroy(c->spare_free[k]);
    if (c->clr_done) hipEventDestroy(c->clr_done);
    if (c->clr_stream) hipStreamDestroy(c->clr_stream);
    hipFree(c->idx_heads); hipFree(c->idx_k6); hipFree(c->idx_mir);
    hipFree(c->evict_buf);
    hipFree(c->d_rule_slot); hipFree(c->d_rule_lens); hipFree(c->d_rule_filter);
    for (int r = 0; r < kRing; ++r)
        for (int i = 0; i < kMaxEv; ++i) if (c->ev[r][i]) hipEventDestroy(c->ev[r][i]);
    if (c->own_stream) hipStreamDestroy(c->own_stream);
    if (c->aux_stream) hipStreamDestroy(c->aux_stream);
    if (c->walk_stream) hipStreamDestroy(c->walk_stream);
    if (c->walk_fork_ev) hipEventDestroy(c->walk_fork_ev);
    if (c->walk_join_ev) hipEventDestroy(c->walk_join_ev);
    if (c->heavy_fork_ev) hipEventDestroy(c->heavy_fork_ev);
    if (c->heavy_flow_ev) hipEventDestroy(c->heavy_flow_ev);
    if (c->fork_ev) hipEventDestroy(c->fork_ev);
    if (c->join_ev) hipEventDestroy(c->join_ev);
    if (c->wait_ev) hipEventDestroy(c->wait_ev);
    delete c;
}

int fsx_open(fsx_ctx **out, const fsx_config *cfg) {
    if (!out) return -EINVAL;
    *out = nullptr;
    fsx_config k;
    if (cfg) k = *cfg; else fsx_config_default(&k);
    // slots = next_pow2(2 * max_entries) <= 2^32: a source id (its slot) fills at most the
    // sort word's 32 id bits (fsx_internal.h pk_id)
    if (k.max_entries == 0 || k.max_entries > (1ull << 31)) return -EINVAL;
    if (k.max_batch == 0 || k.max_batch > kMaxBatchLimit) return -EINVAL;
    if (k.limiter < FSX_LIMIT_FIXED_WINDOW || k.limiter > FSX_LIMIT_TOKEN_BUCKET) return -EINVAL;
    // token bucket: capacity burst * 1e9 nano-tokens must stay <= 2^61
    if (k.limiter == FSX_LIMIT_TOKEN_BUCKET && k.tb_burst > FSX_TB_MAX_BURST) return -EINVAL;
    // sliding window: a carried log holds <= pps_threshold entries (24-bit count)
    if (k.limiter == FSX_LIMIT_SLIDING_WINDOW && k.pps_threshold > FSX_SW_MAX_PPS) return -EINVAL;
    // idle eviction is defined for the reference's fixed window only
    if ((k.flags & FSX_FLAG_EVICT_IDLE) && k.limiter != FSX_LIMIT_FIXED_WINDOW) return -EINVAL;
    // admission: transient slots (slots + segment id) must stay below 2^32 (u32 seg_slot)
    const bool admit = (k.flags & FSX_FLAG_OVERFLOW_ADMIT) != 0;
    if (admit && next_pow2(std::max<uint64_t>(1024, 2 * k.max_entries)) + k.max_batch >= (1ull << 32)) return -EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return -ENODEV;
    if (k.device < 0 || k.device >= ndev) return -EINVAL;
    fsx_ctx *c = new (std::nothrow) fsx_ctx();
    if (!c) return -ENOMEM;
    c->cfg = k;
    c->device = k.device;
    int rc = sel(c);
    if (rc) { fsx_close(c); return rc; }
    c->slots = next_pow2(std::max<uint64_t>(1024, 2 * k.max_entries));
    c->tr_slots = admit ? k.max_batch : 0;
    c->id_slots = admit ? std::max<uint64_t>(c->slots, next_pow2(std::max<uint64_t>(1024, 2 * k.max_batch))) : c->slots;
    auto fail = [&](int r) { fsx_close(c); return r; };
    // stream priorities (A/B: FSX_STREAM_PRIO="own,aux,walk", lower = more urgent): the
    // context stream (parse, sort) first, so a pipelined batch's short sort scans find CU
    // slots among the previous batch's tail (-0.6 % per step, profiles/r03/ab_prio/)
    int prio[3] = {-1, 0, 0};
    if (const char *ps = getenv("FSX_STREAM_PRIO")) sscanf(ps, "%d,%d,%d", &prio[0], &prio[1], &prio[2]);
    if (hipStreamCreateWithPriority(&c->own_stream, hipStreamNonBlocking, prio[0]) != hipSuccess) return fail(-EIO);
    if (hipStreamCreateWithPriority(&c->aux_stream, hipStreamNonBlocking, prio[1]) != hipSuccess) return fail(-EIO);
    if (hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) != hipSuccess) return fail(-EIO);
    if (hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming) != hipSuccess) return fail(-EIO);
    if (hipStreamCreateWithPriority(&c->walk_stream, hipStreamNonBlocking, prio[2]) != hipSuccess) return fail(-EIO);
    if (hipEventCreateWithFlags(&c->walk_fork_ev, hipEventDisableTiming) != hipSuccess) return fail(-EIO);
    if (hipEventCreateWithFlags(&c->walk_join_ev, hipEventDisableTiming) != hipSuccess) return fail(-EIO);
    if (hipEventCreateWithFlags(&c->heavy_fork_ev, hipEventDisableTiming) != hipSuccess) return fail(-EIO);
    if (hipEventCreateWithFlags(&c->heavy_flow_ev, hipEventDisableTiming) != hipSuccess) return fail(-EIO);
    c->stream = c->own_stream;
    if (hipMalloc(&c->table, (c->slots + c->tr_slots) * sizeof(Slot)) != hipSuccess) return fail(-ENOMEM);
    if (hipMalloc(&c->tstate, sizeof(TableState)) != hipSuccess) return fail(-ENOMEM);
    if (hipMalloc(&c->bs, sizeof(BatchState)) != hipSuccess) return fail(-ENOMEM);
    if (hipMalloc(&c->d_res, 64) != hipSuccess) return fail(-ENOMEM);
    if (hipMalloc(&c->d_val, 64) != hipSuccess) return fail(-ENOMEM);
    if (hipMemset(c->table, 0, c->slots * sizeof(Slot)) != hipSuccess) return fail(-EIO);
    if (hipMalloc(&c->idx_heads, c->slots * 8) != hipSuccess) return fail(-ENOMEM);
    if (hipMalloc(&c->idx_k6, c->slots * 16) != hipSuccess) return fail(-ENOMEM);
    if (hipMemset(c->idx_heads, 0, c->slots * 8) != hipSuccess) return fail(-EIO);
    c->idx_epoch = 1;
    while ((1ull << c->idx_shift) < c->slots) ++c->idx_shift;
    if (!getenv("FSX_NO_MIRROR") && mir_bytes(c->idx_shift)) {
        if (hipMalloc(&c->idx_mir, mir_bytes(c->idx_shift)) != hipSuccess) return fail(-ENOMEM);
        if (hipMemset(c->idx_mir, 0, mir_bytes(c->idx_shift)) != hipSuccess) return fail(-EIO);
    }
    if (hipMemset(c->tstate, 0, sizeof(TableState)) != hipSuccess) return fail(-EIO);
    if (hipMemset(c->bs, 0, sizeof(BatchState)) != hipSuccess) return fail(-EIO);
    if (alloc_scratch(c, k.max_batch)) return fail(-ENOMEM);
    {
        fsx_ctx::FrontBufs &f = c->fb[0];
        for (int b = 0; b < 2; ++b) { f.packed[b] = c->sc.packed[b]; f.pay[b] = c->sc.pay[b]; }
        f.hist = c->sc.hist; f.sort_ctl = c->sc.sort_ctl; f.gbase = c->sc.gbase; f.heavy = c->sc.heavy;
        f.chunk_cnt = c->sc.chunk_cnt; f.hrec = c->sc.hrec;
        f.bs = c->bs;
    }
    if (k.limiter == FSX_LIMIT_SLIDING_WINDOW) {
        HistBufs &h = c->hist;
        h.cap = std::max<uint64_t>(2 * k.max_batch, 1u << 16);
        const uint64_t stiles = c->slots / 4096 + 1;
        // (past cap: the heavy sources' staged final logs, k_walk_sw_heavy_sel)
        const uint64_t ent = h.cap + (uint64_t)kHeavyMax * kSwHeavyMaxP;
        for (int b = 0; b < 2; ++b) {
            if (hipMalloc(&h.t[b], ent * 8) != hipSuccess) return fail(-ENOMEM);
            if (hipMalloc(&h.l[b], ent * 4) != hipSuccess) return fail(-ENOMEM);
        }
        if (hipMalloc(&h.tile_cnt, stiles * 4) != hipSuccess) return fail(-ENOMEM);
        if (hipMalloc(&h.tile_off, stiles * 8) != hipSuccess) return fail(-ENOMEM);
        if (hipMalloc(&h.total, 8) != hipSuccess) return fail(-ENOMEM);
    }
    Limits &L = c->lim;
    L.pps = k.pps_threshold; L.bps = k.bps_threshold; L.window = k.window_ns; L.block = k.block_ns;
    L.tb_rate = k.tb_rate;
    L.tb_cap = std::min<uint64_t>(k.tb_burst, FSX_TB_MAX_BURST) * 1000000000ull;
    L.max_entries = k.max_entries;
    L.hist_cap = c->hist.cap;
    L.table_mask = c->slots - 1;
    L.seed = mix64(k.hash_seed);
    L.salt32 = (uint32_t)(mix64(k.hash_seed ^ 0xABCDEFull) >> 32);
    L.limiter = k.limiter;
    L.test_flags = k.flags;
    L.admit_mask = admit ? c->id_slots - 1 : 0;
    if (admit) {   // the per-batch id table and the rank scratch, up front
        if (hipMalloc(&c->sc.id_tab, c->id_slots * 32) != hipSuccess) return fail(-ENOMEM);
        if (hipMemset(c->sc.id_tab, 0, c->id_slots * 32) != hipSuccess) return fail(-EIO);
        if (hipMalloc(&c->sc.admit_rank, std::max<uint64_t>(1, k.max_batch) * 4) != hipSuccess) return fail(-ENOMEM);
        if (hipMalloc(&c->sc.admit_cnt, (k.max_batch / kTile + 2) * 4) != hipSuccess) return fail(-ENOMEM);
    }
    if (hipDeviceSynchronize() != hipSuccess) return fail(-EIO);
    *out = c;
    return 0;
}

int fsx_set_stream(fsx_ctx *c, void *s) {
    if (!c) return -EINVAL;
    int rc = sel(c);   // (the old stream joins the last pipelined tail)
    if (rc) return rc;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return 0;
}

static TableIndex table_index(const fsx_ctx *c) {
    return TableIndex{c->idx_heads, c->idx_k6, c->idx_epoch, c->idx_mir, c->idx_shift};
}

// New epoch of the persistent index (every head reads empty); heads are cleared once
// per 2^16 epochs so a stale cached line can never carry a current epoch. The IPv4 mirror
// carries no epoch: it is cleared at every epoch change (ordered before the next kernel
// on the context stream; the survivors' entries are re-published by the rebuild).
static int next_epoch(fsx_ctx *c) {
    if (++c->idx_epoch == 0x10000u) {
        HIPCHK(c, hipMemsetAsync(c->idx_heads, 0, c->slots * 8, c->stream));
        c->idx_epoch = 1;
    }
    if (c->idx_mir) HIPCHK(c, hipMemsetAsync(c->idx_mir, 0, mir_bytes(c->idx_shift), c->stream));
    return 0;
}

// A limiter batch failed after k_parse inserted its new sources: drop them and
// re-publish the survivors under a new epoch (no map state changed: every limiter
// kernel skips a batch whose error flag is set).
static int rollback_batch(fsx_ctx *c, uint32_t born) {
    int rc = next_epoch(c);
    if (rc) return rc;
    hipError_t e = launch_index_rebuild(c->table, c->lim, table_index(c), born, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "index rebuild: %s", hipGetErrorString(e));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

static int batch_error(fsx_ctx *c, uint32_t err);

// A finished batch's facts the host keeps: a flood of new sources (home-ordered inserts next).
static void note_batch(fsx_ctx *c, const BatchState &h) {
    if (!h.err && h.n_valid) {
        c->flood_hint = 2ull * h.n_new > h.n_valid;
        c->light_dom = 10ull * h.n_light >= 9ull * h.n_valid;
    }
}

static int check_batch(fsx_ctx *c) {
    if (!c->pending) return 0;
    c->pending = false;
    const uint32_t born = c->pending_born;
    c->pending_born = 0;
    BatchState h;
    HIPCHK(c, hipMemcpy(&h, c->bs, sizeof(h), hipMemcpyDeviceToHost));
    note_batch(c, h);
    if (h.err && born) {
        const int rc = rollback_batch(c, born);
        if (rc) return rc;
    }
    return batch_error(c, h.err);
}

// Pipelined batches still in flight, oldest first, with the device idle: the first failed
// one and every later one (cancelled on the device) are rolled back; its error is returned.
static int check_pipelined(fsx_ctx *c) {
    int rc = 0;
    bool failed = false;
    uint32_t fgen = 0;   // (a failure cancels the later batches of its table generation only)
    for (int i = 1; i <= fsx_ctx::kSets; ++i) {   // oldest set first
        const int p = (c->par + i) % fsx_ctx::kSets;
        if (!c->fl_on[p]) continue;
        c->fl_on[p] = false;
        BatchState h;
        HIPCHK(c, hipMemcpy(&h, c->fb[p].bs, sizeof(h), hipMemcpyDeviceToHost));
        note_batch(c, h);
        const bool cancelled = failed && c->fl_tgen[p] == fgen;
        if (!h.err && !cancelled) continue;
        // (a batch on tables a pipelined reset has since replaced changed nothing that is
        // still visible: no rollback)
        if (c->fl_born[p] && c->fl_tgen[p] == c->tgen) {
            const int r = rollback_batch(c, c->fl_born[p]);
            if (r) return r;
        }
        if (!failed) rc = batch_error(c, h.err);
        if (!failed || c->fl_tgen[p] != fgen) fgen = c->fl_tgen[p];
        failed = true;
    }
    // (the tail-side cancel flag of split sliding-window batches: everything it cancelled
    // is rolled back now)
    if (failed) HIPCHK(c, hipMemsetAsync(&c->tstate->tail_fail, 0, sizeof(uint32_t), c->stream));
    return rc;
}

static int batch_error(fsx_ctx *c, uint32_t err) {
    if (err & ERR_TABLE_FULL)
        return set_err(c, -ENOSPC, "map full: more than max_entries=%llu source IPs",
                       (unsigned long long)c->cfg.max_entries);
    if (err & ERR_FIXUP)
        return set_err(c, -EIO, "home-ordered inserts: more than %u packets share one key hash with two sources",
                       512u);
    if (err & ERR_HIST_FULL)
        return set_err(c, -ENOSPC, "sliding-window history full: carried logs + batch > %llu entries",
                       (unsigned long long)c->hist.cap);
    if (err & ERR_HEAVY_VIEW)
        return set_err(c, -EIO, "heavy-source rank view: inconsistent tile-count row or tags (flags 0x%x)", err);
    if (err & ERR_SORT_HANG)
        return set_err(c, -EIO, "a decoupled look-back timed out (flags 0x%x)", err);
    if (err) return set_err(c, -EIO, "device error flags 0x%x", err);
    return 0;
}

int fsx_sync(fsx_ctx *c) {
    if (!c) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((rc = check_pipelined(c))) return rc;
    return check_batch(c);
}

int fsx_stream_wait_batches(fsx_ctx *c, void *hip_stream, int all) {
    if (!c) return -EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    if (all) {   // the last batch's deferred tail goes in first; the context stream joins it
        const int rc = sel(c);
        if (rc) return rc;
    }
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    // the enqueued split tails end in order (each starts after the one before: flush_tail)
    if (c->tail_prev >= 0 && c->tail_done[c->tail_prev])
        HIPCHK(c, hipStreamWaitEvent(s, c->tail_done[c->tail_prev], 0));
    if (s != c->stream) {   // and everything on the context stream so far
        if (!c->wait_ev) HIPCHK(c, hipEventCreateWithFlags(&c->wait_ev, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(c->wait_ev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->wait_ev, 0));
    }
    return 0;
}

static int alloc_spare(fsx_ctx *c);

int fsx_set_pipeline(fsx_ctx *c, int on) {
    if (!c) return -EINVAL;
    int rc = fsx_sync(c);
    if (rc) return rc;
    for (int fs = 1; on && fs < fsx_ctx::kSets; ++fs) {
        if (c->fb[fs].bs) continue;
        // built in a temporary set and committed only when every allocation succeeded (bs,
        // allocated last, marks a set as present); a partial set is freed
        fsx_ctx::FrontBufs f{};
        const uint64_t cap = c->sc.cap;
        auto build = [&]() -> hipError_t {
            hipError_t e;
            for (int b = 0; b < 2; ++b) {
                if ((e = hipMalloc(&f.packed[b], cap * 8)) != hipSuccess) return e;
                if ((e = hipMalloc(&f.pay[b], cap * 8)) != hipSuccess) return e;
            }
            if ((e = hipMalloc(&f.hist, 256ull * std::max<uint64_t>(kSortMaxBlocks, 3 * (cap / kSortTile + 2)) * 4)) != hipSuccess) return e;
            if ((e = hipMalloc(&f.sort_ctl, kSortCtlWords * 4)) != hipSuccess) return e;
            if ((e = hipMalloc(&f.gbase, 1536 * 4)) != hipSuccess) return e;
            if ((e = hipMalloc(&f.heavy, sizeof(HeavySet))) != hipSuccess) return e;
            if ((e = hipMemset(f.heavy, 0, sizeof(HeavySet))) != hipSuccess) return e;
            if ((e = hipMalloc(&f.chunk_cnt, chunk_cnt_bytes(cap))) != hipSuccess) return e;
            if ((e = hipMalloc(&f.hrec, heavy_rec_bytes(cap))) != hipSuccess) return e;
            if ((e = hipMalloc(&f.bs, sizeof(BatchState))) != hipSuccess) return e;
            return hipMemset(f.bs, 0, sizeof(BatchState));
        };
        const hipError_t be = build();
        if (be != hipSuccess) {
            free_front(f);
            return set_err(c, -ENOMEM, "pipeline buffers: %s", hipGetErrorString(be));
        }
        c->fb[fs] = f;
        for (int p = 0; p < fsx_ctx::kSets; ++p)
            if (!c->tail_done[p]) HIPCHK(c, hipEventCreateWithFlags(&c->tail_done[p], hipEventDisableTiming));
        if (!c->front_done) HIPCHK(c, hipEventCreateWithFlags(&c->front_done, hipEventDisableTiming));
        if (!c->parse_done) HIPCHK(c, hipEventCreateWithFlags(&c->parse_done, hipEventDisableTiming));
        if (!c->pro_wait) HIPCHK(c, hipEventCreateWithFlags(&c->pro_wait, hipEventDisableTiming));
        if (!c->pro_done) HIPCHK(c, hipEventCreateWithFlags(&c->pro_done, hipEventDisableTiming));
    }
    if (!on && c->par != 0) {   // back to set 0, keeping the last batch's facts
        HIPCHK(c, hipMemcpy(c->fb[0].bs, c->fb[c->par].bs, sizeof(BatchState), hipMemcpyDeviceToDevice));
        use_front(c, 0);
        c->par = 0;
    }
    c->pipe = on < 0 ? 0 : on > 2 ? 1 : on;
    if (c->pipe == 1) {   // (resets between pipelined batches: DESIGN.md §3 "Pipelined resets")
        const int r = alloc_spare(c);
        if (r) return r;
    }
    return 0;
}

// Fold the recorded per-kernel event intervals of all pending batches into the
// per-name accumulators (synchronizes the stream).
static int drain_timings(fsx_ctx *c) {
    if (c->ring_n == 0) return 0;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int r = 0; r < c->ring_n; ++r) {
        for (int i = 0; i < c->ev_used[r]; ++i) {
            const int p = c->ev_prev[r][i];
            if (p < 0 || !c->ev_names[r][i]) continue;   // start markers
            float t = 0;
            HIPCHK(c, hipEventElapsedTime(&t, c->ev[r][p], c->ev[r][i]));
            const char *nm = c->ev_names[r][i];
            int k = 0;
            while (k < c->acc_n && strcmp(c->acc_name[k], nm) != 0) ++k;
            if (k == c->acc_n) {
                if (c->acc_n == kMaxNames) continue;
                c->acc_name[c->acc_n++] = nm;
            }
            c->acc_ms[k] += t;
            c->acc_cnt[k] += 1;
        }
        c->acc_batches += 1;
    }
    c->ring_n = 0;
    return 0;
}

// A/B switch: FSX_SERIAL_FLOWS=1 keeps the flow features on the batch stream.
static bool fork_flows() {
    static const bool serial = getenv("FSX_SERIAL_FLOWS") != nullptr;
    return !serial;
}

// ------------------------------------------------------------------ prefix rules
// The device tables of the prefix blocklists (RuleSet, fsx_internal.h): the probe table
// (four times as many slots as rules, linear probing by rule_hash), the distinct lengths
// per family longest first, and the per-family /24 filter bits. Rebuilt whole from the
// host map (rules change rarely; 64K rules: 8 MiB of slots + 4 MiB of filter). Called
// with the stream idle.
static int upload_rules(fsx_ctx *c) {
    c->rules_dirty = false;
    if (c->rules.empty()) { c->rs = RuleSet{}; return 0; }
    const uint64_t cap = next_pow2(std::max<uint64_t>(64, 4 * c->rules.size()));
    constexpr size_t kFw = size_t(1) << (kRuleFilterBits - 5);   // filter words per family
    std::vector<uint32_t> filt(2 * kFw, 0u);
    std::vector<RuleSlot> tab(cap);
    memset(tab.data(), 0, cap * sizeof(RuleSlot));
    for (const auto &r : c->rules) {
        const uint32_t a[4] = {r.first[1], r.first[2], r.first[3], r.first[4]};
        uint64_t h = rule_hash(r.first[0], a) & (cap - 1);
        while (tab[h].tag) h = (h + 1) & (cap - 1);
        tab[h].tag = r.first[0];
        tab[h].fp = rule_fp(a);
        tab[h].till = r.second;
        memcpy(tab[h].a, a, 16);
        // the /24s the rule touches: [p, p + 2^(24 - len)) of the first 24 address bits
        const uint32_t L = r.first[0] & 0xFFu, f = (r.first[0] >> 8) - 1u;
        const uint32_t p = (a[0] & 0xFFu) << 16 | (a[0] & 0xFF00u) | ((a[0] >> 16) & 0xFFu);
        const uint32_t span = L >= kRuleFilterBits ? 1u : 1u << (kRuleFilterBits - L);
        uint32_t *fw = filt.data() + f * kFw;
        for (uint32_t q = p; q < p + span;) {
            if ((q & 31u) == 0 && q + 32 <= p + span) { fw[q >> 5] = ~0u; q += 32; continue; }
            fw[q >> 5] |= 1u << (q & 31u);
            ++q;
        }
    }
    uint8_t lens[256] = {};
    uint32_t nl[2] = {0, 0};
    for (int f = 0; f < 2; ++f)
        for (int L = f ? 128 : 32; L >= 0; --L)
            if (c->rule_len_cnt[f][L]) lens[(f ? kRuleLens6 : 0) + nl[f]++] = (uint8_t)L;
    if (cap > c->rule_cap) {
        hipFree(c->d_rule_slot);
        c->d_rule_slot = nullptr;
        c->rule_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rule_slot, cap * sizeof(RuleSlot)));
        c->rule_cap = cap;
    }
    if (!c->d_rule_lens) HIPCHK(c, hipMalloc(&c->d_rule_lens, sizeof(lens)));
    if (!c->d_rule_filter) HIPCHK(c, hipMalloc(&c->d_rule_filter, filt.size() * 4));
    HIPCHK(c, hipMemcpy(c->d_rule_filter, filt.data(), filt.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_rule_slot, tab.data(), cap * sizeof(RuleSlot), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_rule_lens, lens, sizeof(lens), hipMemcpyHostToDevice));
    c->rs = RuleSet{c->d_rule_slot, c->d_rule_lens, c->d_rule_filter, (uint32_t)(cap - 1), nl[0], nl[1]};
    return 0;
}

static bool prefix_map(int map_id) { return map_id == FSX_MAP_IPV4_PREFIX || map_id == FSX_MAP_IPV6_PREFIX; }
static size_t prefix_klen(int map_id) { return map_id == FSX_MAP_IPV6_PREFIX ? 20 : 8; }

// Canonical rule key of a bpf_lpm_trie_key-style map key; -EINVAL on a too-long prefix.
static int prefix_rule_key(int map_id, const void *key, std::array<uint32_t, 5> &rk) {
    const bool v6 = map_id == FSX_MAP_IPV6_PREFIX;
    uint32_t plen, k[4] = {0, 0, 0, 0};
    memcpy(&plen, key, 4);
    if (plen > (v6 ? 128u : 32u)) return -EINVAL;
    memcpy(k, static_cast<const uint8_t *>(key) + 4, v6 ? 16 : 4);
    uint32_t a[4];
    rule_mask(k, plen, a);
    rk = {(v6 ? 2u : 1u) << 8 | plen, a[0], a[1], a[2], a[3]};
    return 0;
}

static void rule_count(fsx_ctx *c, const std::array<uint32_t, 5> &rk, int d) {
    const int f = (int)(rk[0] >> 8) - 1;
    c->rule_cnt[f] += (uint32_t)d;
    c->rule_len_cnt[f][rk[0] & 0xFFu] += (uint32_t)d;
}

// op 0 lookup (longest match of the key's first prefixlen bits), 1 update, 2 delete
static int prefix_op(fsx_ctx *c, int op, int map_id, const void *key, const void *value, void *out,
                     uint64_t flags) {
    std::array<uint32_t, 5> rk;
    int rc = prefix_rule_key(map_id, key, rk);
    if (rc) return rc;
    const int f = map_id == FSX_MAP_IPV6_PREFIX ? 1 : 0;
    if (op == 0) {
        uint32_t k[4] = {rk[1], rk[2], rk[3], rk[4]};
        for (int L = (int)(rk[0] & 0xFFu); L >= 0; --L) {
            if (!c->rule_len_cnt[f][L]) continue;
            uint32_t a[4];
            rule_mask(k, (uint32_t)L, a);
            auto it = c->rules.find({(uint32_t)(f + 1) << 8 | (uint32_t)L, a[0], a[1], a[2], a[3]});
            if (it != c->rules.end()) { memcpy(out, &it->second, 8); return 0; }
        }
        return -ENOENT;
    }
    auto it = c->rules.find(rk);
    if (op == 2) {
        if (it == c->rules.end()) return -ENOENT;
        c->rules.erase(it);
        rule_count(c, rk, -1);
        c->rules_dirty = true;
        return 0;
    }
    if (flags > FSX_BPF_EXIST) return -EINVAL;
    if (flags == FSX_BPF_NOEXIST && it != c->rules.end()) return -EEXIST;
    if (flags == FSX_BPF_EXIST && it == c->rules.end()) return -ENOENT;
    uint64_t till;
    memcpy(&till, value, 8);
    if (it != c->rules.end()) {
        it->second = till;
    } else {
        if (c->rule_cnt[f] >= FSX_PREFIX_MAX_ENTRIES) return -ENOSPC;
        c->rules.emplace(rk, till);
        rule_count(c, rk, +1);
    }
    c->rules_dirty = true;
    return 0;
}

static FlowRequest flow_slots(fsx_ctx *c, const FlowRequest *fr, size_t n, int *rc);

// A pipelined batch (fsx_set_pipeline): its front (parse, sort) on the context stream, its
// tail on the walker stream (flows on the aux stream), so the next batch's front overlaps
// this tail. The batch three back used this batch's front buffers: the host waits for its
// tail (the device still has the previous batch to run) and checks it.
// split = false (other limiters, record mode): the whole batch on the context stream, in
// order after the previous one, still without a host synchronization per call.
static int run_pipelined(fsx_ctx *c, const PacketIn &in0, const uint32_t *d_len, const uint64_t *d_ts, size_t n,
                         uint8_t *d_verdict, const FlowRequest *fr, bool split) {
    HIPCHK(c, hipSetDevice(c->device));
    int rc;
    // record mode (run_records): the set's len / ts buffers (fresh allocations: in use by nobody)
    PacketIn in = in0;
    if (in.rec && !in.rec_len && !c->rec_len_set[0]) {
        for (int p = 0; p < fsx_ctx::kSets; ++p) {
            HIPCHK(c, hipMalloc(&c->rec_len_set[p], (size_t)c->cfg.max_batch * 4));
            HIPCHK(c, hipMalloc(&c->rec_ts_set[p], (size_t)c->cfg.max_batch * 8));
        }
    }
    if (c->pending && (rc = fsx_sync(c))) return rc;
    if (c->rules_dirty) {   // the prefix tables are rebuilt with the device idle
        if ((rc = fsx_sync(c)) || (rc = upload_rules(c))) return rc;
    }
    // an unsplit batch's tail runs on the context stream: a deferred tail goes first
    if (!split && (rc = sel(c))) return rc;
    //  the batch generation wraps in this call: k_born_clear rewrites the flags word
    // of every stamped slot, which a tail still in flight may be storing — the deferred tail goes
    // in first and the context stream waits for the last tail (tails run in order)
    if (split && c->id_gen + 1 == 0x10000u && (rc = sel(c))) return rc;
    const int q = (c->par + 1) % fsx_ctx::kSets;   // the set of the batch three calls back
    if (c->fl_on[q]) {
        HIPCHK(c, hipEventSynchronize(c->tail_done[q]));
        BatchState h;
        HIPCHK(c, hipMemcpy(&h, c->fb[q].bs, sizeof(h), hipMemcpyDeviceToHost));
        note_batch(c, h);
        if (h.err) return fsx_sync(c);   // rolls it back, and the batch after it
        c->fl_on[q] = false;
    }
    FlowRequest frq;
    if (fr) {
        frq = flow_slots(c, fr, n, &rc);
        if (rc) return rc;
        fr = &frq;
    }
    // the batch before this one (still in flight: its failure cancels this one — not across
    // a pipelined reset: this batch runs on other tables)
    const BatchState *prev = c->fl_on[c->par] && !c->fresh_tables ? c->fb[c->par].bs : nullptr;
    c->fresh_tables = false;
    const int old_par = c->par;
    use_front(c, q);
    c->par = q;
    if (in.rec && !in.rec_len) {   // (set q's batch three back has finished: above)
        in.rec_len = c->rec_len_set[q];
        in.rec_ts = c->rec_ts_set[q];
        d_len = in.rec_len;
        d_ts = in.rec_ts;
    }
    if (++c->id_gen == 0x10000u) {
        if (c->sc.id_tab) HIPCHK(c, hipMemsetAsync(c->sc.id_tab, 0, c->id_slots * 32, c->stream));
        HIPCHK(c, launch_born_clear(c->table, c->slots, c->stream));   // (stamps left by k_ord_claim)
        c->id_gen = 1;
    }
    // the early prologue on the aux stream (FSX_NO_EARLY_PROLOGUE=1: on the context stream)
    static const bool no_early = getenv("FSX_NO_EARLY_PROLOGUE") != nullptr;
    if (split && c->pro_fence) {   // (other work on the context stream since the last front)
        HIPCHK(c, hipEventRecord(c->pro_wait, c->stream));
        c->pro_fence = false;
    }
    // (the early prologue on the walker stream: the aux stream carries the previous tail's
    // flows, which the next parse should not wait for)
    // (FSX_TAIL_END_AUX=1: tails end on the aux stream and the early prologue runs on the walker
    // stream; measured 2.99 vs 2.96 ms per step, profiles/r04/ab_r04n.txt)
    static const bool end_aux = getenv("FSX_TAIL_END_AUX") != nullptr;
    const PipeSplit sp = split ? PipeSplit{c->walk_stream, c->front_done, prev, pipe_on_parse, c, &c->tail_args,
                                           no_early ? nullptr : end_aux ? c->walk_stream : c->aux_stream,
                                           c->pro_wait, c->pro_done}
                               : PipeSplit{nullptr, nullptr, prev, nullptr, nullptr, nullptr};
    hipError_t e = launch_verdict_pipeline(in, d_len, d_ts, (uint32_t)n, d_verdict, c->table, c->tstate, c->bs,
                                           c->sc, c->id_gen, table_index(c), c->lim, c->rs, true, fr, c->hist,
                                           c->stream, fork_flows() ? c->aux_stream : nullptr, c->fork_ev,
                                           c->join_ev, split ? nullptr : c->walk_stream, c->walk_fork_ev,
                                           c->walk_join_ev, c->heavy_fork_ev, c->heavy_flow_ev, nullptr, &sp);
    if (e != hipSuccess) {
        // nothing of this batch is in flight: back to the previous set, so the pending tail and
        // the next sel() still refer to the batch that owns them
        use_front(c, old_par);
        c->par = old_par;
        return set_err(c, -EIO, "pipeline launch: %s", hipGetErrorString(e));
    }
    c->fl_on[q] = true;
    c->fl_born[q] = c->id_gen;
    c->fl_tgen[q] = c->tgen;
    if (split) {
        c->tail_pending = true;   // enqueued after the next batch's parse, or by the next sel()
        c->tail_par = q;
        c->tail_join = true;
    } else {
        HIPCHK(c, hipEventRecord(c->tail_done[q], c->stream));
    }
    return 0;
}

// FSX_FLAG_EVICT_IDLE, before a limiter batch of n packets: when the
// tracked sources plus n exceed max_entries, every source idle at the batch's smallest
// timestamp leaves the maps. Synchronous: the previous batches finish first, and the
// survivors move to new slots (open addressing drops no entry in place).
static int evict_idle(fsx_ctx *c, const PacketIn &in, const uint64_t *d_ts, size_t n) {
    c->last_evicted = 0;
    // no synchronization while the bound says the batch fits: a batch adds at
    // most n sources
    if (c->count_bound <= c->cfg.max_entries && n <= c->cfg.max_entries - c->count_bound) {
        c->count_bound += n;
        return 0;
    }
    int rc;
    if ((rc = sel(c)) || (rc = fsx_sync(c))) return rc;
    uint64_t count = 0;
    HIPCHK(c, hipMemcpy(&count, &c->tstate->count, 8, hipMemcpyDeviceToHost));
    c->count_bound = count + n;
    if (count + n <= c->cfg.max_entries) return 0;
    if (c->flow_accum || c->d_slot_acc)
        return set_err(c, -EINVAL, "FSX_FLAG_EVICT_IDLE moves sources between slots: not with fsx_flows_begin");
    if (count > c->evict_cap) {
        hipFree(c->evict_buf);
        c->evict_buf = nullptr;
        c->evict_cap = 0;
        HIPCHK(c, hipMalloc(&c->evict_buf, count * sizeof(Slot)));
        c->evict_cap = count;
    }
    unsigned long long *scal = reinterpret_cast<unsigned long long *>(c->d_val);
    HIPCHK(c, hipMemsetAsync(scal, 0xFF, 8, c->stream));
    HIPCHK(c, hipMemsetAsync(scal + 1, 0, 8, c->stream));
    hipError_t e = launch_evict_scan(c->table, c->lim, in, d_ts, (uint32_t)n, c->evict_buf, c->evict_cap, scal,
                                     c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "evict scan: %s", hipGetErrorString(e));
    uint64_t m = 0;
    HIPCHK(c, hipMemcpyAsync(&m, scal + 1, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (m > count) return set_err(c, -EIO, "evict scan found %llu live sources of %llu",
                                  (unsigned long long)m, (unsigned long long)count);
    if (m == count) return 0;   // nothing idle: the batch decides (-ENOSPC if it overflows)
    if ((rc = next_epoch(c))) return rc;
    HIPCHK(c, launch_clear(c->table, c->slots * sizeof(Slot), c->stream));
    e = launch_evict_reinsert(c->table, c->tstate, c->lim, table_index(c), c->evict_buf, m, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "evict reinsert: %s", hipGetErrorString(e));
    c->last_evicted = count - m;
    c->count_bound = m + n;
    return 0;
}

// Split pipelining for every limiter (FSX_SPLIT_FIXED_ONLY=1: the fixed window only). The
// token bucket's tail was two tile scans over every position and measured slower split (4.73
// vs 4.39 ms, profiles/r04/ab_r04t_token.txt); with the one-pass scan (k_tb_scan) split wins,
// 4.06 vs 4.22 ms (profiles/r05/ab_r05tb5_token_split.txt; FSX_NO_SPLIT_TOKEN=1: whole batches, A/B).
static bool no_split_limiters(const fsx_ctx *c) {
    static const bool fixed_only = getenv("FSX_SPLIT_FIXED_ONLY") != nullptr;
    static const bool no_split_token = getenv("FSX_NO_SPLIT_TOKEN") != nullptr;
    if (c->cfg.limiter == FSX_LIMIT_TOKEN_BUCKET && no_split_token) return true;
    return fixed_only && c->cfg.limiter != FSX_LIMIT_FIXED_WINDOW;
}

// Enqueue one batch: verdicts + maps when d_verdict is set, per-source flows when fr is.
static int run_batch(fsx_ctx *c, const PacketIn &in, const uint32_t *d_len, const uint64_t *d_ts,
                     size_t n, uint8_t *d_verdict, bool do_limit, const FlowRequest *fr) {
    if (n > c->cfg.max_batch) return set_err(c, -E2BIG, "n=%zu exceeds max_batch", n);
    if (do_limit && n && (c->cfg.flags & FSX_FLAG_EVICT_IDLE)) {
        const int rc = evict_idle(c, in, d_ts, n);
        if (rc) return rc;
    }
    // home-ordered inserts for this batch: a flood of new sources (the last
    // checked batch's n_new > half its IP packets) or FSX_FLAG_ORDERED_INSERTS; FSX_ORDERED=0 /
    // 1: never / always (A/B). The fixed window on header records without flows, whole batches.
    static const int ord_env = getenv("FSX_ORDERED") ? atoi(getenv("FSX_ORDERED")) : -1;
    const bool ord_want = ord_env >= 0 ? ord_env > 0 : (c->flood_hint || (c->cfg.flags & FSX_FLAG_ORDERED_INSERTS));
    c->lim.ord = do_limit && !fr && !in.rec && d_verdict && c->cfg.limiter == FSX_LIMIT_FIXED_WINDOW &&
                 !(c->cfg.flags & FSX_FLAG_OVERFLOW_ADMIT) && ord_want ? 1u : 0u;
    c->lim.light_dom = c->light_dom ? 1u : 0u;
    // pipelined (no per-kernel timing): split front / tail for the fixed window on header
    // records, the whole batch on the context stream otherwise
    if (c->pipe && do_limit && n && !c->timing)
        return run_pipelined(c, in, d_len, d_ts, n, d_verdict, fr,
                             c->pipe == 1 && !no_split_limiters(c) &&
                                 !(c->cfg.flags & FSX_FLAG_OVERFLOW_ADMIT) && !c->lim.ord);
    int rc = sel(c);
    if (rc) return rc;
    if (busy(c)) { rc = fsx_sync(c); if (rc) return rc; }
    if (in.rec && !in.rec_len) return set_err(c, -EINVAL, "record batch without its len / ts buffers");
    if (do_limit && c->rules_dirty && (rc = upload_rules(c))) return rc;
    FlowRequest frq;
    if (fr) {
        frq = flow_slots(c, fr, n, &rc);
        if (rc) return rc;
        fr = &frq;
    }
    PipeTiming tmv{};
    PipeTiming *tm = nullptr;
    if (c->timing) {
        if (c->ring_n == kRing && (rc = drain_timings(c))) return rc;
        tmv = PipeTiming{c->ev[c->ring_n], c->ev_names[c->ring_n], c->ev_prev[c->ring_n], kMaxEv, 0};
        tm = &tmv;
    }
    if (!do_limit && !c->sc.id_tab) {   // flow-only batch: its per-batch id table
        HIPCHK(c, hipMalloc(&c->sc.id_tab, c->id_slots * 32));
        HIPCHK(c, hipMemsetAsync(c->sc.id_tab, 0, c->id_slots * 32, c->stream));   // every slot empty
    }
    if (++c->id_gen == 0x10000u) {   // 16-bit generations: clear the id table on wrap
        if (c->sc.id_tab) HIPCHK(c, hipMemsetAsync(c->sc.id_tab, 0, c->id_slots * 32, c->stream));
        HIPCHK(c, launch_born_clear(c->table, c->slots, c->stream));   // (stamps left by k_ord_claim)
        c->id_gen = 1;
    }
    hipError_t e = launch_verdict_pipeline(in, d_len, d_ts, (uint32_t)n, d_verdict, c->table,
                                           c->tstate, c->bs, c->sc, c->id_gen, table_index(c), c->lim,
                                           c->rs, do_limit, fr,
                                           c->hist, c->stream, fork_flows() ? c->aux_stream : nullptr,
                                           c->fork_ev, c->join_ev, fork_flows() ? c->walk_stream : nullptr,
                                           c->walk_fork_ev, c->walk_join_ev, c->heavy_fork_ev,
                                           c->heavy_flow_ev, tm);
    if (tm) c->ev_used[c->ring_n++] = tm->used;
    c->pending = true;
    c->pending_born = do_limit && n ? c->id_gen : 0;
    if (e != hipSuccess) return set_err(c, -EIO, "pipeline launch: %s", hipGetErrorString(e));
    return 0;
}

// The per-source flow accumulators of a batch (context scratch, grown on demand; only the
// flow stream uses them, in batch order).
static FlowRequest flow_slots(fsx_ctx *c, const FlowRequest *fr, size_t n, int *rc) {
    FlowRequest frq = *fr;
    *rc = 0;
    // accumulate mode (fsx_flows_begin .. fsx_flows_end): every source of the call must merge
    // into its SlotAcc, so the scratch covers all n packets' sources; the row cap applies in
    // fsx_flows_end only
    const uint64_t need = frq.sacc ? std::max<uint64_t>(1, n)
                                   : std::max<uint64_t>(1, std::min<uint64_t>(frq.cap, n));
    if (need > c->flow_acc_cap) {
        if (busy(c) && (*rc = fsx_sync(c))) return frq;   // the old accumulators may be in use
        hipFree(c->d_flow_acc);
        c->d_flow_acc = nullptr;
        c->flow_acc_cap = 0;
        if (hipMalloc(&c->d_flow_acc, need * flow_acc_bytes()) != hipSuccess) {
            *rc = set_err(c, -ENOMEM, "flow accumulators");
            return frq;
        }
        c->flow_acc_cap = need;
    }
    frq.acc = c->d_flow_acc;
    frq.cap = frq.sacc ? (uint32_t)need : (uint32_t)std::min<uint64_t>(frq.cap, c->flow_acc_cap);
    return frq;
}

static FlowRequest flow_request(fsx_ctx *c, uint8_t *keys16, uint8_t *fam, float *feat, float *prob,
                                uint8_t *dec, size_t cap) {
    FlowRequest fr{};
    fr.keys16 = keys16; fr.fam = fam; fr.feat = feat; fr.cap = (uint32_t)std::min<size_t>(cap, 0xFFFFFFFFu);
    if (c->flow_accum) {   // rows come from fsx_flows_end
        fr.sacc = c->d_slot_acc;
        fr.epoch = c->flow_epoch;
    }
    if (c->model_loaded && prob && dec) {
        fr.prob = prob; fr.dec = dec;
        fr.score = make_score_params(c->w, c->inv_in, c->zp_in, c->bias_over_ats, c->mult, c->zp_out, c->lut);
    } else {
        fr.score.enabled = 0;
    }
    return fr;
}

int fsx_verdict_batch_device(fsx_ctx *c, const uint8_t *d_hdr, const uint32_t *d_len,
                             const uint64_t *d_ts, size_t n, uint8_t *d_verdict) {
    if (!c) return -EINVAL;
    if (n && (!d_hdr || !d_len || !d_ts || !d_verdict)) return set_err(c, -EINVAL, "null buffer");
    return run_batch(c, PacketIn{d_hdr, nullptr, 0, nullptr, nullptr}, d_len, d_ts, n, d_verdict, true, nullptr);
}

int fsx_process_batch_device(fsx_ctx *c, const uint8_t *d_hdr, const uint32_t *d_len,
                             const uint64_t *d_ts, size_t n, uint8_t *d_verdict, uint8_t *d_keys16,
                             uint8_t *d_family, float *d_features, float *d_prob,
                             uint8_t *d_malicious, size_t flow_cap) {
    if (!c) return -EINVAL;
    if (n && (!d_hdr || !d_len || !d_ts || !d_verdict || (!c->flow_accum && (!d_keys16 || !d_family))))
        return set_err(c, -EINVAL, "null buffer");
    const FlowRequest fr = flow_request(c, d_keys16, d_family, d_features, d_prob, d_malicious, flow_cap);
    return run_batch(c, PacketIn{d_hdr, nullptr, 0, nullptr, nullptr}, d_len, d_ts, n, d_verdict, true, &fr);
}

static int ensure_stage(fsx_ctx *c, uint64_t n);

// Record mode (the owner side of the sharded path): the pipeline reads the exchange
// records directly; their len / ts land in context scratch for the later kernels.
static int run_records(fsx_ctx *c, const void *d_records, size_t n, uint32_t rec_bytes, uint8_t *d_verdict,
                       const FlowRequest *fr, bool do_limit = true) {
    if (rec_bytes != FSX_SHARD_RECORD_BYTES && rec_bytes != FSX_SHARD_RECORD16_BYTES)
        return set_err(c, -EINVAL, "record size must be %d or %d", FSX_SHARD_RECORD16_BYTES,
                       FSX_SHARD_RECORD_BYTES);
    if (n > c->cfg.max_batch) return set_err(c, -E2BIG, "n=%zu exceeds max_batch", n);
    if (n && (!d_records || !d_verdict)) return set_err(c, -EINVAL, "null buffer");
    // pipelined (run_batch takes run_pipelined): the front set's own len / ts buffers, so a
    // split tail reading this batch's overlaps the next front writing its own
    if (c->pipe && do_limit && n && !c->timing)
        return run_batch(c, PacketIn{nullptr, d_records, rec_bytes, nullptr, nullptr}, nullptr, nullptr, n,
                         d_verdict, do_limit, fr);
    int rc = sel(c);
    if (rc) return rc;
    if (n > c->rec_cap) {
        if (busy(c) && (rc = fsx_sync(c))) return rc;   // the old buffers may be in use
        hipFree(c->d_rec_len); hipFree(c->d_rec_ts);
        c->d_rec_len = nullptr; c->d_rec_ts = nullptr; c->rec_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rec_len, n * 4));
        HIPCHK(c, hipMalloc(&c->d_rec_ts, n * 8));
        c->rec_cap = n;
    }
    const PacketIn in{nullptr, d_records, rec_bytes, c->d_rec_len, c->d_rec_ts};
    return run_batch(c, in, c->d_rec_len, c->d_rec_ts, n, d_verdict, do_limit, fr);
}

int fsx_flow_partials_records_device(fsx_ctx *c, const void *d_records, size_t n, uint32_t rec_bytes, uint32_t G,
                                     void *d_partials, size_t cap_per_shard, uint64_t *d_counts) {
    if (!c) return -EINVAL;
    if (G == 0 || G > FSX_MAX_SHARDS) return set_err(c, -EINVAL, "n_shards must be 1..%d", FSX_MAX_SHARDS);
    if (!d_counts || (n && cap_per_shard && !d_partials)) return set_err(c, -EINVAL, "null buffer");
    if (cap_per_shard > 0xFFFFFFFFu) return set_err(c, -EINVAL, "cap_per_shard too large");
    int rc = sel(c);
    if (rc) return rc;
    HIPCHK(c, hipMemsetAsync(d_counts, 0, (size_t)G * 8, c->stream));
    if (n == 0) return 0;
    if ((rc = ensure_stage(c, n))) return rc;   // (verdict scratch: no limiter runs)
    FlowRequest fr{};
    fr.cap = (uint32_t)std::min<size_t>(n, 0xFFFFFFFFu);
    fr.score.enabled = 0;
    fr.part = PartialOut{d_partials, (uint32_t)cap_per_shard, G, reinterpret_cast<unsigned long long *>(d_counts)};
    return run_records(c, d_records, n, rec_bytes, c->d_verdict, &fr, false);
}

int fsx_flows_merge_counted_device(fsx_ctx *c, const void *d_partials, size_t cap, const uint64_t *d_count) {
    if (!c || !d_count) return -EINVAL;
    if (!c->flow_accum) return set_err(c, -EINVAL, "fsx_flows_merge_counted_device outside fsx_flows_begin .. end");
    if (cap && !d_partials) return set_err(c, -EINVAL, "null buffer");
    if (cap > 0xFFFFFFFFu) return set_err(c, -E2BIG, "cap=%zu too large", cap);
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_flows_merge(d_partials, (uint32_t)cap, c->table, c->lim, c->d_slot_acc, c->flow_epoch,
                                      c->stream, d_count);
    if (e != hipSuccess) return set_err(c, -EIO, "flows merge: %s", hipGetErrorString(e));
    return 0;
}

int fsx_flows_merge_device(fsx_ctx *c, const void *d_partials, size_t m) {
    if (!c) return -EINVAL;
    if (!c->flow_accum) return set_err(c, -EINVAL, "fsx_flows_merge_device outside fsx_flows_begin .. end");
    if (m && !d_partials) return set_err(c, -EINVAL, "null buffer");
    if (m > 0xFFFFFFFFu) return set_err(c, -E2BIG, "m=%zu too large", m);
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_flows_merge(d_partials, (uint32_t)m, c->table, c->lim, c->d_slot_acc, c->flow_epoch,
                                      c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "flows merge: %s", hipGetErrorString(e));
    return 0;
}

int fsx_verdict_records_device(fsx_ctx *c, const void *d_records, size_t n, uint32_t rec_bytes,
                               uint8_t *d_verdict) {
    if (!c) return -EINVAL;
    return run_records(c, d_records, n, rec_bytes, d_verdict, nullptr);
}

int fsx_process_records_device(fsx_ctx *c, const void *d_records, size_t n, uint32_t rec_bytes,
                               uint8_t *d_verdict, uint8_t *d_keys16, uint8_t *d_family, float *d_features,
                               float *d_prob, uint8_t *d_malicious, size_t flow_cap) {
    if (!c) return -EINVAL;
    if (n && !c->flow_accum && (!d_keys16 || !d_family)) return set_err(c, -EINVAL, "null buffer");
    const FlowRequest fr = flow_request(c, d_keys16, d_family, d_features, d_prob, d_malicious, flow_cap);
    return run_records(c, d_records, n, rec_bytes, d_verdict, &fr);
}

static int ensure_stage(fsx_ctx *c, uint64_t n) {
    if (n <= c->stage_cap) return 0;
    hipFree(c->d_hdr); hipFree(c->d_len); hipFree(c->d_ts); hipFree(c->d_verdict);
    c->d_hdr = nullptr; c->d_len = nullptr; c->d_ts = nullptr; c->d_verdict = nullptr;
    c->stage_cap = 0;
    HIPCHK(c, hipMalloc(&c->d_hdr, n * 64));
    HIPCHK(c, hipMalloc(&c->d_len, n * 4));
    HIPCHK(c, hipMalloc(&c->d_ts, n * 8));
    HIPCHK(c, hipMalloc(&c->d_verdict, n));
    c->stage_cap = n;
    return 0;
}

int fsx_verdict_batch(fsx_ctx *c, const uint8_t *hdr, const uint32_t *len, const uint64_t *ts,
                      size_t n, uint8_t *verdict) {
    if (!c) return -EINVAL;
    if (n && (!hdr || !len || !ts || !verdict)) return set_err(c, -EINVAL, "null buffer");
    if (n > c->cfg.max_batch) return set_err(c, -E2BIG, "n=%zu exceeds max_batch", n);
    int rc = sel(c);
    if (rc) return rc;
    if (n == 0) return 0;
    if ((rc = ensure_stage(c, n))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_hdr, hdr, n * 64, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_len, len, n * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_ts, ts, n * 8, hipMemcpyHostToDevice, c->stream));
    rc = fsx_verdict_batch_device(c, c->d_hdr, c->d_len, c->d_ts, n, c->d_verdict);
    if (rc) return rc;
    if ((rc = sel(c))) return rc;   // (a pipelined batch's tail writes the verdicts)
    HIPCHK(c, hipMemcpyAsync(verdict, c->d_verdict, n, hipMemcpyDeviceToHost, c->stream));
    return fsx_sync(c);
}

// ------------------------------------------------------------------ maps
static bool map_v6(int map_id) {
    return map_id == FSX_MAP_IPV6_STATS || map_id == FSX_MAP_IPV6_BLACKLIST || map_id == FSX_MAP_IPV6_TOKENS;
}
// value bytes of a per-IP map: ip_stats 24, token bucket 16, blacklist 8
static size_t map_vlen(int map_id) {
    if (map_id == FSX_MAP_IPV4_STATS || map_id == FSX_MAP_IPV6_STATS) return 24;
    if (map_id == FSX_MAP_IPV4_TOKENS || map_id == FSX_MAP_IPV6_TOKENS) return 16;
    return 8;
}

static int key_words(int map_id, const void *key, uint32_t k[4]) {
    k[0] = k[1] = k[2] = k[3] = 0;
    if (map_id < FSX_MAP_IPV4_STATS || map_id > FSX_MAP_IPV6_TOKENS) return -EINVAL;
    memcpy(k, key, map_v6(map_id) ? 16 : 4);
    return 0;
}

static int map_op(fsx_ctx *c, int op, int map_id, const void *key, const void *value, void *out,
                  uint64_t flags) {
    if (!c || !key) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    if ((rc = fsx_sync(c))) return rc;
    if (map_id == FSX_MAP_STATS) {
        uint32_t k0;
        memcpy(&k0, key, 4);
        if (k0 != 0) return op == 0 ? -ENOENT : -E2BIG;  // ARRAY[1]: index 0 only
        if (op == 2) return -EINVAL;                     // array elements cannot be deleted
        if (op == 0) { HIPCHK(c, hipMemcpy(out, c->tstate->stats, 16, hipMemcpyDeviceToHost)); return 0; }
        if (flags == FSX_BPF_NOEXIST) return -EEXIST;
        HIPCHK(c, hipMemcpy(c->tstate->stats, value, 16, hipMemcpyHostToDevice));
        return 0;
    }
    if (prefix_map(map_id)) return prefix_op(c, op, map_id, key, value, out, flags);
    if (op == 1) c->count_bound = ~0ull;
    uint32_t k[4];
    if ((rc = key_words(map_id, key, k))) return set_err(c, rc, "bad map id %d", map_id);
    if (flags > FSX_BPF_EXIST) return -EINVAL;
    uint64_t v[3] = {0, 0, 0};
    const size_t vlen = map_vlen(map_id);
    if (op == 1) memcpy(v, value, vlen);
    hipError_t e = launch_map_op(c->table, c->tstate, c->lim, table_index(c), op, map_id, k, v, flags, c->d_res,
                                 c->d_val, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "map op: %s", hipGetErrorString(e));
    int32_t res = 0;
    HIPCHK(c, hipMemcpyAsync(&res, c->d_res, 4, hipMemcpyDeviceToHost, c->stream));
    uint64_t ov[3];
    HIPCHK(c, hipMemcpyAsync(ov, c->d_val, 24, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (res == 0 && op == 0) memcpy(out, ov, vlen);
    return res;
}

int fsx_map_lookup(fsx_ctx *c, int map_id, const void *key, void *value) {
    if (!value) return -EINVAL;
    return map_op(c, 0, map_id, key, nullptr, value, 0);
}
int fsx_map_update(fsx_ctx *c, int map_id, const void *key, const void *value, uint64_t flags) {
    if (!value) return -EINVAL;
    return map_op(c, 1, map_id, key, value, nullptr, flags);
}
int fsx_map_delete(fsx_ctx *c, int map_id, const void *key) {
    return map_op(c, 2, map_id, key, nullptr, nullptr, 0);
}

int fsx_map_update_batch(fsx_ctx *c, int map_id, const void *keys, const void *values, size_t n,
                         uint64_t flags) {
    if (!c || (n && (!keys || !values))) return -EINVAL;
    if (flags != FSX_BPF_ANY) return set_err(c, -EINVAL, "batched updates take BPF_ANY only");
    if (map_id <= FSX_MAP_STATS || map_id >= FSX_MAP_COUNT)
        return set_err(c, -EINVAL, "map id %d has no batched update", map_id);
    if (n > kMaxBatchLimit) return set_err(c, -E2BIG, "n=%zu too large", n);
    int rc = sel(c);
    if (rc) return rc;
    if ((rc = fsx_sync(c))) return rc;
    if (n == 0) return 0;
    if (prefix_map(map_id)) {   // host map: validated and sized first, all or nothing
        const size_t klen = prefix_klen(map_id);
        const int f = map_id == FSX_MAP_IPV6_PREFIX ? 1 : 0;
        std::vector<std::array<uint32_t, 5>> rks(n);
        std::map<std::array<uint32_t, 5>, int> fresh;
        for (size_t i = 0; i < n; ++i) {
            if ((rc = prefix_rule_key(map_id, static_cast<const uint8_t *>(keys) + i * klen, rks[i])))
                return set_err(c, rc, "prefix key %zu: prefixlen too long", i);
            if (!c->rules.count(rks[i])) fresh[rks[i]] = 1;
        }
        if (c->rule_cnt[f] + fresh.size() > FSX_PREFIX_MAX_ENTRIES)
            return set_err(c, -ENOSPC, "prefix map full");
        for (size_t i = 0; i < n; ++i) {
            uint64_t till;
            memcpy(&till, static_cast<const uint8_t *>(values) + i * 8, 8);
            auto ins = c->rules.insert_or_assign(rks[i], till);
            if (ins.second) rule_count(c, rks[i], +1);
        }
        c->rules_dirty = true;
        return 0;
    }
    const size_t klen = map_v6(map_id) ? 16 : 4, vlen = map_vlen(map_id);
    c->count_bound = ~0ull;
    uint32_t *dk = nullptr;
    uint64_t *dv = nullptr;
    HIPCHK(c, hipMalloc(&dk, n * klen));
    if (hipMalloc(&dv, n * vlen) != hipSuccess) { hipFree(dk); return set_err(c, -ENOMEM, "map import"); }
    hipError_t e = hipMemcpyAsync(dk, keys, n * klen, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dv, values, n * vlen, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && ++c->id_gen == 0x10000u) {   // 16-bit generations (as run_batch)
        if (c->sc.id_tab) e = hipMemsetAsync(c->sc.id_tab, 0, c->id_slots * 32, c->stream);
        if (e == hipSuccess) e = launch_born_clear(c->table, c->slots, c->stream);
        c->id_gen = 1;
    }
    const uint32_t born = c->id_gen;
    if (e == hipSuccess)
        e = launch_map_import(c->table, c->tstate, c->bs, c->lim, table_index(c), born, map_id, dk, dv,
                              (uint32_t)n, c->stream);
    if (e == hipSuccess) {
        c->pending = true;          // checked (and rolled back when the map is full) like a batch
        c->pending_born = born;
        rc = fsx_sync(c);
    }
    hipFree(dk);
    hipFree(dv);
    if (e != hipSuccess) return set_err(c, -EIO, "map import: %s", hipGetErrorString(e));
    return rc;
}

int fsx_map_dump(fsx_ctx *c, int map_id, void *keys, void *values, size_t cap, size_t *n_out) {
    if (!c || !n_out) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    if ((rc = fsx_sync(c))) return rc;
    if (map_id == FSX_MAP_STATS) {
        if (cap >= 1) {
            uint32_t z = 0;
            if (keys) memcpy(keys, &z, 4);
            if (values) HIPCHK(c, hipMemcpy(values, c->tstate->stats, 16, hipMemcpyDeviceToHost));
        }
        *n_out = 1;
        return 0;
    }
    if (prefix_map(map_id)) {
        const size_t klen = prefix_klen(map_id);
        const uint32_t fam = map_id == FSX_MAP_IPV6_PREFIX ? 2u : 1u;
        size_t m = 0;
        for (const auto &r : c->rules) {
            if ((r.first[0] >> 8) != fam) continue;
            if (m < cap) {
                if (keys) {
                    uint8_t *kp = static_cast<uint8_t *>(keys) + m * klen;
                    const uint32_t plen = r.first[0] & 0xFFu;
                    memcpy(kp, &plen, 4);
                    memcpy(kp + 4, &r.first[1], klen - 4);
                }
                if (values) memcpy(static_cast<uint8_t *>(values) + m * 8, &r.second, 8);
            }
            ++m;
        }
        *n_out = m;
        return 0;
    }
    if (map_id < FSX_MAP_IPV4_STATS || map_id >= FSX_MAP_COUNT) return -EINVAL;
    const size_t klen = map_v6(map_id) ? 16 : 4, vlen = map_vlen(map_id);
    const size_t dcap = std::max<size_t>(cap, 1);
    uint8_t *dk = nullptr;
    uint64_t *dv = nullptr;
    unsigned long long *dc = nullptr;
    HIPCHK(c, hipMalloc(&dk, dcap * klen));
    HIPCHK(c, hipMalloc(&dv, dcap * vlen));
    HIPCHK(c, hipMalloc(&dc, 8));
    HIPCHK(c, hipMemsetAsync(dc, 0, 8, c->stream));
    hipError_t e = launch_map_dump(c->table, c->lim, map_id, dk, dv, cap, dc, c->stream);
    unsigned long long cnt = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&cnt, dc, 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    const size_t m = std::min<size_t>(cap, cnt);
    if (e == hipSuccess && m && keys) e = hipMemcpy(keys, dk, m * klen, hipMemcpyDeviceToHost);
    if (e == hipSuccess && m && values) e = hipMemcpy(values, dv, m * vlen, hipMemcpyDeviceToHost);
    hipFree(dk); hipFree(dv); hipFree(dc);
    if (e != hipSuccess) return set_err(c, -EIO, "map dump: %s", hipGetErrorString(e));
    *n_out = cnt;
    return 0;
}

int fsx_get_stats(fsx_ctx *c, fsx_stats *out) {
    if (!c || !out) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    if ((rc = fsx_sync(c))) return rc;
    HIPCHK(c, hipMemcpy(out, c->tstate->stats, 16, hipMemcpyDeviceToHost));
    return 0;
}

// fsx_reset with pipelined batches in flight (DESIGN.md §3 "Pipelined resets"): the spare
// table set becomes current and is cleared on the context stream once the tails that last
// used it are done; the old set stays with the batches in flight (their tails captured it)
// and becomes the spare. No host synchronization, and the next front does not wait for the
// last tail. An in-flight batch's error still surfaces at the next synchronization; it
// changed nothing visible (its tables are gone), so nothing is rolled back, and the first
// batch after the reset does not cancel itself for it.
// Clear-free reset (DESIGN.md §3 "Clear-free reset"): a slot's tag word carries the table
// generation (Limits::tgen), and a line of another generation reads as empty — to the walkers
// (a fresh source's stale line holds no state), the map dumps, the index rebuild, the
// blocklist export and the history rebuild — so fsx_reset moves to the next generation
// instead of clearing the table (config 5: 32 GB of stores per reset). At the 16-bit wrap
// the table is cleared. FSX_RESET_CLEAR=1: clear at every reset (A/B). Returns the wrap.
static bool next_table_gen(fsx_ctx *c) {
    if (++c->lim.tgen < 0x10000u) return false;
    c->lim.tgen = 0;
    return true;
}
static bool reset_clears() {
    static const bool clear = getenv("FSX_RESET_CLEAR") != nullptr;
    return clear;
}

static bool reset_swap_ok(const fsx_ctx *c) {
    static const bool sync_reset = getenv("FSX_RESET_SYNC") != nullptr;
    return !sync_reset && c->pipe == 1 && c->spare.table && pipe_busy(c) && !c->pending && !c->flow_accum &&
           !c->timing && !(c->cfg.flags & FSX_FLAG_EVICT_IDLE);
}

// Test hook (FSX_TEST_SPARE_POISON): fill a freshly allocated spare table with what a recycled
// allocation could hold — live-looking IPv4 lines of the next table generation (state and a
// blacklist entry each) — so a test can check that nothing of it survives the swap-in.
static hipError_t poison_table(Slot *t, uint64_t slots, uint32_t tgen) {
    std::vector<Slot> h(slots);
    for (uint64_t i = 0; i < slots; ++i) {
        Slot &s = h[i];
        memset(&s, 0, sizeof(s));
        s.tag = slot_tag(1u, (tgen + 1u) & 0xFFFFu);
        s.flags = SLOT_HAS_ST | SLOT_HAS_BL;
        s.key[0] = 0x0A000000u | (uint32_t)i;
        s.pps = 7;
        s.bps = 700;
        s.tt = 1;
        s.till = ~0ull;
    }
    return hipMemcpy(t, h.data(), slots * sizeof(Slot), hipMemcpyHostToDevice);
}

// The spare table set, allocated with pipelining (fsx_set_pipeline 1) for the limiters and table
// sizes a pipelined reset serves: the table and index memory once more.
static int alloc_spare(fsx_ctx *c) {
    if (c->spare.table || c->cfg.limiter == FSX_LIMIT_SLIDING_WINDOW || c->tr_slots != 0 ||
        c->slots > (1ull << 25) || getenv("FSX_RESET_SYNC"))
        return 0;
    fsx_ctx::TableSet sp{};
    auto build = [&]() -> hipError_t {
        hipError_t e;
        if ((e = hipMalloc(&sp.table, c->slots * sizeof(Slot))) != hipSuccess) return e;
        // (hipMalloc may hand back recycled memory — e.g. an earlier context's table, whose
        // lines carry table generations this context reaches: the first swap-in must find
        // nothing but empty lines, as fsx_open's table does)
        if (getenv("FSX_TEST_SPARE_POISON")) {
            if ((e = poison_table(sp.table, c->slots, c->lim.tgen)) != hipSuccess) return e;
        }
        if ((e = hipMemset(sp.table, 0, c->slots * sizeof(Slot))) != hipSuccess) return e;
        if ((e = hipMalloc(&sp.tstate, sizeof(TableState))) != hipSuccess) return e;
        if ((e = hipMemset(sp.tstate, 0, sizeof(TableState))) != hipSuccess) return e;
        if ((e = hipMalloc(&sp.heads, c->slots * 8)) != hipSuccess) return e;
        if ((e = hipMemset(sp.heads, 0, c->slots * 8)) != hipSuccess) return e;
        if ((e = hipMalloc(&sp.k6, c->slots * 16)) != hipSuccess) return e;
        if (c->idx_mir && (e = hipMalloc(&sp.mir, mir_bytes(c->idx_shift))) != hipSuccess) return e;
        for (int k = 0; k < 3; ++k)
            if (!c->spare_free[k] && (e = hipEventCreateWithFlags(&c->spare_free[k], hipEventDisableTiming)) != hipSuccess)
                return e;
        if (!c->clr_done && (e = hipEventCreateWithFlags(&c->clr_done, hipEventDisableTiming)) != hipSuccess) return e;
        if (!c->clr_stream && (e = hipStreamCreateWithFlags(&c->clr_stream, hipStreamNonBlocking)) != hipSuccess)
            return e;
        // (nothing uses the new set yet: its "last users" are already done)
        for (int k = 0; k < 3; ++k)
            if ((e = hipEventRecord(c->spare_free[k], c->stream)) != hipSuccess) return e;
        // (the memsets above ran on the null stream: done before any context stream uses the set)
        return hipStreamSynchronize(nullptr);
    };
    const hipError_t e = build();
    if (e != hipSuccess) {   // (no spare: resets stay synchronous)
        hipFree(sp.table); hipFree(sp.tstate); hipFree(sp.heads); hipFree(sp.k6); hipFree(sp.mir);
        return set_err(c, -ENOMEM, "spare table set: %s", hipGetErrorString(e));
    }
    c->spare = sp;
    return 0;
}

static int reset_swap(fsx_ctx *c) {
    HIPCHK(c, hipSetDevice(c->device));
    fsx_ctx::TableSet &sp = c->spare;
    // (two resets with no batch between: the tail deferred before the first one uses the
    // spare — it goes in now, so the events below cover it)
    if (c->spare_tail && c->tail_pending) {
        const hipError_t e = flush_tail(c, c->front_done);
        if (e != hipSuccess) return set_err(c, -EIO, "pipelined tail: %s", hipGetErrorString(e));
    }
    // the spare is cleared on its own stream once its last users are done — beside the front
    // just enqueued, which uses the current set; the next front waits for the clear
    for (int k = 0; k < 3; ++k) HIPCHK(c, hipStreamWaitEvent(c->clr_stream, c->spare_free[k], 0));
    // the current set's last users: every tail enqueued so far, the fronts on the context
    // stream, and the deferred tail when it goes in (flush_tail)
    HIPCHK(c, hipEventRecord(c->spare_free[0], c->walk_stream));
    HIPCHK(c, hipEventRecord(c->spare_free[1], c->aux_stream));
    HIPCHK(c, hipEventRecord(c->spare_free[2], c->stream));
    c->spare_tail = c->tail_pending;
    std::swap(c->table, sp.table);
    std::swap(c->tstate, sp.tstate);
    std::swap(c->idx_heads, sp.heads);
    std::swap(c->idx_k6, sp.k6);
    std::swap(c->idx_mir, sp.mir);
    std::swap(c->idx_epoch, sp.epoch);
    c->pending_born = 0;
    c->count_bound = 0;
    // clear-free (the next table generation): only a set that holds lines of generations that
    // come round again — at the 16-bit wrap — is cleared
    const bool wrap = next_table_gen(c);
    if (c->spare_dirty || wrap || reset_clears())
        HIPCHK(c, launch_clear(c->table, c->slots * sizeof(Slot), c->clr_stream));
    c->spare_dirty = wrap;   // (the set just swapped out: its lines' generations come round again)
    HIPCHK(c, hipMemsetAsync(c->tstate, 0, kTableStateResetBytes, c->clr_stream));   // (path counters kept)
    if (++c->idx_epoch == 0x10000u) {   // (next_epoch, on the clear stream)
        HIPCHK(c, hipMemsetAsync(c->idx_heads, 0, c->slots * 8, c->clr_stream));
        c->idx_epoch = 1;
    }
    if (c->idx_mir) HIPCHK(c, hipMemsetAsync(c->idx_mir, 0, mir_bytes(c->idx_shift), c->clr_stream));
    HIPCHK(c, hipEventRecord(c->clr_done, c->clr_stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->clr_done, 0));
    ++c->tgen;
    c->fresh_tables = true;
    c->pro_fence = true;   // (the next early prologue waits for the clear, via the context stream)
    return 0;
}

int fsx_reset(fsx_ctx *c) {
    if (!c) return -EINVAL;
    if (reset_swap_ok(c)) return reset_swap(c);
    int rc = sel(c);
    if (rc) return rc;
    if (pipe_busy(c) && (rc = fsx_sync(c))) return rc;   // (pipelined batches)
    c->pending_born = 0;   // the whole table is wiped: no rollback of a pending batch
    c->count_bound = 0;    // (no source is tracked after the reset: ADVICE r04)
    // clear-free: the next table generation (every line of this one reads as empty)
    const bool wrap = next_table_gen(c);
    if (wrap || reset_clears()) HIPCHK(c, launch_clear(c->table, c->slots * sizeof(Slot), c->stream));
    if (wrap && c->spare.table) c->spare_dirty = true;
    HIPCHK(c, hipMemsetAsync(c->tstate, 0, kTableStateResetBytes, c->stream));   // (path counters kept)
    return next_epoch(c);   // (the prefix blocklists stay: configuration)   // every index head reads empty
}

// ------------------------------------------------------------------ scoring
int fsx_load_q8_model(fsx_ctx *c, const fsx_q8_model *m) {
    if (!c || !m) return -EINVAL;
    if (!(m->in_scale > 0.0f) || !(m->out_scale > 0.0f) || !(m->weight_scale > 0.0f))
        return set_err(c, -EINVAL, "scales must be positive");
    if (m->in_zero_point < 0 || m->in_zero_point > 255 || m->out_zero_point < 0 || m->out_zero_point > 255)
        return set_err(c, -EINVAL, "quint8 zero points must be in [0,255]");
    memcpy(c->w, m->weight, 8);
    c->inv_in = 1.0f / m->in_scale;
    const float ats = m->in_scale * m->weight_scale;      // act_times_w_scale (fp32)
    c->mult = ats / m->out_scale;                           // requantization multiplier
    c->bias_over_ats = m->bias / ats;                       // float bias folded into acc units
    c->zp_in = m->in_zero_point;
    c->zp_out = m->out_zero_point;
    // quantized sigmoid: output quint8 (scale 1/256, zero point 0), fp32 arithmetic
    for (int q = 0; q < 256; ++q) {
        volatile float x = (float)(q - m->out_zero_point) * m->out_scale;
        volatile float s = 1.0f / (1.0f + expf(-x));
        float r = rintf(s * 256.0f);
        c->lut[q] = (uint8_t)(r > 255.0f ? 255.0f : (r < 0.0f ? 0.0f : r));
    }
    c->model_loaded = true;
    return 0;
}

int fsx_score_device(fsx_ctx *c, const float *d_feat, size_t n, float *d_prob, uint8_t *d_dec) {
    if (!c) return -EINVAL;
    if (!c->model_loaded) return set_err(c, -EINVAL, "no model loaded (fsx_load_q8_model)");
    if (n && (!d_feat || !d_prob || !d_dec)) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_score(d_feat, n, d_prob, d_dec, c->w, c->inv_in, c->zp_in,
                                c->bias_over_ats, c->mult, c->zp_out, c->lut, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "score launch: %s", hipGetErrorString(e));
    return 0;
}

int fsx_score(fsx_ctx *c, const float *feat, size_t n, float *prob, uint8_t *mal) {
    if (!c) return -EINVAL;
    if (n && (!feat || !prob || !mal)) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    if (n == 0) return 0;
    if (n > c->score_cap) {
        hipFree(c->d_feat); hipFree(c->d_prob); hipFree(c->d_dec);
        c->d_feat = nullptr; c->d_prob = nullptr; c->d_dec = nullptr; c->score_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_feat, n * 32));
        HIPCHK(c, hipMalloc(&c->d_prob, n * 4));
        HIPCHK(c, hipMalloc(&c->d_dec, n));
        c->score_cap = n;
    }
    HIPCHK(c, hipMemcpyAsync(c->d_feat, feat, n * 32, hipMemcpyHostToDevice, c->stream));
    if ((rc = fsx_score_device(c, c->d_feat, n, c->d_prob, c->d_dec))) return rc;
    HIPCHK(c, hipMemcpyAsync(prob, c->d_prob, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(mal, c->d_dec, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

int fsx_flow_features(fsx_ctx *c, const uint8_t *hdr, const uint32_t *len, const uint64_t *ts,
                      size_t n, size_t cap, uint8_t *keys16, uint8_t *family, float *features,
                      size_t *n_flows_out) {
    if (!c || !n_flows_out) return -EINVAL;
    if (n && (!hdr || !len || !ts)) return set_err(c, -EINVAL, "null buffer");
    int rc = sel(c);
    if (rc) return rc;
    *n_flows_out = 0;
    if (n == 0) return 0;
    if ((rc = ensure_stage(c, n))) return rc;
    uint8_t *dk = nullptr, *df = nullptr;
    float *dfeat = nullptr;
    HIPCHK(c, hipMalloc(&dk, n * 16));
    HIPCHK(c, hipMalloc(&df, n));
    HIPCHK(c, hipMalloc(&dfeat, n * 32));
    HIPCHK(c, hipMemcpyAsync(c->d_hdr, hdr, n * 64, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_len, len, n * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_ts, ts, n * 8, hipMemcpyHostToDevice, c->stream));
    FlowRequest fr = flow_request(c, dk, df, dfeat, nullptr, nullptr, n);
    // verdict scratch: parse writes default verdicts; the limiter does not run
    rc = run_batch(c, PacketIn{c->d_hdr, nullptr, 0, nullptr, nullptr}, c->d_len, c->d_ts, n, c->d_verdict,
                   false, &fr);
    if (!rc) rc = fsx_sync(c);
    BatchState h{};
    if (!rc && hipMemcpy(&h, c->bs, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) rc = -EIO;
    const size_t m = std::min<size_t>(h.nseg, cap);
    if (!rc && m && keys16 && hipMemcpy(keys16, dk, m * 16, hipMemcpyDeviceToHost) != hipSuccess) rc = -EIO;
    if (!rc && m && family && hipMemcpy(family, df, m, hipMemcpyDeviceToHost) != hipSuccess) rc = -EIO;
    if (!rc && m && features && hipMemcpy(features, dfeat, m * 32, hipMemcpyDeviceToHost) != hipSuccess) rc = -EIO;
    hipFree(dk); hipFree(df); hipFree(dfeat);
    if (rc) return rc == -EIO ? set_err(c, -EIO, "flow features copy failed") : rc;
    *n_flows_out = h.nseg;
    return 0;
}

int fsx_flows_begin(fsx_ctx *c) {
    if (!c) return -EINVAL;
    if (c->cfg.flags & FSX_FLAG_OVERFLOW_ADMIT)   // (transient sources have no slot to carry sums in)
        return set_err(c, -EINVAL, "FSX_FLAG_OVERFLOW_ADMIT: not with fsx_flows_begin");
    int rc = sel(c);
    if (rc) return rc;
    if (!c->d_slot_acc) {
        if (busy(c) && (rc = fsx_sync(c))) return rc;
        HIPCHK(c, hipMalloc(&c->d_slot_acc, c->slots * slot_acc_bytes()));
        HIPCHK(c, hipMemsetAsync(c->d_slot_acc, 0, c->slots * slot_acc_bytes(), c->stream));   // epoch 0
        HIPCHK(c, hipMalloc(&c->d_flow_rows, 8));
        c->flow_epoch = 0;
    }
    if (++c->flow_epoch == 0) {   // (after 2^32 epochs: clear, so no stale epoch can match)
        HIPCHK(c, hipMemsetAsync(c->d_slot_acc, 0, c->slots * slot_acc_bytes(), c->stream));
        c->flow_epoch = 1;
    }
    c->flow_accum = true;
    return 0;
}

int fsx_flows_end(fsx_ctx *c, uint8_t *d_keys16, uint8_t *d_family, float *d_features, float *d_prob,
                  uint8_t *d_malicious, size_t cap, uint64_t *d_rows) {
    if (!c || !c->flow_accum) return -EINVAL;
    if (cap && (!d_keys16 || !d_family)) return set_err(c, -EINVAL, "null buffer");
    int rc = sel(c);
    if (rc) return rc;
    c->flow_accum = false;
    const FlowRequest fr = flow_request(c, d_keys16, d_family, d_features, d_prob, d_malicious, cap);
    unsigned long long *cnt = d_rows ? reinterpret_cast<unsigned long long *>(d_rows) : c->d_flow_rows;
    hipError_t e = launch_flows_end(c->d_slot_acc, c->flow_epoch, c->table, c->slots, c->lim.tgen, fr.keys16, fr.fam,
                                    fr.feat,
                                    fr.prob, fr.dec, fr.cap, fr.score, cnt, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "flows end: %s", hipGetErrorString(e));
    return 0;
}

int fsx_last_batch_info(fsx_ctx *c, uint64_t *info, int cap) {
    if (!c || (!info && cap > 0)) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    BatchState h;
    HIPCHK(c, hipMemcpy(&h, c->bs, sizeof(h), hipMemcpyDeviceToHost));
    TableState t;
    HIPCHK(c, hipMemcpy(&t, c->tstate, sizeof(t), hipMemcpyDeviceToHost));
    if (c->spare.tstate) {   // (the path counters are since fsx_open: both table sets')
        TableState t2;
        HIPCHK(c, hipMemcpy(&t2, c->spare.tstate, sizeof(t2), hipMemcpyDeviceToHost));
        t.n_hfast += t2.n_hfast;
        t.n_hrun += t2.n_hrun;
    }
    const uint64_t v[19] = {h.n_valid, h.nseg, h.n_new, h.any_v6, h.nonmono, h.max_len,
                            h.max_ts, h.allowed, h.dropped, h.n_rule, h.pay_ok, h.n_light,
                            c->last_evicted, h.hfast, h.n_admit, h.n_trans, t.n_hfast, t.n_hrun, h.ord};
    int k = 0;
    for (; k < cap && k < 19; ++k) info[k] = v[k];
    return k;
}

// ------------------------------------------------------------------ sharding
uint32_t fsx_shard_owner(const uint8_t *key16, int family, uint32_t n_shards) {
    if (!key16 || n_shards == 0) return 0;
    uint32_t k[4] = {0, 0, 0, 0};
    memcpy(k, key16, family == 6 ? 16 : 4);
    return shard_owner_of(family == 6 ? 2u : 1u, k, n_shards);
}

static int shard_pack(fsx_ctx *c, const uint8_t *d_hdr, const uint32_t *d_len, const uint64_t *d_ts, size_t n,
                      uint32_t G, uint32_t flags, const uint32_t *d_filter, uint8_t *d_verdict, void *d_records,
                      uint32_t *d_send_idx, uint64_t *d_counts) {
    if (!c) return -EINVAL;
    if (G == 0 || G > FSX_MAX_SHARDS) return set_err(c, -EINVAL, "n_shards must be 1..%d", FSX_MAX_SHARDS);
    if (n > kMaxBatchLimit) return set_err(c, -E2BIG, "n=%zu too large", n);
    if (!d_counts || (n && (!d_hdr || !d_len || !d_ts || !d_verdict || !d_records || !d_send_idx)))
        return set_err(c, -EINVAL, "null buffer");
    int rc = sel(c);
    if (rc) return rc;
    const uint64_t need = (uint64_t)(G + 1) * (n / 4096 + 1);   // (+ the replica-drop group)
    if (need > c->shard_cnt_cap) {
        if (busy(c) && (rc = fsx_sync(c))) return rc;   // (an earlier pack may still use them)
        hipFree(c->d_shard_cnt);
        hipFree(c->d_shard_stat);
        c->d_shard_cnt = nullptr;
        c->d_shard_stat = nullptr;
        c->shard_cnt_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_shard_cnt, need * 4));
        HIPCHK(c, hipMalloc(&c->d_shard_stat, need * 8));
        c->shard_cnt_cap = need;
    }
    if (!c->d_shard_ticket) HIPCHK(c, hipMalloc(&c->d_shard_ticket, 4));
    if (n > c->shard_scr_cap) {
        hipFree(c->d_shard_own);
        hipFree(c->d_shard_crec);
        c->d_shard_own = nullptr;
        c->d_shard_crec = nullptr;
        c->shard_scr_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_shard_own, n));
        HIPCHK(c, hipMalloc(&c->d_shard_crec, n * FSX_SHARD_RECORD16_BYTES));
        c->shard_scr_cap = n;
    }
    const Replica rep{c->d_rep, c->rep_slots ? c->rep_slots - 1 : 0};
    const bool filt = (flags & FSX_SHARD_FILTER_BLOCKLIST) && c->rep_valid;
    const bool compact = (flags & FSX_SHARD_COMPACT) != 0;
    const bool drop_rec = filt && (flags & FSX_SHARD_DROP_RECORDS);
    const bool regions = (flags & FSX_SHARD_REGIONS) != 0;
    hipError_t e = launch_shard_pack(d_hdr, d_len, d_ts, (uint32_t)n, G, d_verdict, d_records, d_send_idx,
                                     d_counts, c->d_shard_cnt, c->d_shard_own, c->d_shard_crec,
                                     filt ? &rep : nullptr, compact, drop_rec, filt ? d_filter : nullptr, regions,
                                     c->d_shard_stat, c->d_shard_ticket, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "shard pack: %s", hipGetErrorString(e));
    return 0;
}

int fsx_shard_pack_device(fsx_ctx *c, const uint8_t *d_hdr, const uint32_t *d_len, const uint64_t *d_ts,
                          size_t n, uint32_t G, uint32_t flags, uint8_t *d_verdict, void *d_records,
                          uint32_t *d_send_idx, uint64_t *d_counts) {
    return shard_pack(c, d_hdr, d_len, d_ts, n, G, flags, nullptr, d_verdict, d_records, d_send_idx, d_counts);
}

int fsx_shard_pack_filtered_device(fsx_ctx *c, const uint8_t *d_hdr, const uint32_t *d_len, const uint64_t *d_ts,
                                   size_t n, uint32_t G, uint32_t flags, const uint32_t *d_filter,
                                   uint8_t *d_verdict, void *d_records, uint32_t *d_send_idx, uint64_t *d_counts) {
    if (!d_filter) return c ? set_err(c, -EINVAL, "null filter flag") : -EINVAL;
    return shard_pack(c, d_hdr, d_len, d_ts, n, G, flags | FSX_SHARD_FILTER_BLOCKLIST, d_filter, d_verdict,
                      d_records, d_send_idx, d_counts);
}

int fsx_shard_filter_plan_device(fsx_ctx *c, const uint64_t *d_clocks, uint32_t G, uint32_t k, uint32_t *d_filter) {
    if (!c || !d_clocks || !d_filter || G == 0 || G > FSX_MAX_SHARDS || k == 0) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_filter_plan(d_clocks, G, k, d_filter, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "filter plan: %s", hipGetErrorString(e));
    return 0;
}

int fsx_shard_clock_device(fsx_ctx *c, const uint64_t *d_ts, size_t n, uint64_t *d_out3) {
    if (!c || !d_out3 || (n && !d_ts)) return -EINVAL;
    if (n > kMaxBatchLimit) return set_err(c, -E2BIG, "n=%zu too large", n);
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_shard_clock(d_ts, (uint32_t)n, d_out3, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "shard clock: %s", hipGetErrorString(e));
    return 0;
}

int fsx_blocklist_export_device(fsx_ctx *c, void *d_entries, size_t cap, uint64_t *d_count) {
    if (!c || !d_count || (cap && !d_entries)) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    // (stream-ordered after a pending batch; its errors surface at the next fsx_sync)
    hipError_t e = launch_blocklist_export(c->table, c->lim.table_mask, c->lim.tgen, reinterpret_cast<ShardBlock *>(d_entries),
                                           cap, reinterpret_cast<unsigned long long *>(d_count), c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "blocklist export: %s", hipGetErrorString(e));
    return 0;
}

int fsx_blocklist_replica_blocks_device(fsx_ctx *c, const void *d_blocks, uint32_t n_blocks, size_t cap) {
    if (!c || (n_blocks && cap && !d_blocks)) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    const uint64_t need = next_pow2(std::max<uint64_t>(64, 2 * (uint64_t)n_blocks * cap));
    if (need > c->rep_slots) {
        HIPCHK(c, hipStreamSynchronize(c->stream));   // (grows once: capacities are fixed per plane)
        hipFree(c->d_rep);
        c->d_rep = nullptr;
        c->rep_slots = 0;
        c->rep_valid = false;
        HIPCHK(c, hipMalloc(&c->d_rep, need * sizeof(ShardBlock)));
        c->rep_slots = need;
    }
    hipError_t e = launch_replica_build_blocks(d_blocks, n_blocks, cap, c->d_rep, c->rep_slots - 1, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "replica build: %s", hipGetErrorString(e));
    c->rep_valid = true;
    return 0;
}

int fsx_blocklist_replica_device(fsx_ctx *c, const void *d_entries, size_t m) {
    if (!c || (m && !d_entries)) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    const uint64_t need = next_pow2(std::max<uint64_t>(64, 2 * (uint64_t)m));
    if (need > c->rep_slots) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        hipFree(c->d_rep);
        c->d_rep = nullptr;
        c->rep_slots = 0;
        c->rep_valid = false;
        HIPCHK(c, hipMalloc(&c->d_rep, need * sizeof(ShardBlock)));
        c->rep_slots = need;
    }
    hipError_t e = launch_replica_build(reinterpret_cast<const ShardBlock *>(d_entries), m, c->d_rep,
                                        c->rep_slots - 1, c->stream);
    if (e != hipSuccess)
        return set_err(c, -EIO, "replica build (m=%zu slots=%llu rep=%p in=%p stream=%p): %s", m,
                       (unsigned long long)c->rep_slots, (void *)c->d_rep, d_entries, (void *)c->stream,
                       hipGetErrorString(e));
    c->rep_valid = true;
    return 0;
}

static int shard_unpack(fsx_ctx *c, const void *d_records, uint32_t rec_bytes, size_t m, uint8_t *d_hdr,
                        uint32_t *d_len, uint64_t *d_ts) {
    if (!c) return -EINVAL;
    if (m > kMaxBatchLimit) return set_err(c, -E2BIG, "m=%zu too large", m);
    if (m && (!d_records || !d_hdr || !d_len || !d_ts)) return set_err(c, -EINVAL, "null buffer");
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_shard_unpack(d_records, rec_bytes, (uint32_t)m, d_hdr, d_len, d_ts, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "shard unpack: %s", hipGetErrorString(e));
    return 0;
}

int fsx_shard_unpack_device(fsx_ctx *c, const void *d_records, size_t m, uint8_t *d_hdr, uint32_t *d_len,
                            uint64_t *d_ts) {
    return shard_unpack(c, d_records, FSX_SHARD_RECORD_BYTES, m, d_hdr, d_len, d_ts);
}

int fsx_shard_unpack16_device(fsx_ctx *c, const void *d_records, size_t m, uint8_t *d_hdr, uint32_t *d_len,
                              uint64_t *d_ts) {
    return shard_unpack(c, d_records, FSX_SHARD_RECORD16_BYTES, m, d_hdr, d_len, d_ts);
}

int fsx_shard_scatter_device(fsx_ctx *c, const uint8_t *d_ret, const uint32_t *d_send_idx, size_t m,
                             uint8_t *d_verdict) {
    if (!c) return -EINVAL;
    if (m > kMaxBatchLimit) return set_err(c, -E2BIG, "m=%zu too large", m);
    if (m && (!d_ret || !d_send_idx || !d_verdict)) return set_err(c, -EINVAL, "null buffer");
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_shard_scatter(d_ret, d_send_idx, (uint32_t)m, d_verdict, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "shard scatter: %s", hipGetErrorString(e));
    return 0;
}

int fsx_shard_scatter_regions_device(fsx_ctx *c, const uint8_t *d_ret, const uint32_t *d_send_idx, size_t m,
                                     size_t region, const uint64_t *d_counts, uint32_t n_shards,
                                     uint8_t *d_verdict) {
    if (!c) return -EINVAL;
    if (m > kMaxBatchLimit) return set_err(c, -E2BIG, "m=%zu too large", m);
    if (n_shards == 0 || n_shards > FSX_MAX_SHARDS) return set_err(c, -EINVAL, "n_shards must be 1..%d", FSX_MAX_SHARDS);
    if (m && (!d_ret || !d_send_idx || !d_verdict || !d_counts)) return set_err(c, -EINVAL, "null buffer");
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_shard_scatter_regions(d_ret, d_send_idx, (uint32_t)m, region, d_counts, n_shards, d_verdict,
                                                c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "shard scatter: %s", hipGetErrorString(e));
    return 0;
}

// ------------------------------------------------------------------ pcap
int fsx_pcap_records_device(fsx_ctx *c, const uint8_t *d_buf, const uint64_t *d_off, const uint32_t *d_caplen,
                            size_t n, uint8_t *d_hdr) {
    if (!c) return -EINVAL;
    if (n > kMaxBatchLimit) return set_err(c, -E2BIG, "n=%zu too large", n);
    if (n && (!d_buf || !d_off || !d_caplen || !d_hdr)) return set_err(c, -EINVAL, "null buffer");
    int rc = sel(c);
    if (rc) return rc;
    hipError_t e = launch_pcap_records(d_buf, d_off, d_caplen, (uint32_t)n, d_hdr, c->stream);
    if (e != hipSuccess) return set_err(c, -EIO, "pcap records: %s", hipGetErrorString(e));
    return 0;
}

// ------------------------------------------------------------------ timing
int fsx_enable_timing(fsx_ctx *c, int on) {
    if (!c) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    if (on && !c->ev_ready) {
        for (int r = 0; r < kRing; ++r)
            for (int i = 0; i < kMaxEv; ++i) HIPCHK(c, hipEventCreate(&c->ev[r][i]));
        c->ev_ready = true;
    }
    if (!on && (rc = drain_timings(c))) return rc;
    c->timing = on != 0;
    return 0;
}

int fsx_last_timings(fsx_ctx *c, float *ms_per_batch, float *launches_per_batch, char *names,
                     int cap, int name_len, int *count) {
    if (!c || !count) return -EINVAL;
    int rc = sel(c);
    if (rc) return rc;
    if ((rc = drain_timings(c))) return rc;
    const double nb = c->acc_batches ? (double)c->acc_batches : 1.0;
    int k = 0;
    for (; k < c->acc_n && k < cap; ++k) {
        if (ms_per_batch) ms_per_batch[k] = (float)(c->acc_ms[k] / nb);
        if (launches_per_batch) launches_per_batch[k] = (float)(c->acc_cnt[k] / nb);
        if (names && name_len > 0) {
            strncpy(names + (size_t)k * name_len, c->acc_name[k], name_len - 1);
            names[(size_t)k * name_len + name_len - 1] = 0;
        }
    }
    *count = k;
    c->acc_n = 0;
    c->acc_batches = 0;
    return 0;
}

}  // extern "C"
