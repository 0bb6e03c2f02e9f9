// Internal state of libmicrorank_hip.so.  gfx950 only: 64-lane wavefronts, 160 KiB LDS/CU.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <unordered_map>
#include <utility>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/microrank_hip.h"

constexpr int WAVE = 64;

struct mr_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t flags = 0;
    std::string err;
    // RCCL (loaded lazily with dlopen so the library loads without it)
    void* comm = nullptr;
    int rank = 0, nranks = 1;
    // host-staged collective backend (mr_comm_set_host), used when no RCCL communicator is set
    mr_host_coll_fn host_coll = nullptr;
    void* host_user = nullptr;
    // live kernel timing of the power-iteration launches (mr_ctx_profile): event pairs on the
    // context stream plus the algorithmic bytes of each launch
    bool prof = false;
    std::vector<hipEvent_t> prof_ev;
    std::vector<double> prof_bytes;
    std::vector<int64_t> prof_iters;   // iterations each record covers
    // stream-ordered caching allocator: every buffer of this context is used on `stream` only,
    // so a block released by one call can be handed to the next without a hipFree/hipMalloc
    // (each of which synchronises the device and costs tens of microseconds)
    std::mutex pool_mu;   // (mr_windows_batch releases a call's graphs while its threads allocate)
    // (free blocks as one stack per size class -- a free is a push, no node allocation; a block's
    // class travels with its DBuf, so a free needs no lookup of the block: a window batch releases
    // thousands of blocks on the host's critical path.  pool_all: every block hipMalloc'ed here,
    // touched only by hipMalloc / hipFree, for the context's destruction)
    std::map<size_t, std::vector<void*>> pool_free;
    std::unordered_map<void*, size_t> pool_all;
    size_t pool_bytes = 0;
    // mr_windows_batch: auxiliary contexts (own stream + pool) for the windows' concurrent
    // detector / graph-build / spectrum phases; created on first use, destroyed with this one
    std::vector<mr_ctx*> aux;
    // mr_windows_batch: the previous call's window graphs, released by the next call while its
    // PageRank stream waits for the first group's builds (or by mr_ctx_destroy)
    std::vector<struct mr_graph*> graveyard;
    // a second stream for work that overlaps the main stream inside one call (wide graphs:
    // k_cold_ops beside k_cold_trace / k_tr_a), joined back by events; created on first use
    hipStream_t side = nullptr;
    hipEvent_t side_ev[2] = {nullptr, nullptr};
    // pinned host words for the small size read-backs of a call (a DMA straight into host memory
    // instead of the runtime's pageable staging path); created on first use
    int64_t* pin = nullptr;
    // pinned error words of the PageRank groups a window batch has in flight (grown per call)
    int32_t* pin_flags = nullptr;
    size_t pin_flags_n = 0;
    // one-shot peer all-reduce (mr_comm_peer_enable; mr_comm.hip): a receive region in uncached
    // device memory exported by IPC -- [flags: PEER_FLAGS u64][data: 2 parities x nranks x
    // peer_words u64] -- and every rank's region mapped into this process (peer_map[rank] = ours)
    bool peer_on = false;
    void* peer_region = nullptr;
    int64_t peer_words = 0, peer_xa = 0, peer_xb = 0;   // all-reduce slot words, exchange areas
    std::vector<void*> peer_map;
    unsigned long long** peer_dev = nullptr;   // device copy of peer_map
    uint64_t peer_seq = 0;                      // all-reduces completed (slot parity)
    uint64_t peer_arrived = 0;                  // blocks every source has pushed so far (the flags' target)
    uint64_t peer_xseq = 0;                     // exchange rounds completed
    int64_t peer_nbf = 0;                       // k_fx_b blocks the block-flag area holds per source
    bool peer_same_dev = false;                 // some other rank runs on this rank's device
    struct PeerOld {   // a replaced region and its mappings, kept until the context goes (mr_comm.hip)
        void* region;
        unsigned long long** dev;
        std::vector<void*> map;
        int rank;
    };
    std::vector<PeerOld> peer_old;
    // status words of the single-pass scans (mr_prim.hip k_scan_dl): per-call epochs, no clearing
    unsigned long long* scan_st = nullptr;
    size_t scan_cap = 0;
    uint32_t scan_epoch = 0;
};

void* mr_pool_alloc(mr_ctx* ctx, size_t bytes, size_t* cls);   // *cls: the block's size class
void mr_graph_delete(struct mr_graph* g);   // delete a graph (defined where mr_graph is complete)
void mr_pool_free(mr_ctx* ctx, void* p, size_t cls);
void mr_pool_release(mr_ctx* ctx);
// n (<= 64) int64 words from the device into out, through the context's pinned words; syncs the stream
int mr_read_words(mr_ctx* ctx, const int64_t* dev, int n, int64_t* out);
// up to MR_PIN_BYTES bytes from the device into the context's pinned buffer (*host points there,
// valid until the next read-back on this context); syncs the stream
constexpr size_t MR_PIN_BYTES = 65536;
int mr_read_bytes(mr_ctx* ctx, const void* dev, size_t bytes, unsigned char** host);
int mr_win_spectrum_small(mr_ctx* ctx, int32_t Na, const int32_t* a_podop, const double* a_w, const int32_t* a_cov,
                          int32_t Nn, const int32_t* n_podop, const double* n_w, const int32_t* n_cov, int32_t NP,
                          int64_t A, int64_t Nl, int method, int32_t k, int32_t* out_codes, double* out_score,
                          int32_t* n_out);

int mr_fail(mr_ctx* ctx, int code, const char* fmt, ...);

#define MR_TRY_HIP(ctx, call)                                                                  \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return mr_fail((ctx), MR_ERR_HIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_),  \
                           __FILE__, __LINE__);                                                \
    } while (0)

#define MR_TRY(expr)                \
    do {                            \
        int rc_ = (expr);           \
        if (rc_ != MR_OK) return rc_; \
    } while (0)

// Owned device allocation.
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    mr_ctx* owner = nullptr;
    size_t cls = 0;   // the pool block's size class
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { reset(); }
    void swap(DBuf& o) {
        std::swap(p, o.p);
        std::swap(n, o.n);
        std::swap(owner, o.owner);
        std::swap(cls, o.cls);
    }
    void reset() {
        if (p) mr_pool_free(owner, p, cls);
        p = nullptr;
        n = 0;
    }
    int alloc(mr_ctx* ctx, size_t count) {
        if (count <= n && p) return MR_OK;
        reset();
        size_t bytes = (count ? count : 1) * sizeof(T);
        p = (T*)mr_pool_alloc(ctx, bytes, &cls);
        if (!p) return mr_fail(ctx, MR_ERR_OOM, "device allocation of %zu bytes failed", bytes);
        owner = ctx;
        n = count;
        return MR_OK;
    }
    int upload(mr_ctx* ctx, const T* host, size_t count) {
        MR_TRY(alloc(ctx, count));
        if (count)
            MR_TRY_HIP(ctx, hipMemcpyAsync(p, host, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
        return MR_OK;
    }
    int download(mr_ctx* ctx, T* host, size_t count) const {
        if (count)
            MR_TRY_HIP(ctx, hipMemcpyAsync(host, p, count * sizeof(T), hipMemcpyDeviceToHost, ctx->stream));
        return MR_OK;
    }
    int zero(mr_ctx* ctx, size_t count) {
        MR_TRY(alloc(ctx, count));
        if (count) MR_TRY_HIP(ctx, hipMemsetAsync(p, 0, count * sizeof(T), ctx->stream));
        return MR_OK;
    }
};

// Device graph: the four reference dicts as incidence lists.
// the kinds hash table (mr_pagerank.hip): 64-bit keys in one array (the CAS-probed one, half the
// footprint of a packed slot -- it stays MALL-resident longer), class size + representative in a
// second 8 B array (one line for k_kind_verify's read)
struct alignas(8) KCnt {
    uint32_t cnt;
    int32_t rep;
};

struct mr_graph {
    mr_ctx* ctx = nullptr;
    int32_t N = 0, T = 0;
    int64_t nnz_sr = 0, nnz_rs = 0, E = 0;
    bool rs_is_sr = true;
    // trace-major P_rs incidence (r' pass) and P_sr incidence (kinds)
    DBuf<int64_t> rs_off;
    DBuf<int32_t> rs_ops;
    DBuf<int64_t> srt_off;   // only when !rs_is_sr
    DBuf<int32_t> srt_ops;
    // trace-major P_rs node ids as u16 when N <= 65536 (the r' pass reads half the bytes)
    DBuf<uint16_t> rs16;
    // fused iteration with N too large for su in LDS beside the accumulators: ops relabelled by
    // descending coverage (perm[new] = old), the kernel's id stream rsp in the new labels, and
    // su of the n_hot most covered ops staged in LDS (the rest gathered from HBM/L2)
    DBuf<int32_t> perm;
    DBuf<uint16_t> rsp;
    bool relabeled = false;
    // trace-parallel layout of the fused iteration (k_tr_a): traces sorted by op count (tperm[p]
    // = trace at position p), wave tiles of 64 consecutive positions, each tile's ids in chunks
    // of 4 per lane stored lane-interleaved ([chunk][lane] x 8 B: one 512-B load per chunk),
    // each trace's ids rotated by (lane mod len) and padded with N + lane
    int32_t n_wt = 0;                // wave tiles
    DBuf<int32_t> tperm;             // [T]
    DBuf<uint16_t> tids;             // [coff[n_wt] * 256]
    DBuf<int32_t> coff;              // [n_wt+1] first chunk of a tile
    std::vector<int32_t> coff_h;     // host copy (the per-wave tile split of a launch)
    DBuf<float> w_tp, c_tp;          // [T] w_t, c_t in position order
    DBuf<int32_t> tpos;              // [T] position of each trace (inverse of tperm; large graphs, built on first use)
    bool tpos_ok = false;
    // register-accumulated hot ops (large graphs, su in LDS): the nhr <= 8 ops present in most
    // traces leave the id chunks; hmask[p] (position order) says which of them trace p holds
    int32_t nhr = 0;
    int32_t hop[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    DBuf<uint8_t> hmask;
    // kind compression (MR_PR_KIND_COMPRESS): a graph of one representative trace per kind whose
    // q carries the kind's multiplicity (mw_tp = w_t * mult in position order); kind = mult
    bool kinds_given = false;
    // wide fused graphs (N > 16384, e.g. C5's 100k ops): ops relabelled by coverage, the NA
    // most covered ("hot") ops go through k_tr_a (their u16 ids, LDS accumulator); each trace's
    // other ("cold") entries are summed per position by k_cold_trace (cold_acc, added to r') and
    // accumulated per op range in LDS by k_cold_ops from (position, op) pairs sorted by range
    bool wide = false;
    int32_t NA = 0;                  // k_tr_a's ops (= N unless wide)
    DBuf<int64_t> hot_off;           // [T+1] hot entries per trace (u16 ids in hot16)
    DBuf<uint16_t> hot16;
    DBuf<int32_t> cold_off_p, cold_ops_p;   // [T+1], [n_cold]: cold op ids per position
    DBuf<int32_t> cp_pos;            // [n_cold] cold pairs, by (range, position): position ...
    DBuf<uint16_t> cp_op;            // ... and op - range base
    int32_t cold_rw = 0, n_ranges = 0, n_cb = 0;
    int64_t n_cold = 0;
    uint64_t cold_span = 0;          // widest position span of a k_cold_ops block (its scale)
    DBuf<int32_t> cold_rowbase;      // [n_ranges+1] first k_cold_ops block (row) of each range
    DBuf<int64_t> cb_beg;            // [n_cb+1] pair slice of each block
    DBuf<uint64_t> cold_part;        // [n_cb * cold_rw] partial rows of the cold ranges
    DBuf<double> cold_acc;           // [T] per position: sum of su over the trace's cold entries
    // the short-tile walk takes each tile's cold entries itself (su gathered from L2): per wave
    // tile ceil(max cold / 2) chunks of 64 lanes x 2 u32 op labels (pads N + lane), cold_acc only
    // for the long tiles of the general walk and the tiles with more than two cold chunks (ctl)
    DBuf<uint32_t> ctids;
    DBuf<int32_t> ccoff;             // [n_wt+1] first cold chunk of a tile
    DBuf<int32_t> ctl;               // [n_ctl] tiles whose cold sums k_cold_trace computes
    int32_t n_ctl = 0;
    DBuf<double> mult, mw_tp;
    std::vector<int64_t> tile_mult_h;   // per wave tile: the multiplicity its traces stand for
    DBuf<int32_t> krep;              // [T] class representative of each trace (when allocated)
    int64_t kc_kinds = 0;            // kinds of the last kind-compressed ranking (0: none)
    std::unique_ptr<mr_graph> kc;    // the representatives' graph of a kind-compressed ranking, kept for the next call
    // mr_pagerank_presetup: kinds / preference / iteration state already set up for the next call
    bool pre_ok = false, pre_fp32 = false;
    int pre_anomaly = 0;
    double pre_d = 0.0, pre_phi = 0.5;
    // the anomaly preference's weight phi (pagerank.py:82-84: 0.5 at both places), set per call
    double phi = 0.5;
    uint32_t pre_flags = 0;
    uint64_t pre_seed = 0, pre_hmask = 0;
    DBuf<int32_t> wtile;             // [waves+1] first tile of each wave of the last launch plan
    int32_t wtile_nw = 0;            // waves that wtile was cut for
    int32_t wtile_tpb = 0;           // most tiles of one block under that cut
    DBuf<double> dscale;             // {2^SC, 2^-SC} of a device-side cut (k_tr_cut; wtile_msum < 0)
    int64_t wtile_msum = 0;          // most traces one block stands for (x multiplicity when compressed)
    // P_sr in compressed sparse blocks for the s' pass: traces cut in tiles of 2^tshift; within a
    // tile the distinct (op, trace) entries sorted by (op, trace) as u16 tile-local trace
    // indices; a "pair" is the run of one op inside one tile.
    int32_t tshift = 0, n_tiles = 0;
    int64_t n_pairs = 0;
    DBuf<uint16_t> tl_ltr;    // [nnz_sr] tile-local trace index, (tile, op, trace) order
    DBuf<int32_t> pr_op;      // [n_pairs] op of the pair
    DBuf<int64_t> pr_beg;     // [n_pairs+1] first entry in tl_ltr
    DBuf<int32_t> tile_pr0;   // [n_tiles+1] first pair of a tile
    DBuf<int32_t> lp;         // [<= n_pairs] long pairs (summed by a whole wave), tile order
    DBuf<int32_t> tile_lp0;   // [n_tiles+1]
    DBuf<int32_t> op_pr_off;  // [N+1] pairs of an op ...
    DBuf<int32_t> op_pr;      // [n_pairs] ... in tile order (the s' reduction order)
    // fused single-pass iteration (N <= FX_NMAX, P_rs == P_sr): one read of the trace-major ids
    // per iteration; the s' side accumulates per trace block in LDS as 64-bit fixed point and
    // leaves one dense row of N partials per block (exact integer sums: order-free)
    bool fused = false;
    bool traces_nonempty = true;   // every trace has an op (span-built graphs; checked at upload)
    bool force_tile = false;       // the ranks of a sharded graph agreed on the tile path
    int64_t T_all = 0;             // traces over all shards (0: this graph is whole)
    bool sharded_done = false;     // mr_pagerank_sharded's graph-level exchange has run
    DBuf<uint64_t> fx_part;   // [n_blocks * N]
    DBuf<double> fx_ssv;      // [N] alpha * (P_ss s_k)[o] / M_s(k), from k_fx_a for k_fx_b
    DBuf<uint64_t> fx_limb;   // [2N] sharded graphs: exact limb sums per op, all-reduced per iteration
    DBuf<double> op_sum;      // [N] sharded tile-path graphs: this rank's P_sr r per op, all-reduced
    // per-trace / per-op constants
    DBuf<int32_t> len_t, len_o, nchild, cov;
    bool cov_ready = false;          // cov filled by the build (the indexed K1), else by mr_graph_prepare
    DBuf<float> w_t, u_o, pw;    // fp32(1/len_t), fp32(1/len_o), fp32(1/nchild)
    DBuf<int64_t> ss_off;        // P_ss by child
    DBuf<int32_t> ss_par;
    int32_t n_pr = 0;
    bool pr_identity = true;     // pr_trace keys == operation_trace keys in order
    DBuf<int32_t> pr_trace, pr_len;
    // node order / trace codes (graphs built from spans)
    DBuf<int32_t> node_podop, trace_code;
    // iteration state and outputs
    DBuf<double> kind;           // [T]
    DBuf<float> pref;            // [T] preference vector v (fp32, as the reference)
    DBuf<float> c_t;             // [T] fp32((1-d) * v)
    DBuf<double> q64[2];         // [T] w_t * r'_t (fp64 mode)
    DBuf<float> q32[2];          // [T] (fp32 mode)
    DBuf<double> part;           // [n_pairs] per-(tile, op) partial sums of the s' pass
    DBuf<unsigned long long> mslot;  // [6] bits of (M_s, M_r) for iterations k%3
    DBuf<double> spb[2];         // [N] unnormalised s' (double-buffered)
    DBuf<double> sub[2];         // [N] u_o * s'[o]
    DBuf<float> suf[2];          // fp32 wide graphs: the same, as floats (k_tr_a's warm gathers)
    DBuf<double> sn;             // [N] final normalised s
    DBuf<double> scal;           // [8] M_s, M_r, sums
    DBuf<double> ppart;          // preference-sum block partials
    DBuf<double> weight;         // [N]
    DBuf<unsigned long long> ht_key;   // kinds hash table keys
    DBuf<KCnt> ht_cr;                  // per slot: class size, representative
    DBuf<int32_t> slot_of;
    DBuf<uint64_t> ht_chk;   // sharded on >1 rank: check hash of each class's representative
    DBuf<int32_t> flag;          // [4] error flags written by kernels
    // a window graph tiled from its table's layout order (mr_lo_prepare_batch): no trace-major
    // incidence (rs_off / rs_ops / rs16 / tperm are empty); kind counts and span counts by
    // position (kind, lo_lenp) and the preference partials (ppart) stay for a re-set-up
    bool lo = false;
    DBuf<int32_t> lo_lenp;       // [T] span count by position
    // [T] by position: the length of the run of identical traces (one kind class, adjacent in a
    // wave tile) a position heads, 0 for the run's other positions (k_tr_a's walk merges the run)
    DBuf<uint8_t> trun;
    int lo_merged = 0;           // MR_TR_MERGE at prepare: 1 runs share a rotation and k_tr_a walks
                                 // each by its head (trun); 2 the rotations only (tests); 0 neither
    int32_t lo_nbp = 0;          // preference partial blocks
};

// edge entries from which the index also keeps them in edge-id order (mr_spans.eb_*);
// MR_IX_EB (read per ingest / build): "0" never, "force" at any size (tests)
constexpr int64_t ED_BYID_MIN = (int64_t)1 << 22;
struct mr_spans {
    mr_ctx* ctx = nullptr;
    int64_t S = 0;
    int32_t n_traces = 0, n_podops = 0, n_svcops = 0;
    DBuf<int32_t> trace, podop, svcop;
    DBuf<int64_t> span, parent, duration, tstart, tend;
    bool has_times = false;
    DBuf<int32_t> grow;          // global row index per row (a shard of a larger table), or empty
    int row_bits = 0;            // bits of the largest (global) row index + 1
    // spanID -> rows multimap over the whole table (static; built at upload)
    int64_t n_span_codes = 0;
    DBuf<int64_t> id_off;   // [n_span_codes+1]
    DBuf<int32_t> id_rows;  // [S]
    // Per-trace index (mr_span_index.hip), built once at upload: everything a window needs from
    // a trace, so detector and graph builds of a window are per-trace gathers with no row sort.
    bool indexed = false;        // index built (key bits fit)
    bool uniform_times = false;  // tstart/tend constant within every trace (window = trace set)
    DBuf<int32_t> tlen;                  // [NT] rows of the trace
    DBuf<long long> tmaxd, tts, tte;     // [NT] max duration, trace-level start / end
    int64_t n_po = 0, n_sv = 0, n_ed = 0, n_xj = 0;
    int64_t n_edge_keys = 0;             // distinct (parent op, child op) over the table: edge-set bound
    DBuf<uint64_t> ekey;                 // [n_edge_keys] those keys, ascending (parent << 32 | child)
    DBuf<int32_t> ed_eid, xj_eid;        // [n_ed], [n_xj] the dense edge id (index into ekey) of a key
    DBuf<int64_t> po_off;                // [NT+1] distinct pod-ops of a trace (code order) ...
    DBuf<int32_t> po_op, po_cnt, po_first, po_tr;   // ... with span count, first row and trace
    DBuf<int64_t> sv_off;                // [NT+1] distinct service-ops of a trace (code order) ...
    DBuf<int32_t> sv_op, sv_cnt;         // ... with span count
    DBuf<int64_t> ed_off;                // [NT+1] distinct (parent pod-op, child pod-op) join keys
    DBuf<uint64_t> ed_key;               //        inside the trace, (parent << 32 | child) ...
    DBuf<int32_t> ed_cnt, ed_tr;         // ... with multiplicity and trace
    // large tables (n_ed >= ED_BYID_MIN): the edge entries again, in edge-id order (trace, count,
    // id), so a build counts its edges by a segmented sum per id instead of an atomic per entry
    DBuf<int32_t> eb_tr, eb_cnt, eb_eid;
    DBuf<int32_t> xj_tc, xj_tp;          // [n_xj] join pairs across traces (T11): child / parent trace
    DBuf<uint64_t> xj_key;               //        and key
    // Window-independent layout of the traces (mr_span_index.hip lo_index; tables of <= NS_PMAX
    // pod-ops): the trace ORDER k_tr_a tiles a graph in (by distinct pod-op count, then code), each
    // trace's pod-op codes as u16 in that order, its span count, and its exact kind class among the
    // table's traces (pagerank.py:54-66's key -- distinct op set, fp32(1/len_t) -- is a property of
    // the trace alone, so a graph's class size is a histogram of the class ids of its traces).  A
    // window's graphs then tile, fill and set up from these by position, without re-sorting,
    // re-hashing or gathering per-trace lists in tile order (mr_lo_launch_batch / _prepare_batch).
    // The window build (k_lo_build_b) reads everything of a trace from these copies in layout
    // order: its detector inputs (times, max duration, service-op entries), its pod-op entries (code,
    // span count, first row) and its join entries (dense edge id, multiplicity) -- consecutive lanes,
    // consecutive traces, contiguous entries.
    bool lo_ok = false;
    int32_t lo_nk = 0;                   // kind classes of the table
    DBuf<int32_t> lo_tr, lo_len, lo_kid; // [NT] by layout index: trace code, span count, kind class
    DBuf<int64_t> lo_off;                // [NT+1] first entry of each trace in lo16
    DBuf<uint16_t> lo16, lo_cnt;         // [n_po] pod-op codes (ascending) and span counts, layout order
    DBuf<int32_t> lo_first;              // [n_po] first row of each pod-op entry
    DBuf<long long> lo_ts, lo_te, lo_mx; // [NT] trace-level start / end, max duration
    DBuf<int32_t> lo_bstart;             // [lo_nblk+1] window-build blocks: layout ranges (LO_BT_MAX / LO_BE)
    int32_t lo_nblk = 0;
    DBuf<int64_t> lsv_off, le_off;       // [NT+1] service-op entries / join entries of each trace
    DBuf<uint32_t> lsv, le;              // svcop | count << 16 (code order); dense edge id | count << 16
    // tables ingested from strings (mr_spans_ingest): the first row of each trace / pod-op /
    // service-op code, in code order (the host builds the name lists from them)
    DBuf<int32_t> dict_rows[3];
    // streaming tables (mr_spans_append): the six string columns stay on the device (offsets +
    // bytes with 16 zero bytes of tail padding, ParentSpanId validity bitmap or empty) so the next
    // append uploads only its chunk, and src[row] numbers every row by its position in the stream
    // of appended chunks (the host looks names up in the chunk that holds that row)
    bool raw = false;
    DBuf<int64_t> raw_off[6];
    DBuf<uint8_t> raw_bytes[6], raw_valid;
    DBuf<int64_t> src;
    int64_t src_next = 0;
};

int mr_spans_index(mr_ctx* ctx, mr_spans* s);

// Handles given out across the ABI (graphs, span tables) are registered with their context:
// mr_ctx_destroy frees the ones still live, and freeing a handle that is not registered (its
// context already destroyed it) does nothing.
void mr_handle_add(mr_ctx* ctx, void* h, void (*del)(void*));
bool mr_handle_take(void* h);   // unregister; false when h is not live

// collectives over the context's backend (RCCL communicator or host callback); device buffers
enum { MR_DT_F64 = 0, MR_DT_I32 = 1, MR_DT_U64 = 2, MR_DT_I64 = 3 };
int mr_coll_allreduce(mr_ctx* ctx, void* dbuf, int64_t n, int dtype, int op /*0 sum, 1 max*/);
int mr_coll_allgather(mr_ctx* ctx, const void* dsend, void* drecv, int64_t n, int dtype);
inline bool mr_coll_ready(const mr_ctx* ctx) { return ctx->comm || ctx->host_coll; }
// SUM all-reduce of n uint64 words through the peer receive regions (one push to every rank, one
// local sum in rank order); MR_ERR_STATE when the peer path is off (callers then use
// mr_coll_allreduce).  Collective: every rank calls it with the same n.
int mr_peer_allreduce_u64(mr_ctx* ctx, unsigned long long* dbuf, int64_t n);
int mr_peer_allreduce_f64(mr_ctx* ctx, double* dbuf, int64_t n);   // (fp64 sums in rank order)
// (collective) MR_ERR_COMM when a round timed out on any rank (a peer never pushed); the regions
// are then reset on every rank
int mr_peer_check(mr_ctx* ctx, const char* what);
// the exchange fused into k_fx_b (mr_comm.hip): region addresses and the round
struct MrPeerX {
    unsigned long long* const* peers;   // device table of every rank's region (null: off)
    unsigned long long* region;         // this rank's region
    int32_t R, rank, nbf, spin;         // spin: mode-2 blocks wait themselves (0: k_peer_bwait did)
    int32_t mute;                       // (tests: MR_PEER_TEST_MUTE) this rank never signals its rounds
    int64_t slots, W, bflags, err;      // word offsets in a region: slot area, words per slot, block flags, error word
    uint64_t seq;                       // the round (slot parity seq & 1, flags store seq + 1)
    unsigned long long timeout;         // s_memrealtime ticks
};
int mr_peer_fx_prepare(mr_ctx* ctx, int64_t words, int32_t nbf, MrPeerX* px);   // (collective)
int mr_peer_fx_wait(mr_ctx* ctx, const MrPeerX& px, int32_t nb);   // one block waits for every flag of the round
void mr_peer_fx_round_done(mr_ctx* ctx, MrPeerX* px);
bool mr_peer_same_device(const mr_ctx* ctx);
unsigned long long mr_peer_timeout_ticks();
// exchanges through the peer regions: areas A (0) and B (1) of every rank's region
bool mr_peer_ready(const mr_ctx* ctx);
int mr_peer_xensure(mr_ctx* ctx, int64_t xa, int64_t xb);    // (collective) area sizes in words
unsigned long long* mr_peer_area(mr_ctx* ctx, int rank, int area);   // rank's area as mapped here
int mr_peer_put(mr_ctx* ctx, const unsigned long long* d_src, int64_t n, int rank, int area, int64_t offset);
int mr_peer_round(mr_ctx* ctx);   // signal every rank, wait until every rank signalled this round
unsigned long long* const* mr_peer_map_dev(mr_ctx* ctx);   // [nranks] device table of the regions
void mr_comm_peer_destroy(mr_ctx* ctx);

// MR_WIN_TIMING diagnostics: wall-clock phase marks (each mark synchronises the stream)
struct PhaseTimer {
    hipStream_t st;
    const char* tag;
    bool on;
    std::vector<std::pair<const char*, double>> marks;
    PhaseTimer(hipStream_t s, const char* t);
    void mark(const char* name);
    ~PhaseTimer();
};

// Launch helpers
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

int mr_graph_prepare(mr_ctx* ctx, mr_graph* g);   // derived arrays + segments after structure upload
// several graphs' prepare in one launch per step when they allow it (keep: host descriptors)
int mr_graph_prepare_batch(mr_ctx* ctx, mr_graph* const* gs, int n, std::vector<unsigned char>& keep);
int mr_graph_post_build(mr_ctx* ctx, mr_graph* g);   // trace-role fields + mr_graph_prepare after K1
// An indexed K1 build between its launches and its size read-back (mr_graph_build.hip): several
// builds (and the detector's counters) share one host round trip.  d_out receives 5 int64 words
// (N, E, overflow, T, nnz); mr_ix_finish takes them (null when b.small is false) and prepares g.
struct IxBuild {
    DBuf<int32_t> tflag, ocnt, ofirst, ocov, node_of_code;
    DBuf<int64_t> tpos, zoff;
    DBuf<uint64_t> gk;
    DBuf<uint32_t> gc;
    uint64_t ecap = 0;
    const uint64_t* gkp = nullptr;   // the edge table's keys: gk (hash table) or the table's ekey (dense ids)
    bool dense = false;              // edge counts per dense edge id (gc[ecap], ecap = n_edge_keys)
    bool small = false;   // the one-block node order ran: its sizes are in d_out
    DBuf<int32_t> pinv;   // layout-order builds (mr_lo_launch_batch): position -> layout index
    uint32_t* kcnt = nullptr;   // ... and the graph's kind-class histogram (caller's zeroed buffer)
};
int mr_ix_launch(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_mask, mr_graph* g, IxBuild& b, int64_t* d_out);
struct DetIn;   // (mr_detect_dev.h)
int mr_ix_launch2(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_state, mr_graph* g0, mr_graph* g1, IxBuild& b0,
                  IxBuild& b1, int64_t* d_out, const DetIn* det = nullptr);
// the same for n <= 8 windows, one launch per stage (det: each window's detector inputs, fused
// into the selection launch when fuse, else launched before it; null: states given)
// A PageRank batch enqueued without its closing read-back (mr_windows_batch keeps one group of
// windows in flight while it enqueues the next): its kernels' descriptors and error words stay
// alive in the handle; finish waits for it and reports a kind-hash collision (rerun with the
// synchronous batch) or an error.  hflag: 4 * ng pinned words.  defer: the error words' copy and
// the finish's event are left for mr_pagerank_async_commit (the caller enqueues work that needs no
// words first -- a single window's spectrum -- so no event sits between it and the iterations)
struct PrAsync;
int mr_pagerank_batch_async(mr_ctx* ctx, mr_graph* const* gs, const int* anomaly, int ng, double d, double alpha,
                            int iters, int precision, int32_t* hflag, PrAsync** out, bool defer = false);
int mr_pagerank_async_commit(mr_ctx* ctx, PrAsync* a);
int mr_pagerank_async_finish(mr_ctx* ctx, PrAsync* a, bool* rerun);
void mr_pagerank_async_free(PrAsync* a);
int mr_ix_launch2_batch(mr_ctx* ctx, int n, const mr_spans* const* sps, uint8_t* const* d_states, mr_graph* const* g0s,
                        mr_graph* const* g1s, IxBuild* const* b0s, IxBuild* const* b1s, int64_t* const* d_outs,
                        const DetIn* dets, bool fuse);
constexpr int MR_DETECT_SHARDS = 64;
int mr_detect_indexed_launch(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* d_a3,
                             const uint8_t* d_a3v, uint8_t* d_state, unsigned long long* counts);
void mr_detect_sum(const unsigned long long* sh, int32_t* n_abn, int32_t* n_nor, int64_t* n_in);
int mr_detect_sweep_launch(mr_ctx* ctx, const mr_spans* s, int64_t t_begin, int64_t grain, int64_t window, int32_t M,
                           const double* d_a3, const uint8_t* d_a3v, uint8_t* d_state, unsigned long long* diff);
// the window spectrum kernel alone, into a device slot of MR_WS_SLOT bytes (codes, scores, count);
// MR_ERR_STATE when the window exceeds the one-block limits
constexpr size_t MR_WS_SLOT = 12 * 256 + 16;
int mr_win_spectrum_launch(mr_ctx* ctx, int32_t Na, const int32_t* a_podop, const double* a_w, const int32_t* a_cov,
                           int32_t Nn, const int32_t* n_podop, const double* n_w, const int32_t* n_cov, int32_t NP,
                           int64_t A, int64_t Nl, int method, int32_t k, unsigned char* d_slot);
void mr_win_spectrum_unpack(const unsigned char* slot, int32_t* out_codes, double* out_score, int32_t* n_out);
// several windows' spectra in one launch (a block each; every window within the one-block limits:
// mr_win_spectrum_fits), at most MR_WS_BATCH per launch
constexpr int MR_WS_BATCH = 8;
struct MrWsWin {
    const int32_t *a_podop, *a_cov, *n_podop, *n_cov;
    const double *a_w, *n_w;
    unsigned char* out;
    int64_t A, Nl;
    int32_t Na, Nn, NP;
};
bool mr_win_spectrum_fits(int32_t Na, int32_t Nn, int32_t NP, int32_t k);
int mr_win_spectrum_launch_n(mr_ctx* ctx, const MrWsWin* ws, int n, int method, int32_t k);
int mr_ix_finish(mr_ctx* ctx, const mr_spans* sp, mr_graph* g, IxBuild& b, const int64_t* h);
// Window graph pairs from the tables' layout order (sp->lo_ok; mr_graph_build.hip k_lo_build_b):
// detector, selection by layout position with the kind histograms, the graphs' per-op and per-edge
// counts, the node pass; d_outs as mr_ix_launch2_batch's (N, E, overflow, T, nnz per graph; words 5
// / 6 of each graph's 8 must be zero: the build's totals), dets[k] the window's detector inputs,
// zw[k] mr_lo_zero_words(sps[k]) zeroed words.  MR_ERR_STATE: a window outside the limits (the
// caller takes mr_ix_launch2_batch)
bool mr_lo_fits(const mr_spans* sp);
// a window-build block (k_lo_build_b) holds at most LO_BT_MAX traces and, past its first trace, at
// most LO_BE pod-op entries: the layout's long traces spread over many blocks
constexpr int32_t LO_BT_MAX = 1024;
constexpr int64_t LO_BE = 12288;
int64_t mr_lo_zero_words(const mr_spans* sp);
int mr_lo_launch_batch(mr_ctx* ctx, int n, const mr_spans* const* sps, mr_graph* const* g0s, mr_graph* const* g1s,
                       IxBuild* const* b0s, IxBuild* const* b1s, int64_t* const* d_outs, const DetIn* dets,
                       uint32_t* const* zw);
// their prepare and PageRank set-up (tiles, ids, kinds, preference, iteration state: pre_ok) in
// four launches; gs[i] built from sps[i / 2] with builds bs[i]
int mr_lo_prepare_batch(mr_ctx* ctx, mr_graph* const* gs, const mr_spans* const* sps, IxBuild* const* bs,
                        const int* anomaly, int n, double d, int precision, std::vector<unsigned char>& keep);
// a graph of mr_ix_launch / mr_ix_launch2 finished WITHOUT its prepare: the caller prepares many
// such graphs together (mr_graph_prepare_batch)
int mr_ix_finish_unprepared(mr_ctx* ctx, const mr_spans* sp, mr_graph* g, IxBuild& b, const int64_t* h);
int mr_pagerank_presetup(mr_ctx* ctx, mr_graph* g, int anomaly, double d, int precision, uint32_t flags);
// mr_pagerank_presetup of n graphs in six launches when all allow the batched set-up (keep: its
// host descriptors, alive until the stream has used them)
int mr_pagerank_presetup_n(mr_ctx* ctx, mr_graph* const* gs, const int* anomaly, int n, double d, int precision,
                           std::vector<unsigned char>& keep);
