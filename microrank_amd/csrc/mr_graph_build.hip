// K1: preprocess_data.get_pagerank_graph (preprocess_data.py:146-171) on gfx950.
//
// From HBM-resident int-coded span columns and a trace mask (the trace_list, :148):
//   1. compact the selected rows, keeping row order (first appearance, T10)
//   2. per row: span counts per trace (len_t, :165) and per pod-op (len_o, :167), first
//      appearance row per pod-op, and the parent join ParentSpanId == spanID over the selected
//      rows regardless of traceID (preprocess_data.py:157-158, T11) -> distinct (parent op, child op) edges with
//      multiplicity (children multiset size, :159).  Hot keys (the root op is in every trace)
//      are aggregated in LDS per block before any global atomic.
//   3. node order: parent ops sorted by name (= code), then the other ops by first appearance
//      (preprocess_data.py:159-163, T10)
//   4. (trace, node) pairs -> stable radix sort -> distinct pairs = trace-major CSR (the
//      op-major side is derived by mr_graph_prepare as tiles); call edges sorted by
//      (child, parent) give P_ss by child.
#include <algorithm>
#include <cstring>
#include <vector>

#include "mr_detect_dev.h"
#include "mr_prim.h"
#include "mr_sort.h"

namespace {
constexpr int BT = 256;
constexpr int LDS_HIST = 8192;     // pod-op histograms in LDS up to this many codes
constexpr int ESET = 1024;         // per-block LDS edge set slots
constexpr uint64_t EMPTY = ~0ull;

__device__ __forceinline__ uint64_t hmix(uint64_t z) {
    z ^= z >> 33;
    z *= 0xff51afd7ed558ccdull;
    z ^= z >> 33;
    z *= 0xc4ceb9fe1a85ec53ull;
    return z ^ (z >> 33);
}

// ---------------------------------------------------------------- spans upload: spanID multimap
__global__ void k_count_codes(const int64_t* span, int64_t S, int32_t* cnt) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S) atomicAdd(&cnt[span[i]], 1);
}
__global__ void k_fill_ids(const int64_t* span, int64_t S, const int64_t* off, int32_t* cur, int32_t* rows) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S) {
        int64_t c = span[i];
        rows[off[c] + atomicAdd(&cur[c], 1)] = (int32_t)i;
    }
}
// rows inside a spanID bucket ascending (buckets hold duplicates only: tiny)
__global__ void k_sort_buckets(const int64_t* off, int64_t n_codes, int32_t* rows) {
    int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_codes) return;
    int64_t a = off[c], b = off[c + 1];
    for (int64_t i = a + 1; i < b; ++i) {
        int32_t v = rows[i];
        int64_t j = i - 1;
        while (j >= a && rows[j] > v) {
            rows[j + 1] = rows[j];
            --j;
        }
        rows[j + 1] = v;
    }
}

// ---------------------------------------------------------------- selection
// rows of masked traces; with a window (ts non-null) also inside it (the window's span_df)
__global__ void k_sel_flags(const int32_t* trace, int64_t S, const uint8_t* mask, const int64_t* ts, const int64_t* te,
                            int64_t t0, int64_t t1, int32_t* flag) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S) flag[i] = (mask[trace[i]] && (!ts || (ts[i] >= t0 && te[i] <= t1))) ? 1 : 0;
}
__global__ void k_compact_rows(const int32_t* flag, const int64_t* pos, int64_t S, int32_t* rows) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S && flag[i]) rows[pos[i]] = (int32_t)i;
}

// ---------------------------------------------------------------- per-row statistics + join
__device__ __forceinline__ void global_edge_add(uint64_t key, uint32_t c, uint64_t* gk, uint32_t* gc, uint64_t gmask) {
    uint64_t s = hmix(key) & gmask;
    for (;;) {
        unsigned long long k = atomicCAS((unsigned long long*)&gk[s], (unsigned long long)EMPTY, (unsigned long long)key);
        if (k == EMPTY || k == key) break;
        s = (s + 1) & gmask;
    }
    atomicAdd(&gc[s], c);
}

__global__ void __launch_bounds__(BT) k_rows(const int32_t* rows, int64_t Ssel, const int32_t* trace,
                                             const int32_t* podop, const int64_t* parent, const int32_t* selflag,
                                             const int64_t* id_off, const int32_t* id_rows, int64_t n_codes,
                                             int32_t n_podops, int use_lds_hist, int32_t* tcnt, int32_t* ocnt,
                                             int32_t* ofirst, uint64_t* gk, uint32_t* gc, uint64_t gmask) {
    extern __shared__ int32_t lh[];   // [2*n_podops] counts, first rows (when use_lds_hist)
    __shared__ unsigned long long ek[ESET];
    __shared__ uint32_t ec[ESET];
    int32_t* lcnt = lh;
    int32_t* lfirst = lh + n_podops;
    if (use_lds_hist)
        for (int32_t i = threadIdx.x; i < n_podops; i += BT) {
            lcnt[i] = 0;
            lfirst[i] = 0x7fffffff;
        }
    for (int i = threadIdx.x; i < ESET; i += BT) {
        ek[i] = EMPTY;
        ec[i] = 0;
    }
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * BT * 8;
    for (int c = 0; c < 8; ++c) {
        const int64_t li = base + (int64_t)c * BT + threadIdx.x;   // local (selected) row index
        if (li >= Ssel) break;
        const int32_t r = rows[li];
        const int32_t op = podop[r];
        atomicAdd(&tcnt[trace[r]], 1);
        if (use_lds_hist) {
            atomicAdd(&lcnt[op], 1);
            atomicMin(&lfirst[op], (int32_t)li);
        } else {
            atomicAdd(&ocnt[op], 1);
            atomicMin(&ofirst[op], (int32_t)li);
        }
        const int64_t p = parent[r];
        if (p < 0 || p >= n_codes) continue;
        for (int64_t e = id_off[p]; e < id_off[p + 1]; ++e) {
            const int32_t j = id_rows[e];
            if (!selflag[j]) continue;
            const uint64_t key = ((uint64_t)(uint32_t)podop[j] << 32) | (uint32_t)op;   // (parent, child)
            uint32_t s = (uint32_t)(hmix(key) & (ESET - 1));
            bool done = false;
            for (int probe = 0; probe < 32; ++probe) {
                unsigned long long k = atomicCAS(&ek[s], (unsigned long long)EMPTY, (unsigned long long)key);
                if (k == EMPTY || k == key) {
                    atomicAdd(&ec[s], 1u);
                    done = true;
                    break;
                }
                s = (s + 1) & (ESET - 1);
            }
            if (!done) global_edge_add(key, 1u, gk, gc, gmask);   // LDS set crowded: go global
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < ESET; i += BT)
        if (ek[i] != EMPTY) global_edge_add(ek[i], ec[i], gk, gc, gmask);
    if (use_lds_hist)
        for (int32_t i = threadIdx.x; i < n_podops; i += BT)
            if (lcnt[i]) {
                atomicAdd(&ocnt[i], lcnt[i]);
                atomicMin(&ofirst[i], lfirst[i]);
            }
}

// ---------------------------------------------------------------- node order
// a slot holds an edge when its key is set and counted (the dense form lists every key of the
// table, counted or not)
__global__ void k_edge_flags(const uint64_t* gk, const uint32_t* gc, int64_t cap, int32_t* flag) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap) flag[i] = gk[i] != EMPTY && gc[i] != 0u;
}
__global__ void k_edge_compact(const uint64_t* gk, const uint32_t* gc, const int32_t* flag, const int64_t* pos,
                               int64_t cap, uint64_t* ekey, uint32_t* ecnt, int32_t* is_par, int32_t* nchild_code) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap || !flag[i]) return;
    const uint64_t k = gk[i];
    ekey[pos[i]] = k;
    ecnt[pos[i]] = gc[i];
    const int32_t par = (int32_t)(k >> 32);
    is_par[par] = 1;
    atomicAdd(&nchild_code[par], (int32_t)gc[i]);
}
// flags: parent codes (sorted by code) and present non-parents keyed by first row
__global__ void k_node_flags(const int32_t* ocnt, const int32_t* is_par, int32_t n, int32_t* pflag, int32_t* qflag) {
    int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    pflag[c] = is_par[c] ? 1 : 0;
    qflag[c] = (ocnt[c] > 0 && !is_par[c]) ? 1 : 0;
}
__global__ void k_node_parents(const int32_t* pflag, const int64_t* ppos, const int32_t* qflag, const int64_t* qpos,
                               const int32_t* ofirst, int32_t n, int32_t* node_of_code, int32_t* node_podop,
                               uint64_t* qkey, uint32_t* qval) {
    int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    if (pflag[c]) {
        node_of_code[c] = (int32_t)ppos[c];
        node_podop[ppos[c]] = c;
    }
    if (qflag[c]) {
        qkey[qpos[c]] = (uint64_t)(uint32_t)ofirst[c];
        qval[qpos[c]] = (uint32_t)c;
    }
}
__global__ void k_node_rest(const uint32_t* qval, int64_t nq, int32_t P, int32_t* node_of_code, int32_t* node_podop) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const int32_t c = (int32_t)qval[i];
    node_of_code[c] = P + (int32_t)i;
    node_podop[P + i] = c;
}

// ---------------------------------------------------------------- traces
__global__ void k_trace_flags(const int32_t* tcnt, int32_t n, int32_t* flag) {
    int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n) flag[c] = tcnt[c] > 0;
}
__global__ void k_trace_index(const int32_t* flag, const int64_t* pos, const int32_t* tcnt, int32_t n,
                              int32_t* tidx_of_code, int32_t* trace_code, int32_t* len_t) {
    int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n || !flag[c]) return;
    const int32_t t = (int32_t)pos[c];
    tidx_of_code[c] = t;
    trace_code[t] = c;
    len_t[t] = tcnt[c];
}

// ---------------------------------------------------------------- pairs
__global__ void k_pair_keys(const int32_t* rows, int64_t Ssel, const int32_t* trace, const int32_t* podop,
                            const int32_t* tidx_of_code, const int32_t* node_of_code, int nb, uint64_t* keys) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Ssel) return;
    const int32_t r = rows[i];
    keys[i] = ((uint64_t)(uint32_t)tidx_of_code[trace[r]] << nb) | (uint32_t)node_of_code[podop[r]];
}
__global__ void k_run_heads(const uint64_t* keys, int64_t n, int32_t* flag) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}
// distinct pairs in (trace, node) order; every present trace has >= 1 pair, so its CSR offset is
// the position of its first pair (no per-trace counting atomics)
__global__ void k_pairs_out(const uint64_t* keys, const int32_t* flag, const int64_t* pos, int64_t n, int nb,
                            int64_t* rs_off, int32_t* rs_ops) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const uint64_t k = keys[i];
    const uint32_t t = (uint32_t)(k >> nb);
    const int64_t e = pos[i];
    rs_ops[e] = (int32_t)(k & ((1ull << nb) - 1));
    if (i == 0 || (keys[i - 1] >> nb) != t) rs_off[t] = e;
}
__global__ void k_set_last(int64_t* off, int32_t n, int64_t v) { off[n] = v; }

// ---------------------------------------------------------------- per-node arrays
__global__ void k_node_arrays(const int32_t* node_podop, int32_t N, const int32_t* ocnt, const int32_t* nchild_code,
                              const int32_t* ocov, int32_t* len_o, int32_t* nchild, int32_t* cov) {
    int32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const int32_t c = node_podop[n];
    len_o[n] = ocnt[c];
    nchild[n] = nchild_code[c];
    if (ocov) cov[n] = ocov[c];
}
__global__ void k_edge_nodes(const uint64_t* ekey, int64_t E, const int32_t* node_of_code, int nb, uint64_t* skey) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E) return;
    const uint64_t k = ekey[i];
    const uint32_t par = (uint32_t)node_of_code[(int32_t)(k >> 32)];
    const uint32_t ch = (uint32_t)node_of_code[(int32_t)(k & 0xffffffffu)];
    skey[i] = ((uint64_t)ch << nb) | par;    // sort by (child, parent)
}
__global__ void k_edge_csr(const uint64_t* skey, int64_t E, int nb, int32_t* ss_par, int32_t* ccount) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E) return;
    ss_par[i] = (int32_t)(skey[i] & ((1ull << nb) - 1));
    atomicAdd(&ccount[skey[i] >> nb], 1);
}

// ---------------------------------------------------------------- node order of a window graph, one block
// Windows (C2/C3: up to a few thousand pod-ops and call edges) take the whole of build_nodes in
// ONE single-block launch -- edges out of the hash table, parent flags and child counts, the
// node order (parents by code, the rest by first row, T10), per-node arrays, and P_ss by child --
// instead of ~15 launches and two host round trips.  Sizes go to `out` (N, E, overflow); a graph
// with more than NS_EMAX edges sets overflow and the caller runs build_nodes instead.
constexpr int NS_T = 1024, NS_PMAX = 4096, NS_EMAX = 8192;
static_assert(NS_EMAX <= 2 * NS_PMAX, "nodes_small: the CSR parents reuse the 64-bit key buffer");
__device__ __forceinline__ void ns_bitonic(uint64_t* a, int n) {   // n a power of two
    for (int k = 2; k <= n; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += NS_T) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t x = a[i], y = a[ixj];
                    if ((x > y) == ((i & k) == 0)) {
                        a[i] = y;
                        a[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
}
// exclusive prefix of v over the block's threads (in thread order); total in *tot
__device__ __forceinline__ int32_t ns_scan(int32_t v, int32_t* sbuf, int32_t* tot) {
    sbuf[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < NS_T; o <<= 1) {
        const int32_t a = threadIdx.x >= o ? sbuf[threadIdx.x - o] : 0;
        __syncthreads();
        sbuf[threadIdx.x] += a;
        __syncthreads();
    }
    const int32_t incl = sbuf[threadIdx.x];
    if (threadIdx.x == NS_T - 1) *tot = incl;
    __syncthreads();
    return incl - v;
}
__device__ void nodes_small(const uint64_t* gk, const uint32_t* gc, int64_t ecap, const int32_t* ocnt,
                            const int32_t* ofirst, int32_t NP, int32_t* node_of_code, int32_t* node_podop,
                            int32_t* len_o, int32_t* nchild, const int32_t* ocov, int32_t* cov, int32_t* ss_par,
                            int64_t* ss_off, const int64_t* T_dev, const int64_t* nnz_dev, int64_t* rs_off,
                            int64_t* out, float* u_o = nullptr, float* pw = nullptr, bool first_inv = false) {
    __shared__ int32_t is_par[NS_PMAX], nch[NS_PMAX], noc[NS_PMAX];
    __shared__ uint64_t qb[NS_PMAX], eb[NS_EMAX];
    __shared__ int32_t sbuf[NS_T];
    __shared__ int32_t ecount, tot, P, Q;
    const int tid = threadIdx.x;
    for (int c = tid; c < NP; c += NS_T) {
        is_par[c] = 0;
        nch[c] = 0;
    }
    if (tid == 0) ecount = 0;
    __syncthreads();
    // call edges out of the hash table (parent code << 32 | child code): parents and child counts
    for (int64_t i = tid; i < ecap; i += NS_T) {
        const uint64_t k = gk[i];
        if (k == EMPTY || gc[i] == 0u) continue;   // (dense ids: a key of the table not in this graph)
        const int32_t par = (int32_t)(k >> 32);
        is_par[par] = 1;
        atomicAdd(&nch[par], (int32_t)gc[i]);
        const int32_t e = atomicAdd(&ecount, 1);
        if (e < NS_EMAX) eb[e] = k;
    }
    __syncthreads();
    const int32_t E = ecount;
    if (tid == 0) {   // the trace side's sizes (its scans ran before this launch)
        out[3] = *T_dev;
        out[4] = *nnz_dev;
        if (rs_off) rs_off[*T_dev] = *nnz_dev;
    }
    if (E > NS_EMAX) {
        if (tid == 0) out[2] = 1;
        return;
    }
    // node order: parents by code, then present non-parents by first row (T10)
    const int per = (NP + NS_T - 1) / NS_T, c0 = tid * per;   // each thread a run of codes
    int32_t np = 0, nq = 0;
    for (int c = c0; c < min(c0 + per, NP); ++c) {
        np += is_par[c] ? 1 : 0;
        nq += (!is_par[c] && ocnt[c] > 0) ? 1 : 0;
    }
    int32_t pp = ns_scan(np, sbuf, &tot);
    if (tid == 0) P = tot;
    __syncthreads();
    int32_t qp = ns_scan(nq, sbuf, &tot);
    if (tid == 0) Q = tot;
    __syncthreads();
    const int32_t nP = P, nQ = Q;
    for (int c = c0; c < min(c0 + per, NP); ++c) {
        if (is_par[c]) {
            noc[c] = pp;
            node_podop[pp] = c;
            ++pp;
        } else if (ocnt[c] > 0) {
            // (first_inv: the layout-order build keeps INT_MAX - first row, max-reduced)
            const int32_t fr = first_inv ? 0x7fffffff - ofirst[c] : ofirst[c];
            qb[qp++] = ((uint64_t)(uint32_t)fr << 32) | (uint32_t)c;
        }
    }
    __syncthreads();
    if (nQ <= NS_T) {   // rank of each (distinct) key by counting: one pass, no sorting network
        if (tid < nQ) {
            const uint64_t key = qb[tid];
            int32_t r = 0;
            for (int j = 0; j < nQ; ++j) r += qb[j] < key;
            const int32_t c = (int32_t)(key & 0xffffffffu);
            noc[c] = nP + r;
            node_podop[nP + r] = c;
        }
    } else {
        int qn = 1;
        while (qn < nQ) qn <<= 1;
        for (int i = nQ + tid; i < qn; i += NS_T) qb[i] = EMPTY;
        __syncthreads();
        ns_bitonic(qb, qn);
        for (int i = tid; i < nQ; i += NS_T) {
            const int32_t c = (int32_t)(qb[i] & 0xffffffffu);
            noc[c] = nP + i;
            node_podop[nP + i] = c;
        }
    }
    __syncthreads();
    const int32_t N = nP + nQ;
    for (int c = tid; c < NP; c += NS_T) node_of_code[c] = (is_par[c] || ocnt[c] > 0) ? noc[c] : -1;
    for (int c = c0; c < min(c0 + per, NP); ++c)   // per-node arrays (node_podop's writes are this block's)
        if (is_par[c] || ocnt[c] > 0) {
            len_o[noc[c]] = ocnt[c];
            nchild[noc[c]] = nch[c];
            cov[noc[c]] = ocov[c];
            if (u_o) {   // (layout-order builds: graph_consts' fp32 reciprocals, pagerank.py:39-52)
                u_o[noc[c]] = ocnt[c] > 0 ? (float)(1.0 / (double)ocnt[c]) : 0.0f;
                pw[noc[c]] = nch[c] > 0 ? (float)(1.0 / (double)nch[c]) : 0.0f;
            }
        }
    // P_ss by child (edges sorted by (child node, parent node)): a counting sort by child into
    // the CSR, then each child's few parents sorted in place.  (is_par / nch / qb are free now.)
    __syncthreads();
    int32_t* ccnt = nch;           // edges per child node
    int32_t* cpos = is_par;        // running insert position per child node
    int32_t* cpar = (int32_t*)qb;  // parents in CSR order (NS_EMAX <= 2 NS_PMAX slots)
    for (int n = tid; n < N; n += NS_T) ccnt[n] = 0;
    __syncthreads();
    for (int e = tid; e < E; e += NS_T) {
        const uint64_t k = eb[e];
        const int32_t ch = noc[(int32_t)(k & 0xffffffffu)];
        eb[e] = ((uint64_t)(uint32_t)ch << 32) | (uint32_t)noc[(int32_t)(k >> 32)];
        atomicAdd(&ccnt[ch], 1);
    }
    __syncthreads();
    {
        const int perN = (N + NS_T - 1) / NS_T, n0 = tid * perN;
        int32_t run = 0;
        for (int n = n0; n < min(n0 + perN, N); ++n) run += ccnt[n];
        int32_t off = ns_scan(run, sbuf, &tot);
        for (int n = n0; n < min(n0 + perN, N); ++n) {
            cpos[n] = off;
            ss_off[n] = off;
            off += ccnt[n];
        }
        if (tid == 0) ss_off[N] = E;
    }
    __syncthreads();
    for (int e = tid; e < E; e += NS_T) {
        const uint64_t k = eb[e];
        cpar[atomicAdd(&cpos[(int32_t)(k >> 32)], 1)] = (int32_t)(k & 0xffffffffu);
    }
    __syncthreads();
    for (int n = tid; n < N; n += NS_T) {   // cpos[n] is now the end of child n's run
        const int32_t b = cpos[n], a = b - ccnt[n];
        for (int32_t i = a + 1; i < b; ++i) {   // insertion sort: runs are a child's few parents
            const int32_t v = cpar[i];
            int32_t j = i - 1;
            while (j >= a && cpar[j] > v) {
                cpar[j + 1] = cpar[j];
                --j;
            }
            cpar[j + 1] = v;
        }
    }
    __syncthreads();
    for (int e = tid; e < E; e += NS_T) ss_par[e] = cpar[e];
    if (tid == 0) {
        out[0] = N;
        out[1] = E;
        out[2] = 0;
    }
}
__global__ void __launch_bounds__(NS_T) k_nodes_small(const uint64_t* gk, const uint32_t* gc, int64_t ecap,
                                                     const int32_t* ocnt, const int32_t* ofirst, int32_t NP,
                                                     int32_t* node_of_code, int32_t* node_podop, int32_t* len_o,
                                                     int32_t* nchild, const int32_t* ocov, int32_t* cov,
                                                     int32_t* ss_par, int64_t* ss_off, const int64_t* T_dev,
                                                     const int64_t* nnz_dev, int64_t* rs_off, int64_t* out) {
    nodes_small(gk, gc, ecap, ocnt, ofirst, NP, node_of_code, node_podop, len_o, nchild, ocov, cov, ss_par, ss_off,
                T_dev, nnz_dev, rs_off, out);
}
// the two graphs of a window (mr_ix_launch2): block g builds graph g
struct NsArgs {
    const uint32_t* gc;
    const int32_t *ocnt, *ofirst, *ocov;
    int32_t *node_of_code, *node_podop, *len_o, *nchild, *cov, *ss_par;
    int64_t* ss_off;
    const int64_t *T_dev, *nnz_dev;
    int64_t *rs_off, *out;
    float *u_o, *pw;   // (layout-order builds; else null)
    int32_t first_inv;  // (layout-order builds: ofirst holds INT_MAX - first row)
};
struct NsArgs2 {
    NsArgs g[2];
};
__global__ void __launch_bounds__(NS_T) k_nodes_small2(const uint64_t* gk, int64_t ecap, int32_t NP, NsArgs2 a) {
    const NsArgs& x = a.g[blockIdx.x];
    nodes_small(gk, x.gc, ecap, x.ocnt, x.ofirst, NP, x.node_of_code, x.node_podop, x.len_o, x.nchild, x.ocov, x.cov,
                x.ss_par, x.ss_off, x.T_dev, x.nnz_dev, x.rs_off, x.out);
}

// ---------------------------------------------------------------- indexed build (whole traces)
constexpr int IX_EPT = 16;  // index entries per thread in k_ix_stats (fewer blocks: fewer global flushes)
// ... and in the window batches' k_ix_stats2_b for windows of >= IX_EPT_BIG index entries (C2's
// 2.3M, 256 windows per call: 16 / 64 -> 5752-5799 / 5926-5996 windows/s, profiles/r04ag); small
// windows (C3's 400k) keep 16: their blocks are few already
constexpr int IX_EPT_BATCH = 64;
constexpr int64_t IX_EPT_BIG = (int64_t)1 << 20;
// k_ix_stats: 16-wave blocks (one per CU) whose LDS holds the per-pod-op counts and first rows
// of up to IX_HIST codes (128 KB) beside the edge set: the C4 graph's 10k ops aggregate in LDS
// instead of a global atomic pair per index entry
constexpr int IX_BT = 1024;
constexpr int IX_HIST = 12288;   // three per-code counters (span count, first row, traces)
constexpr int IX_B = 8;     // entries per thread whose loads are batched
constexpr int64_t IX_LDS_WORDS = 36864;   // k_ix_stats' dynamic LDS budget (144 KB) in 4-B words
// The indexed build's first launch: the trace selection with BOTH exclusive scans -- tpos over
// the selection flags, zoff over the selected traces' op-list lengths -- chained across tiles by
// decoupled look-back (two status chains), plus the clearing of the per-code counters and the
// edge hash (a grid-stride share per block): one launch where there were four.
constexpr int SEL_T = 256, SEL_I = 8, SEL_TILE = SEL_T * SEL_I;
static_assert(SEL_T == 4 * WAVE, "k_ix_sel_scan2: one wave per look-back chain");
__global__ void __launch_bounds__(SEL_T) k_ix_sel_scan(const uint8_t* mask, const int32_t* tlen, const int64_t* po_off,
                                                      int32_t NT, int32_t* tflag, int64_t* tpos, int64_t* zoff,
                                                      unsigned long long* st, uint64_t epoch, int32_t* ocnt,
                                                      int32_t* ofirst, int32_t* ocov, int32_t NP, uint64_t* gk,
                                                      uint32_t* gc, int64_t ecap) {
    __shared__ int64_t sa[SEL_T], sb[SEL_T];
    __shared__ int64_t ex[2];
    const int tid = threadIdx.x;
    const int64_t gsz = (int64_t)gridDim.x * SEL_T, gi = (int64_t)blockIdx.x * SEL_T + tid;
    for (int64_t i = gi; i < max((int64_t)NP, ecap); i += gsz) {
        if (i < NP) {
            ocnt[i] = 0;
            ofirst[i] = 0x7f7f7f7f;   // larger than any row
            ocov[i] = 0;
        }
        if (i < ecap) {
            if (gk) gk[i] = ~0ull;
            gc[i] = 0u;
        }
    }
    const int64_t tile = blockIdx.x, base = tile * SEL_TILE + (int64_t)tid * SEL_I;
    int32_t f[SEL_I];
    int64_t z[SEL_I], a = 0, b = 0;
#pragma unroll
    for (int i = 0; i < SEL_I; ++i) {
        const int64_t t = base + i;
        const bool on = t < NT && mask[t] && tlen[t] > 0;
        f[i] = on ? 1 : 0;
        z[i] = on ? po_off[t + 1] - po_off[t] : 0;
        if (t < NT) tflag[t] = f[i];
        a += f[i];
        b += z[i];
    }
    sa[tid] = a;
    sb[tid] = b;
    __syncthreads();
    for (int o = 1; o < SEL_T; o <<= 1) {
        const int64_t x = tid >= o ? sa[tid - o] : 0, y = tid >= o ? sb[tid - o] : 0;
        __syncthreads();
        sa[tid] += x;
        sb[tid] += y;
        __syncthreads();
    }
    if (tid < 2 * WAVE) {   // wave c: chain c
        const int c = tid / WAVE;
        const int64_t agg = c ? sb[SEL_T - 1] : sa[SEL_T - 1];
        const int64_t e = dl_lookback_wave(st + (size_t)c * gridDim.x, tile, agg, epoch);
        if ((tid & (WAVE - 1)) == 0) {
            ex[c] = e;
            if (tile == (int64_t)gridDim.x - 1) (c ? zoff : tpos)[NT] = e + agg;
        }
    }
    __syncthreads();
    int64_t ra = ex[0] + sa[tid] - a, rb = ex[1] + sb[tid] - b;
#pragma unroll
    for (int i = 0; i < SEL_I; ++i) {
        const int64_t t = base + i;
        if (t < NT) {
            tpos[t] = ra;
            zoff[t] = rb;
        }
        ra += f[i];
        rb += z[i];
    }
}
// Wide op spaces (more pod-op codes than one LDS histogram): the selected index entries of share b
// (the same 1/nblk shares k_ix_stats takes) grouped by op range of IX_HIST codes into out[p0, p1):
// a counting pass, then a scatter through wave-aggregated LDS cursors; tab[b (R + 1) + r] = the
// offset of range r in the share.  Each range's k_ix_stats blocks then read only their entries,
// once, instead of every range reading (and flag-checking) the whole index.
constexpr int IX_RMAX = 64;   // op ranges the grouping takes (786k codes)
__global__ void __launch_bounds__(IX_BT) k_ix_rpart(const int32_t* tflag, int64_t n_po, const int32_t* po_tr,
                                                 const int32_t* po_op, const int32_t* po_cnt, const int32_t* po_first,
                                                 int32_t nrange, int4* out, int32_t* tab) {
    __shared__ int32_t cnt[IX_RMAX], cur[IX_RMAX];
    const int32_t tid = (int32_t)threadIdx.x, lane = tid & (WAVE - 1);
    const int64_t pper = (n_po + gridDim.x - 1) / gridDim.x, p0 = (int64_t)blockIdx.x * pper, p1 = min(p0 + pper, n_po);
    if (tid < IX_RMAX) cnt[tid] = 0;
    __syncthreads();
    for (int64_t rb = p0; rb < p1; rb += IX_BT) {   // counts per range (a ballot per range present)
        const int64_t r = rb + tid;
        int32_t g = -1;
        if (r < p1 && tflag[po_tr[r]]) g = po_op[r] / IX_HIST;
        for (uint64_t todo = __ballot(g >= 0); todo;) {
            const int32_t q = __builtin_amdgcn_readlane(g, __ffsll((unsigned long long)todo) - 1);
            const uint64_t m = __ballot(g == q);
            if (lane == 0) atomicAdd(&cnt[q], __popcll(m));
            todo &= ~m;
        }
    }
    __syncthreads();
    if (tid == 0) {
        int32_t a = 0;
        int32_t* tb = tab + (size_t)blockIdx.x * (nrange + 1);
        for (int q = 0; q < nrange; ++q) {
            cur[q] = a;
            tb[q] = a;
            a += cnt[q];
        }
        tb[nrange] = a;
    }
    __syncthreads();
    for (int64_t rb = p0; rb < p1; rb += IX_BT) {   // the scatter: one cursor add per range present
        const int64_t r = rb + tid;
        int32_t g = -1, op = 0, c = 0, f = 0;
        if (r < p1 && tflag[po_tr[r]]) {
            op = po_op[r];
            c = po_cnt[r];
            f = po_first[r];
            g = op / IX_HIST;
        }
        for (uint64_t todo = __ballot(g >= 0); todo;) {
            const int ld = __ffsll((unsigned long long)todo) - 1;
            const int32_t q = __builtin_amdgcn_readlane(g, ld);
            const uint64_t m = __ballot(g == q);
            int32_t base = 0;
            if (lane == ld) base = atomicAdd(&cur[q], __popcll(m));
            base = __builtin_amdgcn_readlane(base, ld);
            if (g == q) {
                const int32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                out[p0 + base + k] = make_int4(op - q * IX_HIST, c, f, 0);
            }
            todo &= ~m;
        }
    }
}
// entry-parallel over the index: span counts and first rows per pod-op of the selected traces
// (LDS-aggregated per block), and their join keys with multiplicity into the block's LDS edge
// set (hot keys aggregated before global atomics).  Block b takes a 1/gridDim share of each list.
__global__ void __launch_bounds__(IX_BT) k_ix_stats(const int32_t* tflag, int64_t n_po, const int32_t* po_tr,
                                                 const int32_t* po_op, const int32_t* po_cnt, const int32_t* po_first,
                                                 int64_t n_ed, const int32_t* ed_tr, const uint64_t* ed_key,
                                                 const int32_t* ed_cnt, int32_t n_podops, int use_lds_hist,
                                                 int32_t* ocnt, int32_t* ofirst, int32_t* ocov, uint64_t* gk,
                                                 uint32_t* gc, uint64_t gmask, const int32_t* ed_eid, int32_t n_ek,
                                                 int lds_ek, const int4* rent, const int32_t* rtab, int32_t nshare) {
    extern __shared__ int32_t lh[];
    __shared__ unsigned long long ek[ESET];
    __shared__ uint32_t ec[ESET];
    // more pod-op codes than one LDS histogram holds (wide op spaces, C5's 100k ops): blockIdx.x is an
    // op range of IX_HIST codes whose entries this block counts in LDS (the range's blocks share the
    // index: each reads its share of every entry and keeps those of its range); range 0 also takes
    // the join keys.  Was: three global atomics per entry at up to 10^5 codes.  blockIdx.y is the
    // share of the index.  rent: the share's selected entries grouped by range (k_ix_rpart) -- the
    // block reads only its range's.
    const int32_t rng = (int32_t)blockIdx.x, chunk = (int32_t)blockIdx.y, nchunk = (int32_t)gridDim.y;
    const int32_t op_lo = rng * IX_HIST;
    const bool ranged = gridDim.x > 1;
    const int32_t NPL = ranged ? min(IX_HIST, n_podops - op_lo) : n_podops;   // this block's codes
    n_podops = NPL;
    int32_t* lcnt = lh;
    int32_t* lfirst = lh + n_podops;
    int32_t* lcov = lh + 2 * n_podops;   // traces per pod-op (the graph's coverage)
    uint32_t* lec = (uint32_t*)(lh + (use_lds_hist ? 3 * n_podops : 0));   // dense edge ids: counts per id
    if (use_lds_hist)
        for (int32_t i = threadIdx.x; i < n_podops; i += IX_BT) {
            lcnt[i] = 0;
            lfirst[i] = 0x7fffffff;
            lcov[i] = 0;
        }
    if (ed_eid && lds_ek)
        for (int32_t i = threadIdx.x; i < n_ek; i += IX_BT) lec[i] = 0u;
    else if (!ed_eid)
        for (int i = threadIdx.x; i < ESET; i += IX_BT) {
            ek[i] = EMPTY;
            ec[i] = 0;
        }
    __syncthreads();
    const int64_t pper = (n_po + nchunk - 1) / nchunk, eper = (n_ed + nchunk - 1) / nchunk;
    // a round of IX_B entries per thread: its trace-flag gathers go out, then the NEXT round's loads,
    // then this round's atomics (the flags' wait leaves the younger loads in flight)
    const int64_t p0 = (int64_t)chunk * pper, p1 = min(p0 + pper, n_po);
    int32_t tr[IX_B], op[IX_B], cn[IX_B], fr[IX_B];
    auto po_load = [&](int64_t rb) {
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            const int64_t r = min(rb + threadIdx.x + (int64_t)j * IX_BT, p1 - 1);
            tr[j] = po_tr[r];
            op[j] = po_op[r];
            cn[j] = po_cnt[r];
            fr[j] = po_first[r];
        }
    };
    // (ranged: LDS histograms; this block's chunk = rpart's shares [s0, s1))
    const int32_t s0 = rent ? (int32_t)((int64_t)chunk * nshare / nchunk) : 0;
    const int32_t s1 = rent ? (int32_t)((int64_t)(chunk + 1) * nshare / nchunk) : 0;
    const int64_t sper = rent ? (n_po + nshare - 1) / nshare : 0;
    for (int32_t sh = s0; sh < s1; ++sh) {
        const int32_t* tb = rtab + (size_t)sh * (gridDim.x + 1);
        const int64_t e0 = sh * sper + tb[rng], e1 = sh * sper + tb[rng + 1];
        for (int64_t rb = e0; rb < e1; rb += (int64_t)IX_BT * IX_B) {
            int4 v[IX_B];
#pragma unroll
            for (int j = 0; j < IX_B; ++j) v[j] = rent[min(rb + threadIdx.x + (int64_t)j * IX_BT, e1 - 1)];
#pragma unroll
            for (int j = 0; j < IX_B; ++j) {
                if (rb + threadIdx.x + (int64_t)j * IX_BT >= e1) continue;
                atomicAdd(&lcnt[v[j].x], v[j].y);
                atomicMin(&lfirst[v[j].x], v[j].z);
                atomicAdd(&lcov[v[j].x], 1);
            }
        }
    }
    if (!rent && p0 < p1) po_load(p0);
    for (int64_t rb = p0; !rent && rb < p1; rb += (int64_t)IX_BT * IX_B) {
        int32_t fl[IX_B], cop[IX_B], ccn[IX_B], cfr[IX_B];
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            fl[j] = tflag[tr[j]];
            cop[j] = op[j] - op_lo;   // (0 unless ranged)
            ccn[j] = cn[j];
            cfr[j] = fr[j];
        }
        if (rb + (int64_t)IX_BT * IX_B < p1) po_load(rb + (int64_t)IX_BT * IX_B);
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            if (!(rb + threadIdx.x + (int64_t)j * IX_BT < p1 && (!ranged || (uint32_t)cop[j] < (uint32_t)NPL) && fl[j]))
                continue;
            if (use_lds_hist) {
                atomicAdd(&lcnt[cop[j]], ccn[j]);
                atomicMin(&lfirst[cop[j]], cfr[j]);
                atomicAdd(&lcov[cop[j]], 1);
            } else {
                atomicAdd(&ocnt[cop[j]], ccn[j]);
                atomicMin(&ofirst[cop[j]], cfr[j]);
                atomicAdd(&ocov[cop[j]], 1);
            }
        }
    }
    const int64_t q0 = (int64_t)chunk * eper, q1 = rng ? q0 : min(q0 + eper, n_ed);   // (range 0: the keys)
    if (ed_eid) {   // dense edge ids: one counter add per selected entry
        for (int64_t rb = q0; rb < q1; rb += (int64_t)IX_BT * IX_B) {
            int32_t tr[IX_B], cn[IX_B], id[IX_B];
#pragma unroll
            for (int j = 0; j < IX_B; ++j) {
                const int64_t r = min(rb + threadIdx.x + (int64_t)j * IX_BT, q1 - 1);
                tr[j] = ed_tr[r];
                id[j] = ed_eid[r];
                cn[j] = ed_cnt[r];
            }
#pragma unroll
            for (int j = 0; j < IX_B; ++j)
                if (rb + threadIdx.x + (int64_t)j * IX_BT < q1 && tflag[tr[j]]) {
                    if (lds_ek) atomicAdd(&lec[id[j]], (uint32_t)cn[j]);
                    else atomicAdd(&gc[id[j]], (uint32_t)cn[j]);
                }
        }
        __syncthreads();
        if (lds_ek)
            for (int32_t i = threadIdx.x; i < n_ek; i += IX_BT)
                if (lec[i]) atomicAdd(&gc[i], lec[i]);
        if (use_lds_hist)
            for (int32_t i = threadIdx.x; i < n_podops; i += IX_BT)
                if (lcnt[i]) {
                    atomicAdd(&ocnt[op_lo + i], lcnt[i]);
                    atomicMin(&ofirst[op_lo + i], lfirst[i]);
                    atomicAdd(&ocov[op_lo + i], lcov[i]);
                }
        return;
    }
    for (int64_t rb = q0; rb < q1; rb += (int64_t)IX_BT * IX_B) {
        int32_t tr[IX_B], cn[IX_B];
        uint64_t ky[IX_B];
        bool on[IX_B];
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            const int64_t r = min(rb + threadIdx.x + (int64_t)j * IX_BT, q1 - 1);
            tr[j] = ed_tr[r];
            ky[j] = ed_key[r];
            cn[j] = ed_cnt[r];
        }
#pragma unroll
        for (int j = 0; j < IX_B; ++j) on[j] = rb + threadIdx.x + (int64_t)j * IX_BT < q1 && tflag[tr[j]];
        for (int j = 0; j < IX_B; ++j) {
            if (!on[j]) continue;
            const uint64_t key = ky[j];
            uint32_t s = (uint32_t)(hmix(key) & (ESET - 1));
            bool done = false;
            for (int probe = 0; probe < 32; ++probe) {
                unsigned long long kk = atomicCAS(&ek[s], (unsigned long long)EMPTY, (unsigned long long)key);
                if (kk == EMPTY || kk == key) {
                    atomicAdd(&ec[s], (uint32_t)cn[j]);
                    done = true;
                    break;
                }
                s = (s + 1) & (ESET - 1);
            }
            if (!done) global_edge_add(key, (uint32_t)cn[j], gk, gc, gmask);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < ESET; i += IX_BT)
        if (ek[i] != EMPTY) global_edge_add(ek[i], ec[i], gk, gc, gmask);
    if (use_lds_hist)
        for (int32_t i = threadIdx.x; i < n_podops; i += IX_BT)
            if (lcnt[i]) {
                atomicAdd(&ocnt[op_lo + i], lcnt[i]);
                atomicMin(&ofirst[op_lo + i], lfirst[i]);
                atomicAdd(&ocov[op_lo + i], lcov[i]);
            }
}
// Edges counted in edge-id order (mr_spans.eb_*, large tables): a lane per entry, the wave's runs
// of one id summed by a segmented scan (ids ascend along the wave), a wave walking EC_CH chunks
// with the last run's sum carried from chunk to chunk, one add per run into cnt[id] -- in place of
// an atomic (or a hash probe) per entry, and a hot id (millions of entries) takes one add per
// 2048 entries, not per 64.  The selection is read from a
// bitmap of the traces (NT / 8 bytes: the gathers stay in L2).
__global__ void k_tbits(const int32_t* tflag, int32_t NT, uint64_t* bits) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t m = __ballot(t < NT && tflag[t] != 0);
    if ((threadIdx.x & (WAVE - 1)) == 0 && t < NT) bits[t >> 6] = m;
}
constexpr int EC_CH = 32;   // k_ix_ecount: chunks of 64 entries per wave (a run's sum carried across them)
__global__ void k_ix_ecount(const int32_t* eb_tr, const int32_t* eb_cnt, const int32_t* eb_eid, int64_t n,
                            const uint64_t* tb, uint32_t* cnt) {
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    int32_t ce = -1;   // the run that continues into the next chunk (wave-uniform) and its sum so far
    uint32_t cv = 0u;
    for (int c = 0; c < EC_CH; ++c) {
        const int64_t i = (w * EC_CH + c) * WAVE + lane;
        if (w * EC_CH * WAVE + (int64_t)c * WAVE >= n) break;   // (wave-uniform)
        const bool in = i < n;
        const int32_t e = in ? eb_eid[i] : -1;
        const int32_t t = in ? eb_tr[i] : 0;
        uint32_t v = (in && ((tb[t >> 6] >> (t & 63)) & 1ull)) ? (uint32_t)eb_cnt[i] : 0u;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {   // inclusive segmented scan (ids ascend along the wave)
            const uint32_t u = __shfl_up(v, o, WAVE);
            const int32_t eu = __shfl_up(e, o, WAVE);
            if (lane >= o && eu == e) v += u;
        }
        if (e == ce) v += cv;   // (the chunk's first run continues the carried one)
        else if (lane == 0 && ce >= 0 && cv) atomicAdd(&cnt[ce], cv);   // (or the carried run ended with the chunk)
        const int32_t en = __shfl_down(e, 1, WAVE);
        if (in && v && lane != WAVE - 1 && en != e) atomicAdd(&cnt[e], v);
        ce = __builtin_amdgcn_readlane(e, WAVE - 1);
        cv = (uint32_t)__builtin_amdgcn_readlane((int)v, WAVE - 1);
    }
    if (lane == 0 && ce >= 0 && cv) atomicAdd(&cnt[ce], cv);
}
// a sharded build's hash set from the per-id counts (one insert per id present, not per entry)
__global__ void k_ix_edense_hash(const uint64_t* ekey, const uint32_t* cnt, int64_t E, uint64_t* gk, uint32_t* gc,
                                 uint64_t gmask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < E && cnt[i]) global_edge_add(ekey[i], cnt[i], gk, gc, gmask);
}
// join pairs whose rows lie in different traces count when both traces are selected (T11)
__global__ void k_ix_cross(const uint8_t* mask, const int32_t* tc, const int32_t* tp, const uint64_t* key, int64_t n,
                           uint64_t* gk, uint32_t* gc, uint64_t gmask, const int32_t* eid) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && mask[tc[i]] && mask[tp[i]]) {
        if (eid) atomicAdd(&gc[eid[i]], 1u);
        else global_edge_add(key[i], 1u, gk, gc, gmask);
    }
}
// the selected traces' rows (trace_code, len_t, CSR offsets) and, entry-parallel, their op lists
// rs_ops[zoff[t] + k] = node of the k-th pod-op: one launch over max(NT, n_po)
__global__ void k_ix_traces(const int32_t* tflag, const int64_t* tpos, const int64_t* zoff, int32_t NT,
                            const int32_t* tlen, int32_t* trace_code, int32_t* len_t, int64_t* rs_off, int64_t n_po,
                            const int32_t* po_tr, const int64_t* po_off, const int32_t* po_op,
                            const int32_t* node_of_code, int32_t* rs_ops) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < NT && tflag[i]) {
        const int32_t p = (int32_t)tpos[i];
        trace_code[p] = (int32_t)i;
        len_t[p] = tlen[i];
        rs_off[p] = zoff[i];
    }
    if (i < n_po) {
        const int32_t t = po_tr[i];
        if (tflag[t]) rs_ops[zoff[t] + (i - po_off[t])] = node_of_code[po_op[i]];
    }
}
// ---------------------------------------------------------------- both graphs of a window in one pass
// A window's two graphs (online_rca.py:180,185: the detector's abnormal traces, state 2 -> graph 0
// "normal"; its normal traces, state 1 -> graph 1, T1) select disjoint traces of one table, so one
// pass over the per-trace index serves both: each entry goes to the graph of its trace's state.
struct IxSide {
    int32_t *tflag, *ocnt, *ofirst, *ocov;
    int64_t *tpos, *zoff;
    uint32_t* gc;
};
struct IxSide2 {
    IxSide g[2];
};
__device__ __forceinline__ int side_of(uint8_t st) { return st == 2 ? 0 : st == 1 ? 1 : -1; }
// selection + the four exclusive scans (tpos and zoff of each graph) by decoupled look-back, and the
// clearing of both graphs' counters
__device__ __forceinline__ void ix_sel_scan2_body(const uint8_t* state, const int32_t* tlen, const int64_t* po_off,
                                                       int32_t NT, IxSide2 x, unsigned long long* st, uint64_t epoch,
                                                       int32_t NP, int64_t ecap, int32_t blk_, int32_t nblk_) {
    __shared__ int64_t sa[4][SEL_T];
    __shared__ int64_t ex[4];
    __shared__ int64_t so[SEL_TILE];   // the tile's outputs, staged for coalesced stores
    const int tid = threadIdx.x;
    const int64_t gsz = (int64_t)nblk_ * SEL_T, gi = (int64_t)blk_ * SEL_T + tid;
    for (int64_t i = gi; i < max((int64_t)NP, ecap); i += gsz)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            if (i < NP) {
                x.g[g].ocnt[i] = 0;
                x.g[g].ofirst[i] = 0x7f7f7f7f;
                x.g[g].ocov[i] = 0;
            }
            if (i < ecap) x.g[g].gc[i] = 0u;
        }
    const int64_t tile = blk_, t0 = tile * SEL_TILE, base = t0 + (int64_t)tid * SEL_I;
    int8_t sd[SEL_I];
    int64_t z[SEL_I], acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < SEL_I; ++i) {
        const int64_t t = base + i;
        const int s_ = t < NT && tlen[t] > 0 ? side_of(state[t]) : -1;
        sd[i] = (int8_t)s_;
        z[i] = s_ >= 0 ? po_off[t + 1] - po_off[t] : 0;
        if (s_ >= 0) {
            acc[2 * s_] += 1;
            acc[2 * s_ + 1] += z[i];
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) sa[c][tid] = acc[c];
    __syncthreads();
    for (int o = 1; o < SEL_T; o <<= 1) {
        int64_t v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = tid >= o ? sa[c][tid - o] : 0;
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 4; ++c) sa[c][tid] += v[c];
        __syncthreads();
    }
    {   // wave c: chain c (graph c / 2, tpos or zoff)
        const int c = tid / WAVE;
        const int64_t agg = sa[c][SEL_T - 1];
        const int64_t e = dl_lookback_wave(st + (size_t)c * nblk_, tile, agg, epoch);
        if ((tid & (WAVE - 1)) == 0) {
            ex[c] = e;
            if (tile == (int64_t)nblk_ - 1) {
                int64_t* dst = (c & 1) ? x.g[c >> 1].zoff : x.g[c >> 1].tpos;
                dst[NT] = e + agg;
            }
        }
    }
    __syncthreads();
    // A thread's SEL_I values are consecutive traces: stored directly, each store instruction would
    // write 8 B into each of 64 lines (measured: 117 MB of WRITE_SIZE per 4-window chunk for 32 MB of
    // values); staged through LDS, every store is a coalesced run.  (Values of the graph a trace is
    // not in are never read.)
    int32_t* so32 = reinterpret_cast<int32_t*>(so);
#pragma unroll
    for (int i = 0; i < SEL_I; ++i) {   // both graphs' trace flags: halves of the stage
        so32[tid * SEL_I + i] = sd[i] == 0;
        so32[SEL_TILE + tid * SEL_I + i] = sd[i] == 1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SEL_I; ++k) {
        const int j = k * SEL_T + tid;
        if (t0 + j < NT) {
            x.g[0].tflag[t0 + j] = so32[j];
            x.g[1].tflag[t0 + j] = so32[SEL_TILE + j];
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {   // c: graph c / 2, tpos (even) or zoff (odd)
        int64_t run = ex[c] + sa[c][tid] - acc[c];
        __syncthreads();   // (the previous round's stage has been read)
#pragma unroll
        for (int i = 0; i < SEL_I; ++i) {
            so[tid * SEL_I + i] = run;
            if (sd[i] == (c >> 1)) run += (c & 1) ? z[i] : 1;
        }
        __syncthreads();
        int64_t* dst = (c & 1) ? x.g[c >> 1].zoff : x.g[c >> 1].tpos;
#pragma unroll
        for (int k = 0; k < SEL_I; ++k) {
            const int j = k * SEL_T + tid;
            if (t0 + j < NT) dst[t0 + j] = so[j];
        }
    }
}
__global__ void __launch_bounds__(SEL_T) k_ix_sel_scan2(const uint8_t* state, const int32_t* tlen, const int64_t* po_off,
                                                       int32_t NT, IxSide2 x, unsigned long long* st, uint64_t epoch,
                                                       int32_t NP, int64_t ecap) {
    ix_sel_scan2_body(state, tlen, po_off, NT, x, st, epoch, NP, ecap, (int32_t)blockIdx.x, (int32_t)gridDim.x);
}
// The window's detector and k_ix_sel_scan2's selection scans in ONE launch: tiles of DB traces,
// each thread its trace's state (detect_block, into d.state for the later passes) and then the
// four look-back chains over one trace per thread.
__device__ __forceinline__ void ix_detect_scan2_body(DetIn d, const int64_t* po_off, int32_t NT, IxSide2 x,
                                                        unsigned long long* st, uint64_t epoch, int32_t NP,
                                                        int64_t ecap, int32_t blk_, int32_t nblk_) {
    __shared__ double term[DB * DCAP];
    __shared__ int64_t sa[4][DB];
    __shared__ int64_t ex[4];
    const int tid = threadIdx.x;
    const int64_t gsz = (int64_t)nblk_ * DB, gi = (int64_t)blk_ * DB + tid;
    for (int64_t i = gi; i < max((int64_t)NP, ecap); i += gsz)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            if (i < NP) {
                x.g[g].ocnt[i] = 0;
                x.g[g].ofirst[i] = 0x7f7f7f7f;
                x.g[g].ocov[i] = 0;
            }
            if (i < ecap) x.g[g].gc[i] = 0u;
        }
    const int stt = detect_block(NT, d, term, blk_);
    const int64_t tile = blk_, t = tile * DB + tid;
    const int s_ = t < NT && d.tlen[t] > 0 ? side_of((uint8_t)stt) : -1;
    const int64_t z = s_ >= 0 ? po_off[t + 1] - po_off[t] : 0;
    if (t < NT) {
        x.g[0].tflag[t] = s_ == 0;
        x.g[1].tflag[t] = s_ == 1;
    }
    int64_t acc[4] = {0, 0, 0, 0};
    if (s_ >= 0) {
        acc[2 * s_] = 1;
        acc[2 * s_ + 1] = z;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) sa[c][tid] = acc[c];
    __syncthreads();
    for (int o = 1; o < DB; o <<= 1) {
        int64_t v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = tid >= o ? sa[c][tid - o] : 0;
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 4; ++c) sa[c][tid] += v[c];
        __syncthreads();
    }
    {   // wave c: chain c (graph c / 2, tpos or zoff)
        const int c = tid / WAVE;
        const int64_t agg = sa[c][DB - 1];
        const int64_t e = dl_lookback_wave(st + (size_t)c * nblk_, tile, agg, epoch);
        if ((tid & (WAVE - 1)) == 0) {
            ex[c] = e;
            if (tile == (int64_t)nblk_ - 1) {
                int64_t* dst = (c & 1) ? x.g[c >> 1].zoff : x.g[c >> 1].tpos;
                dst[NT] = e + agg;
            }
        }
    }
    __syncthreads();
    if (t < NT) {   // (values of the graph the trace is not in are never read)
        x.g[0].tpos[t] = ex[0] + sa[0][tid] - acc[0];
        x.g[0].zoff[t] = ex[1] + sa[1][tid] - acc[1];
        x.g[1].tpos[t] = ex[2] + sa[2][tid] - acc[2];
        x.g[1].zoff[t] = ex[3] + sa[3][tid] - acc[3];
    }
}
__global__ void __launch_bounds__(DB) k_ix_detect_scan2(DetIn d, const int64_t* po_off, int32_t NT, IxSide2 x,
                                                        unsigned long long* st, uint64_t epoch, int32_t NP,
                                                        int64_t ecap) {
    ix_detect_scan2_body(d, po_off, NT, x, st, epoch, NP, ecap, (int32_t)blockIdx.x, (int32_t)gridDim.x);
}
static_assert(DB == 4 * WAVE, "k_ix_detect_scan2: one wave per look-back chain");
// both graphs' per-pod-op counts / first rows / coverage and edge counts per dense id, one pass
__device__ __forceinline__ void ix_stats2_body(const uint8_t* state, int64_t n_po, const int32_t* po_tr,
                                                    const int32_t* po_op, const int32_t* po_cnt,
                                                    const int32_t* po_first, int64_t n_ed, const int32_t* ed_tr,
                                                    const int32_t* ed_eid, const int32_t* ed_cnt, int32_t NP,
                                                    int32_t n_ek, IxSide2 x, int32_t blk_, int32_t nblk_) {
    extern __shared__ int32_t lh[];
    const int32_t W = 3 * NP + n_ek;   // words per graph: cnt, first, cov, edge counts
    for (int32_t i = threadIdx.x; i < 2 * W; i += IX_BT) {
        const int32_t j = i % W;
        lh[i] = (j >= NP && j < 2 * NP) ? 0x7fffffff : 0;
    }
    __syncthreads();
    const int64_t pper = (n_po + nblk_ - 1) / nblk_, eper = (n_ed + nblk_ - 1) / nblk_;
    const int64_t p0 = (int64_t)blk_ * pper, p1 = min(p0 + pper, n_po);
    // (as k_ix_stats: a round's state gathers, then the next round's loads, then its atomics)
    int32_t tr[IX_B], op[IX_B], cn[IX_B], fr[IX_B];
    auto po_load = [&](int64_t rb) {
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            const int64_t r = min(rb + threadIdx.x + (int64_t)j * IX_BT, p1 - 1);
            tr[j] = po_tr[r];
            op[j] = po_op[r];
            cn[j] = po_cnt[r];
            fr[j] = po_first[r];
        }
    };
    if (p0 < p1) po_load(p0);
    for (int64_t rb = p0; rb < p1; rb += (int64_t)IX_BT * IX_B) {
        uint8_t sv[IX_B];
        int32_t cop[IX_B], ccn[IX_B], cfr[IX_B];
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            sv[j] = state[tr[j]];
            cop[j] = op[j];
            ccn[j] = cn[j];
            cfr[j] = fr[j];
        }
        if (rb + (int64_t)IX_BT * IX_B < p1) po_load(rb + (int64_t)IX_BT * IX_B);
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            const int sd = rb + threadIdx.x + (int64_t)j * IX_BT < p1 ? side_of(sv[j]) : -1;
            if (sd < 0) continue;
            int32_t* L = lh + sd * W;
            atomicAdd(&L[cop[j]], ccn[j]);
            atomicMin(&L[NP + cop[j]], cfr[j]);
            atomicAdd(&L[2 * NP + cop[j]], 1);
        }
    }
    const int64_t q0 = (int64_t)blk_ * eper, q1 = min(q0 + eper, n_ed);
    int32_t et[IX_B], ei[IX_B], en[IX_B];
    auto ed_load = [&](int64_t rb) {
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            const int64_t r = min(rb + threadIdx.x + (int64_t)j * IX_BT, q1 - 1);
            et[j] = ed_tr[r];
            ei[j] = ed_eid[r];
            en[j] = ed_cnt[r];
        }
    };
    if (q0 < q1) ed_load(q0);
    for (int64_t rb = q0; rb < q1; rb += (int64_t)IX_BT * IX_B) {
        uint8_t sv[IX_B];
        int32_t cid[IX_B], ccn[IX_B];
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            sv[j] = state[et[j]];
            cid[j] = ei[j];
            ccn[j] = en[j];
        }
        if (rb + (int64_t)IX_BT * IX_B < q1) ed_load(rb + (int64_t)IX_BT * IX_B);
#pragma unroll
        for (int j = 0; j < IX_B; ++j) {
            const int sd = rb + threadIdx.x + (int64_t)j * IX_BT < q1 ? side_of(sv[j]) : -1;
            if (sd >= 0) atomicAdd((uint32_t*)&lh[sd * W + 3 * NP + cid[j]], (uint32_t)ccn[j]);
        }
    }
    __syncthreads();
    for (int32_t i = threadIdx.x; i < 2 * W; i += IX_BT) {
        const int32_t g = i / W, j = i % W;
        const int32_t v = lh[i];
        if (j < NP) {
            if (v) {
                atomicAdd(&x.g[g].ocnt[j], v);
                atomicMin(&x.g[g].ofirst[j], lh[g * W + NP + j]);
                atomicAdd(&x.g[g].ocov[j], lh[g * W + 2 * NP + j]);
            }
        } else if (j >= 3 * NP && v) {
            atomicAdd(&x.g[g].gc[j - 3 * NP], (uint32_t)v);
        }
    }
}
__global__ void __launch_bounds__(IX_BT) k_ix_stats2(const uint8_t* state, int64_t n_po, const int32_t* po_tr,
                                                    const int32_t* po_op, const int32_t* po_cnt,
                                                    const int32_t* po_first, int64_t n_ed, const int32_t* ed_tr,
                                                    const int32_t* ed_eid, const int32_t* ed_cnt, int32_t NP,
                                                    int32_t n_ek, IxSide2 x) {
    ix_stats2_body(state, n_po, po_tr, po_op, po_cnt, po_first, n_ed, ed_tr, ed_eid, ed_cnt, NP, n_ek, x, (int32_t)blockIdx.x, (int32_t)gridDim.x);
}
// join pairs across traces (T11): counted in a graph when both traces are in it
__global__ void k_ix_cross2(const uint8_t* state, const int32_t* tc, const int32_t* tp, const int32_t* eid, int64_t n,
                            IxSide2 x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int sd = side_of(state[tc[i]]);
    if (sd >= 0 && side_of(state[tp[i]]) == sd) atomicAdd(&x.g[sd].gc[eid[i]], 1u);
}
// both graphs' trace rows and op lists (k_ix_traces per graph)
struct TrOut {
    int32_t *trace_code, *len_t, *rs_ops;
    int64_t* rs_off;
    const int32_t* node_of_code;
};
struct TrOut2 {
    TrOut g[2];
};
__global__ void k_ix_traces2(const uint8_t* state, IxSide2 x, int32_t NT, const int32_t* tlen, int64_t n_po,
                             const int32_t* po_tr, const int64_t* po_off, const int32_t* po_op, TrOut2 o) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < NT) {
        const int sd = side_of(state[i]);
        if (sd >= 0 && x.g[sd].tflag[i]) {
            const int32_t p = (int32_t)x.g[sd].tpos[i];
            o.g[sd].trace_code[p] = (int32_t)i;
            o.g[sd].len_t[p] = tlen[i];
            o.g[sd].rs_off[p] = x.g[sd].zoff[i];
        }
    }
    if (i < n_po) {
        const int32_t t = po_tr[i];
        const int sd = side_of(state[t]);
        if (sd >= 0 && x.g[sd].tflag[t])
            o.g[sd].rs_ops[x.g[sd].zoff[t] + (i - po_off[t])] = o.g[sd].node_of_code[po_op[i]];
    }
}

// ---------------------------------------------------------------- sharded build: the join across ranks
// A child row's parent rows may lie in traces of another rank (T11).  Each rank publishes a
// Bloom filter of the ParentSpanIds of its selected rows; a rank exports the selected rows whose
// spanID may be a parent on another rank (both filter bits set there); every rank joins its
// children against the other ranks' exports (exact spanID compare), counting edges at the child.
__device__ __forceinline__ uint32_t bloom_bit(uint64_t k, int i, int fb) {
    return (uint32_t)(hmix(k + (i ? 0x9E3779B97F4A7C15ull : 0ull)) >> 20) & ((1u << fb) - 1u);
}
__global__ void k_bloom_set(const int32_t* trace, const int64_t* parent, int64_t S, const uint8_t* mask, int fb,
                            uint32_t* F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S || !mask[trace[i]] || parent[i] < 0) return;
    for (int h = 0; h < 2; ++h) {
        const uint32_t b = bloom_bit((uint64_t)parent[i], h, fb);
        atomicOr(&F[b >> 5], 1u << (b & 31));
    }
}
__global__ void k_export_flags(const int32_t* trace, const int64_t* span, int64_t S, const uint8_t* mask, int fb,
                               const uint32_t* Fall, int64_t words, int R, int me, int32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    int32_t hit = 0;
    if (mask[trace[i]]) {
        const uint32_t b0 = bloom_bit((uint64_t)span[i], 0, fb), b1 = bloom_bit((uint64_t)span[i], 1, fb);
        for (int r = 0; r < R && !hit; ++r) {
            if (r == me) continue;
            const uint32_t* F = Fall + (size_t)r * words;
            hit = ((F[b0 >> 5] >> (b0 & 31)) & (F[b1 >> 5] >> (b1 & 31)) & 1u) ? 1 : 0;
        }
    }
    flag[i] = hit;
}
// export record: (spanID code, pod-op | rank << 32); pads (~0, ~0) sort last
__global__ void k_export_fill(const int32_t* flag, const int64_t* pos, int64_t S, const int64_t* span,
                              const int32_t* podop, int me, int64_t cap, uint64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S && flag[i]) {
        out[2 * pos[i]] = (uint64_t)span[i];
        out[2 * pos[i] + 1] = (uint64_t)(uint32_t)podop[i] | ((uint64_t)(uint32_t)me << 32);
    }
    const int64_t n = pos[S];
    if (i >= n && i < cap) out[2 * i] = out[2 * i + 1] = ~0ull;
}
__global__ void k_export_keys(const uint64_t* rec, int64_t n, uint64_t* key, uint32_t* val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        key[i] = rec[2 * i];
        val[i] = (uint32_t)i;
    }
}
// per selected child row: the other ranks' export records with spanID == its parent
template <bool ADD>
__global__ void k_cross_join(const int32_t* trace, const int64_t* parent, const int32_t* podop, int64_t S,
                             const uint8_t* mask, const uint64_t* skey, const uint32_t* sval, const uint64_t* rec,
                             int64_t n, int me, unsigned long long* count, uint64_t* gk, uint32_t* gc, uint64_t gmask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S || !mask[trace[i]] || parent[i] < 0) return;
    const uint64_t p = (uint64_t)parent[i];
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (skey[mid] < p) lo = mid + 1;
        else hi = mid;
    }
    uint32_t c = 0;
    for (int64_t j = lo; j < n && skey[j] == p; ++j) {
        const uint64_t w = rec[2 * (size_t)sval[j] + 1];
        if ((int)(w >> 32) == me) continue;   // this rank's own rows: joined locally
        ++c;
        if (ADD) global_edge_add(((w & 0xffffffffull) << 32) | (uint32_t)podop[i], 1u, gk, gc, gmask);
    }
    if (!ADD && c) atomicAdd(count, (unsigned long long)c);
}
__global__ void k_neg_i32(int32_t* a, int32_t n) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = -a[i];
}
}  // namespace

// ------------------------------------------------------------------------------ host
int mr_spans_finish(mr_ctx* ctx, mr_spans* s);

extern "C" int mr_spans_upload(mr_ctx* ctx, const mr_span_cols* c, mr_spans** out) {
    if (!ctx || !c || !out) return mr_fail(ctx, MR_ERR_ARG, "mr_spans_upload: null argument");
    *out = nullptr;
    const int64_t S = c->n_spans;
    if (S < 0 || S >= (1ll << 31)) return mr_fail(ctx, MR_ERR_ARG, "n_spans out of range (int32 row ids)");
    if (S && (!c->trace || !c->podop || !c->svcop || !c->span || !c->parent || !c->duration))
        return mr_fail(ctx, MR_ERR_ARG, "mr_spans_upload: missing column");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    int64_t max_code = -1;
    for (int64_t i = 0; i < S; ++i) {
        if (c->span[i] < 0) return mr_fail(ctx, MR_ERR_ARG, "negative span code at row %lld", (long long)i);
        if (c->trace[i] < 0 || c->trace[i] >= c->n_traces || c->podop[i] < 0 || c->podop[i] >= c->n_podops ||
            c->svcop[i] < 0 || c->svcop[i] >= c->n_svcops)
            return mr_fail(ctx, MR_ERR_ARG, "code out of range at row %lld", (long long)i);
        max_code = std::max(max_code, c->span[i]);
    }
    auto* s = new mr_spans();
    s->ctx = ctx;
    s->S = S;
    s->n_traces = c->n_traces;
    s->n_podops = c->n_podops;
    s->n_svcops = c->n_svcops;
    s->n_span_codes = max_code + 1;
    s->has_times = c->tstart && c->tend;
    int64_t row_max = S;
    if (c->row) {
        row_max = 0;
        for (int64_t i = 0; i < S; ++i) {
            if (c->row[i] < 0 || (i && c->row[i] <= c->row[i - 1]))
                return mr_fail(ctx, MR_ERR_ARG, "row: global row indices must be non-negative and ascending");
            row_max = std::max<int64_t>(row_max, c->row[i]);
        }
    }
    s->row_bits = bits_for((uint64_t)std::max<int64_t>(row_max, 1));
    int rc = MR_OK;
    auto fail = [&](int code) {
        delete s;
        return code;
    };
    if ((rc = s->trace.upload(ctx, c->trace, S)) || (rc = s->podop.upload(ctx, c->podop, S)) ||
        (rc = s->svcop.upload(ctx, c->svcop, S)) || (rc = s->span.upload(ctx, c->span, S)) ||
        (rc = s->parent.upload(ctx, c->parent, S)) || (rc = s->duration.upload(ctx, c->duration, S)))
        return fail(rc);
    if (s->has_times && ((rc = s->tstart.upload(ctx, c->tstart, S)) || (rc = s->tend.upload(ctx, c->tend, S))))
        return fail(rc);
    if (c->row && (rc = s->grow.upload(ctx, c->row, S))) return fail(rc);
    if ((rc = mr_spans_finish(ctx, s))) return fail(rc);
    mr_handle_add(ctx, s, [](void* h) { delete (mr_spans*)h; });
    *out = s;
    return MR_OK;
}

// device columns in place -> the spanID -> rows multimap (counting sort by code) and the
// per-trace index; shared by mr_spans_upload (int codes) and mr_spans_ingest (strings)
int mr_spans_finish(mr_ctx* ctx, mr_spans* s) {
    const int64_t S = s->S, U = s->n_span_codes;
    DBuf<int32_t> cnt;
    DBuf<int64_t> tmp;
    MR_TRY(cnt.zero(ctx, (size_t)U));
    MR_TRY(s->id_off.alloc(ctx, (size_t)U + 1));
    MR_TRY(s->id_rows.alloc(ctx, (size_t)S));
    MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(U)));
    if (S) hipLaunchKernelGGL(k_count_codes, dim3(cdiv(S, 256)), dim3(256), 0, ctx->stream, s->span.p, S, cnt.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, cnt.p, s->id_off.p, U, tmp.p));
    if (U) MR_TRY_HIP(ctx, hipMemsetAsync(cnt.p, 0, U * sizeof(int32_t), ctx->stream));
    if (S)
        hipLaunchKernelGGL(k_fill_ids, dim3(cdiv(S, 256)), dim3(256), 0, ctx->stream, s->span.p, S, s->id_off.p, cnt.p,
                           s->id_rows.p);
    if (U) hipLaunchKernelGGL(k_sort_buckets, dim3(cdiv(U, 256)), dim3(256), 0, ctx->stream, s->id_off.p, U, s->id_rows.p);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess)
        return mr_fail(ctx, MR_ERR_HIP, "span table setup: kernel failure");
    return mr_spans_index(ctx, s);
}

extern "C" int mr_spans_free(mr_spans* s) {
    if (!s || !mr_handle_take(s)) return MR_OK;   // (freed with its context)
    (void)hipSetDevice(s->ctx->device);
    (void)hipStreamSynchronize(s->ctx->stream);
    delete s;
    return MR_OK;
}

static int read_i64(mr_ctx* ctx, const int64_t* dev, int64_t* host) { return mr_read_words(ctx, dev, 1, host); }

// Shared by both builds, after the per-pod-op statistics and the call-edge hash are complete:
// call edges -> node order (sorted parent ops, then the others by first appearance, T10) ->
// per-node arrays (len_o, nchild) and P_ss by child.  ofirst holds a key per pod-op that orders
// first appearances like the DataFrame rows (row_bits wide).
// two int32 arrays of n cleared in one launch (instead of two memsets)
__global__ void k_zero2_i32(int32_t* a, int32_t* b, int32_t n) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        a[i] = 0;
        b[i] = 0;
    }
}
// sharded: node presence (span counts), first appearances and parent flags are reduced over the
// ranks for the node order (every rank the same N and order); len_o / nchild stay this rank's.
static int build_nodes(mr_ctx* ctx, mr_graph* g, int32_t NP, const int32_t* ocnt, const int32_t* ofirst,
                       const int32_t* ocov, int row_bits,
                       const uint64_t* gk, const uint32_t* gc, uint64_t ecap, DBuf<int32_t>& node_of_code,
                       PhaseTimer* pt = nullptr, bool sharded = false) {
    hipStream_t st = ctx->stream;
    DBuf<int32_t> eflag, is_par, nchild_code;
    DBuf<int64_t> epos, etmp, tmp;
    MR_TRY(eflag.alloc(ctx, ecap));
    MR_TRY(epos.alloc(ctx, ecap + 1));
    MR_TRY(etmp.alloc(ctx, scan_tmp_elems(ecap)));
    MR_TRY(tmp.alloc(ctx, std::max<int64_t>(scan_tmp_elems(NP), 1)));
    MR_TRY(is_par.alloc(ctx, NP));
    MR_TRY(nchild_code.alloc(ctx, NP));
    if (NP) hipLaunchKernelGGL(k_zero2_i32, dim3(cdiv(NP, 256)), dim3(256), 0, st, is_par.p, nchild_code.p, NP);
    hipLaunchKernelGGL(k_edge_flags, dim3(cdiv(ecap, 256)), dim3(256), 0, st, gk, gc, (int64_t)ecap, eflag.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, eflag.p, epos.p, ecap, etmp.p));
    int64_t E = 0;
    MR_TRY(read_i64(ctx, epos.p + ecap, &E));
    DBuf<uint64_t> ekey;
    DBuf<uint32_t> ecnt;
    MR_TRY(ekey.alloc(ctx, E));
    MR_TRY(ecnt.alloc(ctx, E));
    hipLaunchKernelGGL(k_edge_compact, dim3(cdiv(ecap, 256)), dim3(256), 0, st, gk, gc, eflag.p, epos.p, (int64_t)ecap,
                       ekey.p, ecnt.p, is_par.p, nchild_code.p);
    if (pt) pt->mark("edges");
    DBuf<int32_t> ocnt_g, ofirst_g;
    const int32_t* ocnt_o = ocnt;     // the node order's presence counts and first rows
    const int32_t* ofirst_o = ofirst;
    if (sharded && NP) {
        MR_TRY(ocnt_g.alloc(ctx, NP));
        MR_TRY(ofirst_g.alloc(ctx, NP));
        MR_TRY_HIP(ctx, hipMemcpyAsync(ocnt_g.p, ocnt, NP * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
        MR_TRY_HIP(ctx, hipMemcpyAsync(ofirst_g.p, ofirst, NP * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(k_neg_i32, dim3(cdiv(NP, 256)), dim3(256), 0, st, ofirst_g.p, NP);
        MR_TRY(mr_coll_allreduce(ctx, is_par.p, NP, MR_DT_I32, 1));
        MR_TRY(mr_coll_allreduce(ctx, ocnt_g.p, NP, MR_DT_I32, 0));
        MR_TRY(mr_coll_allreduce(ctx, ofirst_g.p, NP, MR_DT_I32, 1));   // max of -first = min first
        hipLaunchKernelGGL(k_neg_i32, dim3(cdiv(NP, 256)), dim3(256), 0, st, ofirst_g.p, NP);
        ocnt_o = ocnt_g.p;
        ofirst_o = ofirst_g.p;
    }
    // node order
    DBuf<int32_t> pflag, qflag;
    DBuf<int64_t> ppos, qpos;
    MR_TRY(pflag.alloc(ctx, NP));
    MR_TRY(qflag.alloc(ctx, NP));
    MR_TRY(ppos.alloc(ctx, NP + 1));
    MR_TRY(qpos.alloc(ctx, NP + 1));
    MR_TRY(node_of_code.alloc(ctx, NP));
    if (NP) hipLaunchKernelGGL(k_node_flags, dim3(cdiv(NP, 256)), dim3(256), 0, st, ocnt_o, is_par.p, NP, pflag.p, qflag.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, pflag.p, ppos.p, NP, tmp.p));
    MR_TRY(mr_exclusive_scan_i32(ctx, qflag.p, qpos.p, NP, tmp.p));
    int64_t PQ[2] = {0, 0};
    MR_TRY_HIP(ctx, hipMemcpyAsync(&PQ[0], ppos.p + NP, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipMemcpyAsync(&PQ[1], qpos.p + NP, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    const int64_t P = PQ[0], Q = PQ[1];
    const int32_t N = (int32_t)(P + Q);
    MR_TRY(g->node_podop.alloc(ctx, N));
    DBuf<uint64_t> qkey;
    DBuf<uint32_t> qval;
    MR_TRY(qkey.alloc(ctx, Q));
    MR_TRY(qval.alloc(ctx, Q));
    if (NP)
        hipLaunchKernelGGL(k_node_parents, dim3(cdiv(NP, 256)), dim3(256), 0, st, pflag.p, ppos.p, qflag.p, qpos.p, ofirst_o,
                           NP, node_of_code.p, g->node_podop.p, qkey.p, qval.p);
    SortScratch ws;
    MR_TRY(mr_radix_sort(ctx, qkey.p, qval.p, Q, row_bits, ws));
    if (Q)
        hipLaunchKernelGGL(k_node_rest, dim3(cdiv(Q, 256)), dim3(256), 0, st, qval.p, Q, (int32_t)P, node_of_code.p,
                           g->node_podop.p);
    if (pt) pt->mark("order");
    // per-node arrays and P_ss
    const int nb = std::max(1, bits_for((uint64_t)std::max(N - 1, 0)));
    MR_TRY(g->len_o.alloc(ctx, N));
    MR_TRY(g->nchild.alloc(ctx, N));
    if (ocov) MR_TRY(g->cov.alloc(ctx, (size_t)std::max(N, 1)));
    if (N)
        hipLaunchKernelGGL(k_node_arrays, dim3(cdiv(N, 256)), dim3(256), 0, st, g->node_podop.p, N, ocnt, nchild_code.p,
                           ocov, g->len_o.p, g->nchild.p, g->cov.p);
    g->cov_ready = ocov != nullptr;
    DBuf<uint64_t> skey;
    MR_TRY(skey.alloc(ctx, E));
    if (E) hipLaunchKernelGGL(k_edge_nodes, dim3(cdiv(E, 256)), dim3(256), 0, st, ekey.p, E, node_of_code.p, nb, skey.p);
    MR_TRY(mr_radix_sort(ctx, skey.p, nullptr, E, 2 * nb, ws));
    DBuf<int32_t> ccount;
    DBuf<int64_t> ntmp;
    MR_TRY(ccount.zero(ctx, N));
    MR_TRY(ntmp.alloc(ctx, scan_tmp_elems(std::max(N, 1))));
    MR_TRY(g->ss_par.alloc(ctx, E));
    MR_TRY(g->ss_off.alloc(ctx, N + 1));
    if (E) hipLaunchKernelGGL(k_edge_csr, dim3(cdiv(E, 256)), dim3(256), 0, st, skey.p, E, nb, g->ss_par.p, ccount.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, ccount.p, g->ss_off.p, N, ntmp.p));
    MR_TRY_HIP(ctx, hipGetLastError());
    g->N = N;
    g->E = E;
    return MR_OK;
}

static uint64_t edge_capacity(int64_t want, int32_t NP) {
    const uint64_t w = (uint64_t)std::min<int64_t>(std::max<int64_t>(want, 1), (int64_t)NP * NP + 1);
    uint64_t cap = 1024;
    while (cap < 2 * w) cap <<= 1;
    return cap;
}

// Row-level build: any span table (rows selected by trace mask and, when `win`, by the
// trace-level time window of each row).
static int graph_build_rows(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_mask, const int64_t* win, mr_graph* g) {
    hipStream_t st = ctx->stream;
    const int64_t S = sp->S;
    const int32_t NT = sp->n_traces, NP = sp->n_podops;
    // 1. selected rows
    DBuf<int32_t> selflag, rows;
    DBuf<int64_t> pos, tmp;
    const int64_t tmpn = std::max<int64_t>({scan_tmp_elems(S), scan_tmp_elems(NT), scan_tmp_elems(NP), 1});
    MR_TRY(selflag.alloc(ctx, S));
    MR_TRY(pos.alloc(ctx, S + 1));
    MR_TRY(tmp.alloc(ctx, tmpn));
    if (S)
        hipLaunchKernelGGL(k_sel_flags, dim3(cdiv(S, 256)), dim3(256), 0, st, sp->trace.p, S, d_mask, win ? sp->tstart.p : nullptr,
                           win ? sp->tend.p : nullptr, win ? win[0] : 0, win ? win[1] : 0, selflag.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, selflag.p, pos.p, S, tmp.p));
    int64_t Ssel = 0;
    MR_TRY(read_i64(ctx, pos.p + S, &Ssel));
    MR_TRY(rows.alloc(ctx, Ssel));
    if (S) hipLaunchKernelGGL(k_compact_rows, dim3(cdiv(S, 256)), dim3(256), 0, st, selflag.p, pos.p, S, rows.p);
    // 2. statistics + join
    DBuf<int32_t> tcnt, ocnt, ofirst;
    MR_TRY(tcnt.zero(ctx, NT));
    MR_TRY(ocnt.zero(ctx, NP));
    MR_TRY(ofirst.alloc(ctx, NP));
    if (NP) MR_TRY_HIP(ctx, hipMemsetAsync(ofirst.p, 0x7f, NP * sizeof(int32_t), st));
    const uint64_t ecap = edge_capacity(Ssel, NP);
    DBuf<uint64_t> gk;
    DBuf<uint32_t> gc;
    MR_TRY(gk.alloc(ctx, ecap));
    MR_TRY(gc.zero(ctx, ecap));
    MR_TRY_HIP(ctx, hipMemsetAsync(gk.p, 0xff, ecap * sizeof(uint64_t), st));
    const int use_lds = NP <= LDS_HIST;
    const size_t lds = use_lds ? 2 * (size_t)NP * sizeof(int32_t) : 0;
    if (Ssel)
        hipLaunchKernelGGL(k_rows, dim3(cdiv(Ssel, BT * 8)), dim3(BT), lds, st, rows.p, Ssel, sp->trace.p, sp->podop.p,
                           sp->parent.p, selflag.p, sp->id_off.p, sp->id_rows.p, sp->n_span_codes, NP, use_lds, tcnt.p,
                           ocnt.p, ofirst.p, gk.p, gc.p, ecap - 1);
    // 3. edges, node order, per-node arrays, P_ss
    DBuf<int32_t> node_of_code;
    MR_TRY(build_nodes(ctx, g, NP, ocnt.p, ofirst.p, nullptr, bits_for((uint64_t)std::max<int64_t>(Ssel, 1)), gk.p,
                       gc.p, ecap, node_of_code));
    const int32_t N = g->N;
    // traces
    DBuf<int32_t> tflag, tidx_of_code;
    DBuf<int64_t> tpos;
    MR_TRY(tflag.alloc(ctx, NT));
    MR_TRY(tpos.alloc(ctx, NT + 1));
    MR_TRY(tidx_of_code.alloc(ctx, NT));
    if (NT) hipLaunchKernelGGL(k_trace_flags, dim3(cdiv(NT, 256)), dim3(256), 0, st, tcnt.p, NT, tflag.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, tflag.p, tpos.p, NT, tmp.p));
    int64_t T64 = 0;
    MR_TRY(read_i64(ctx, tpos.p + NT, &T64));
    const int32_t T = (int32_t)T64;
    MR_TRY(g->trace_code.alloc(ctx, T));
    MR_TRY(g->len_t.alloc(ctx, T));
    if (NT)
        hipLaunchKernelGGL(k_trace_index, dim3(cdiv(NT, 256)), dim3(256), 0, st, tflag.p, tpos.p, tcnt.p, NT,
                           tidx_of_code.p, g->trace_code.p, g->len_t.p);
    // 4. pairs -> trace-major CSR
    const int nb = std::max(1, bits_for((uint64_t)std::max(N - 1, 0)));
    DBuf<uint64_t> keys;
    MR_TRY(keys.alloc(ctx, Ssel));
    if (Ssel)
        hipLaunchKernelGGL(k_pair_keys, dim3(cdiv(Ssel, 256)), dim3(256), 0, st, rows.p, Ssel, sp->trace.p, sp->podop.p,
                           tidx_of_code.p, node_of_code.p, nb, keys.p);
    SortScratch ws;
    MR_TRY(mr_radix_sort(ctx, keys.p, nullptr, Ssel, nb + bits_for((uint64_t)std::max(T - 1, 0)), ws));
    DBuf<int32_t> head;
    DBuf<int64_t> hpos;
    MR_TRY(head.alloc(ctx, Ssel));
    MR_TRY(hpos.alloc(ctx, Ssel + 1));
    if (Ssel) hipLaunchKernelGGL(k_run_heads, dim3(cdiv(Ssel, 256)), dim3(256), 0, st, keys.p, Ssel, head.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, head.p, hpos.p, Ssel, tmp.p));
    int64_t nnz = 0;
    MR_TRY(read_i64(ctx, hpos.p + Ssel, &nnz));
    MR_TRY(g->rs_ops.alloc(ctx, nnz));
    MR_TRY(g->rs_off.alloc(ctx, T + 1));
    if (Ssel)
        hipLaunchKernelGGL(k_pairs_out, dim3(cdiv(Ssel, 256)), dim3(256), 0, st, keys.p, head.p, hpos.p, Ssel, nb,
                           g->rs_off.p, g->rs_ops.p);
    hipLaunchKernelGGL(k_set_last, dim3(1), dim3(1), 0, st, g->rs_off.p, T, nnz);
    MR_TRY_HIP(ctx, hipGetLastError());
    g->T = T;
    g->nnz_sr = g->nnz_rs = nnz;
    return MR_OK;
}

// Indexed build (mr_span_index.hip): whole traces selected by the mask; every per-row fact comes
// from the per-trace index, so no row is sorted.  Each trace's op list is written in pod-op code
// order (a fixed order for the kind keys; mr_graph_export sorts by node id for inspection).
// The sharded build's cross-rank exchange (see k_bloom_set): the other ranks' export records
// sorted by spanID (keys / record index) and the number of cross-rank (child, parent) matches.
struct CrossJoin {
    DBuf<uint64_t> rec, key;
    DBuf<uint32_t> val;
    int64_t n = 0;
    int64_t matches = 0;
};
static int cross_exchange(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_mask, CrossJoin& X) {
    hipStream_t st = ctx->stream;
    const int64_t S = sp->S;
    const int R = ctx->nranks, me = ctx->rank;
    DBuf<int64_t> sc;
    int64_t h = S;
    MR_TRY(sc.upload(ctx, &h, 1));
    MR_TRY(mr_coll_allreduce(ctx, sc.p, 1, MR_DT_I64, 1));   // the largest shard sizes the filters
    MR_TRY(sc.download(ctx, &h, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    const int fb = std::min(28, std::max(16, bits_for((uint64_t)std::max<int64_t>(h, 1)) + 4));   // >= 16 bits per row
    const int64_t words = ((int64_t)1 << fb) / 32;
    DBuf<uint32_t> F, Fall;
    MR_TRY(F.zero(ctx, (size_t)words));
    MR_TRY(Fall.alloc(ctx, (size_t)words * R));
    if (S) hipLaunchKernelGGL(k_bloom_set, dim3(cdiv(S, 256)), dim3(256), 0, st, sp->trace.p, sp->parent.p, S, d_mask, fb, F.p);
    MR_TRY(mr_coll_allgather(ctx, F.p, Fall.p, words, MR_DT_I32));
    DBuf<int32_t> flag;
    DBuf<int64_t> pos, tmp;
    MR_TRY(flag.alloc(ctx, (size_t)std::max<int64_t>(S, 1)));
    MR_TRY(pos.alloc(ctx, (size_t)S + 1));
    MR_TRY(tmp.alloc(ctx, (size_t)std::max<int64_t>(scan_tmp_elems(S), 1)));
    if (S)
        hipLaunchKernelGGL(k_export_flags, dim3(cdiv(S, 256)), dim3(256), 0, st, sp->trace.p, sp->span.p, S, d_mask, fb,
                           Fall.p, words, R, me, flag.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, flag.p, pos.p, S, tmp.p));
    MR_TRY_HIP(ctx, hipMemcpyAsync(sc.p, pos.p + S, sizeof(int64_t), hipMemcpyDeviceToDevice, st));
    MR_TRY(mr_coll_allreduce(ctx, sc.p, 1, MR_DT_I64, 1));   // the largest export list sizes the gather
    MR_TRY(sc.download(ctx, &h, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    const int64_t cap = std::max<int64_t>(h, 1);
    DBuf<uint64_t> send;
    MR_TRY(send.alloc(ctx, 2 * (size_t)cap));
    hipLaunchKernelGGL(k_export_fill, dim3(cdiv(std::max<int64_t>(S, cap), 256)), dim3(256), 0, st, flag.p, pos.p, S,
                       sp->span.p, sp->podop.p, me, cap, send.p);
    X.n = cap * R;
    MR_TRY(X.rec.alloc(ctx, 2 * (size_t)X.n));
    MR_TRY(mr_coll_allgather(ctx, send.p, X.rec.p, 2 * cap, MR_DT_U64));
    MR_TRY(X.key.alloc(ctx, (size_t)X.n));
    MR_TRY(X.val.alloc(ctx, (size_t)X.n));
    hipLaunchKernelGGL(k_export_keys, dim3(cdiv(X.n, 256)), dim3(256), 0, st, X.rec.p, X.n, X.key.p, X.val.p);
    SortScratch ws;
    MR_TRY(mr_radix_sort(ctx, X.key.p, X.val.p, X.n, 64, ws));
    DBuf<unsigned long long> cnt;
    MR_TRY(cnt.zero(ctx, 1));
    if (S)
        hipLaunchKernelGGL(k_cross_join<false>, dim3(cdiv(S, 256)), dim3(256), 0, st, sp->trace.p, sp->parent.p,
                           sp->podop.p, S, d_mask, X.key.p, X.val.p, X.rec.p, X.n, me, cnt.p, (uint64_t*)nullptr,
                           (uint32_t*)nullptr, (uint64_t)0);
    unsigned long long m = 0;
    MR_TRY(cnt.download(ctx, &m, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    X.matches = (int64_t)m;
    return MR_OK;
}

// Split in two so a caller can read the sizes of several builds (and other counters) in ONE host
// round trip: mr_ix_launch enqueues everything up to the one-block node order (sizes to d_out:
// N, E, overflow, T, nnz), mr_ix_finish takes them (h, or null: read here) and completes the
// graph -- on overflow / sharded graphs through the general node order.
static int ix_launch(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_mask, mr_graph* g, IxBuild& b, int64_t* d_out,
                     bool sharded) {
    hipStream_t st = ctx->stream;
    const int32_t NT = sp->n_traces, NP = sp->n_podops;
    CrossJoin X;
    if (sharded && ctx->nranks > 1) MR_TRY(cross_exchange(ctx, sp, d_mask, X));   // (one rank: all joins local)
    MR_TRY(b.tflag.alloc(ctx, NT));
    MR_TRY(b.tpos.alloc(ctx, NT + 1));
    MR_TRY(b.zoff.alloc(ctx, NT + 1));
    MR_TRY(b.ocnt.alloc(ctx, NP));
    MR_TRY(b.ofirst.alloc(ctx, NP));
    MR_TRY(b.ocov.alloc(ctx, NP));
    // dense edge ids (one table's keys, counted per id) unless joins across ranks bring keys the
    // table does not hold
    const bool no_dense = getenv("MR_EDGE_HASH") != nullptr;   // A/B knob (read per call: tests flip it)
    b.dense = !sharded && !no_dense && sp->ekey.p != nullptr;
    b.ecap = b.dense ? (uint64_t)sp->n_edge_keys : edge_capacity(sp->n_edge_keys + X.matches, NP);
    const uint64_t ecap = b.ecap;
    if (!b.dense) MR_TRY(b.gk.alloc(ctx, ecap));
    MR_TRY(b.gc.alloc(ctx, std::max<uint64_t>(ecap, 1)));
    b.gkp = b.dense ? sp->ekey.p : b.gk.p;
    {   // selection + both trace scans + clearing, one launch
        const int64_t nt = std::max<int64_t>(cdiv((int64_t)NT, SEL_TILE), 1);
        unsigned long long* dst = nullptr;
        uint64_t epoch = 0;
        MR_TRY(mr_dl_status(ctx, 2 * nt, &dst, &epoch));
        hipLaunchKernelGGL(k_ix_sel_scan, dim3((unsigned)nt), dim3(SEL_T), 0, st, d_mask, sp->tlen.p, sp->po_off.p, NT,
                           b.tflag.p, b.tpos.p, b.zoff.p, dst, epoch, b.ocnt.p, b.ofirst.p, b.ocov.p, NP,
                           b.dense ? (uint64_t*)nullptr : b.gk.p, b.gc.p, (int64_t)ecap);
    }
    if (NT) {
        // more codes than one LDS histogram: op ranges of IX_HIST codes in blockIdx.y
        const int nrange = NP > IX_HIST ? cdiv(NP, IX_HIST) : 1;
        const int use_lds = NP <= IX_HIST || nrange > 1;
        const int64_t NPL = std::min<int64_t>(NP, IX_HIST);
        // dense edge counts in LDS beside the pod-op histogram while both fit (else global adds)
        const int lds_ek = b.dense && (use_lds ? 3 * NPL : 0) + (int64_t)ecap <= IX_LDS_WORDS;
        const size_t lds = (use_lds ? 3 * (size_t)NPL * sizeof(int32_t) : 0) + (lds_ek ? ecap * sizeof(uint32_t) : 0);
        constexpr int ix_cap = 256;   // block cap: one per CU
        int nblk = std::max(1, std::min(ix_cap, cdiv(std::max(sp->n_po, sp->n_ed), IX_BT * IX_EPT)));
        if (nrange > 1) nblk = std::max(1, std::min(nblk, 2 * ix_cap / nrange));   // ~2 rounds of one block per CU
        // ranged: the entries grouped by range first (k_ix_rpart over nshare shares, 4 blocks per CU)
        DBuf<int4> rent;
        DBuf<int32_t> rtab;
        int32_t nshare = 0;
        if (nrange > 1 && nrange <= IX_RMAX && sp->n_po > 0) {
            nshare = (int32_t)std::max<int64_t>(nblk, std::min<int64_t>(4 * (int64_t)ix_cap, cdiv(sp->n_po, IX_BT * 16)));
            MR_TRY(rent.alloc(ctx, (size_t)sp->n_po));
            MR_TRY(rtab.alloc(ctx, (size_t)nshare * (nrange + 1)));
            hipLaunchKernelGGL(k_ix_rpart, dim3(nshare), dim3(IX_BT), 0, st, b.tflag.p, sp->n_po, sp->po_tr.p, sp->po_op.p,
                               sp->po_cnt.p, sp->po_first.p, (int32_t)nrange, rent.p, rtab.p);
        }
        // edges in edge-id order when the table keeps them (large tables) and the counts do not sit
        // in LDS beside the histogram: a segmented sum per id (k_ix_ecount) instead of k_ix_stats'
        // atomic or hash probe per entry; sharded builds then insert each id's count into the hash set
        const char* ebe = getenv("MR_IX_EB");   // (read per call) "0": never
        const bool eb = sp->eb_eid.p && sp->n_ed > 0 && !(ebe && !strcmp(ebe, "0")) &&
                        (!lds_ek || (ebe && !strcmp(ebe, "force")));
        hipLaunchKernelGGL(k_ix_stats, dim3(nrange, nblk), dim3(IX_BT), lds, st, b.tflag.p, sp->n_po, sp->po_tr.p, sp->po_op.p,
                           sp->po_cnt.p, sp->po_first.p, eb ? (int64_t)0 : sp->n_ed, sp->ed_tr.p, sp->ed_key.p, sp->ed_cnt.p,
                           NP, use_lds, b.ocnt.p, b.ofirst.p, b.ocov.p, b.gk.p, b.gc.p, ecap - 1,
                           b.dense ? (const int32_t*)sp->ed_eid.p : nullptr, (int32_t)ecap, lds_ek,
                           (const int4*)rent.p, (const int32_t*)rtab.p, nshare);
        if (eb) {
            const int64_t E = sp->n_edge_keys;
            DBuf<uint64_t> tb;
            DBuf<uint32_t> idc;   // (sharded: the per-id counts before the hash set)
            MR_TRY(tb.alloc(ctx, (size_t)cdiv((int64_t)NT, 64)));
            if (!b.dense) MR_TRY(idc.zero(ctx, (size_t)E));
            hipLaunchKernelGGL(k_tbits, dim3(cdiv((int64_t)NT, 256)), dim3(256), 0, st, b.tflag.p, NT, tb.p);
            hipLaunchKernelGGL(k_ix_ecount, dim3(cdiv(sp->n_ed, 256 * EC_CH)), dim3(256), 0, st, sp->eb_tr.p, sp->eb_cnt.p,
                               sp->eb_eid.p, sp->n_ed, tb.p, b.dense ? b.gc.p : idc.p);
            if (!b.dense)
                hipLaunchKernelGGL(k_ix_edense_hash, dim3(cdiv(E, 256)), dim3(256), 0, st, sp->ekey.p, idc.p, E, b.gk.p,
                                   b.gc.p, ecap - 1);
        }
    }
    if (sp->n_xj)
        hipLaunchKernelGGL(k_ix_cross, dim3(cdiv(sp->n_xj, 256)), dim3(256), 0, st, d_mask, sp->xj_tc.p, sp->xj_tp.p,
                           sp->xj_key.p, sp->n_xj, b.gk.p, b.gc.p, ecap - 1,
                           b.dense ? (const int32_t*)sp->xj_eid.p : nullptr);
    if (X.matches && sp->S)   // cross-rank parent joins, counted at the child's rank
        hipLaunchKernelGGL(k_cross_join<true>, dim3(cdiv(sp->S, 256)), dim3(256), 0, st, sp->trace.p, sp->parent.p,
                           sp->podop.p, sp->S, d_mask, X.key.p, X.val.p, X.rec.p, X.n, ctx->rank,
                           (unsigned long long*)nullptr, b.gk.p, b.gc.p, ecap - 1);
    b.small = !sharded && NP <= NS_PMAX;
    if (b.small) {
        // one launch for the node order and P_ss, the trace rows / op lists into upper-bound
        // buffers right behind it; the sizes (N, E, T, nnz) go to d_out
        MR_TRY(b.node_of_code.alloc(ctx, std::max(NP, 1)));
        MR_TRY(g->node_podop.alloc(ctx, std::max(NP, 1)));
        MR_TRY(g->len_o.alloc(ctx, std::max(NP, 1)));
        MR_TRY(g->nchild.alloc(ctx, std::max(NP, 1)));
        MR_TRY(g->cov.alloc(ctx, std::max(NP, 1)));
        MR_TRY(g->ss_par.alloc(ctx, NS_EMAX));
        MR_TRY(g->ss_off.alloc(ctx, (size_t)NP + 1));
        MR_TRY(g->trace_code.alloc(ctx, std::max(NT, 1)));
        MR_TRY(g->len_t.alloc(ctx, std::max(NT, 1)));
        MR_TRY(g->rs_ops.alloc(ctx, (size_t)std::max<int64_t>(sp->n_po, 1)));
        MR_TRY(g->rs_off.alloc(ctx, (size_t)NT + 1));
        hipLaunchKernelGGL(k_nodes_small, dim3(1), dim3(NS_T), 0, st, b.gkp, b.gc.p, (int64_t)ecap, b.ocnt.p,
                           b.ofirst.p, NP, b.node_of_code.p, g->node_podop.p, g->len_o.p, g->nchild.p, b.ocov.p,
                           g->cov.p, g->ss_par.p, g->ss_off.p, b.tpos.p + NT, b.zoff.p + NT, g->rs_off.p, d_out);
        if (NT || sp->n_po)
            hipLaunchKernelGGL(k_ix_traces, dim3(cdiv(std::max<int64_t>(NT, sp->n_po), 256)), dim3(256), 0, st,
                               b.tflag.p, b.tpos.p, b.zoff.p, NT, sp->tlen.p, g->trace_code.p, g->len_t.p, g->rs_off.p,
                               sp->n_po, sp->po_tr.p, sp->po_off.p, sp->po_op.p, b.node_of_code.p, g->rs_ops.p);
    }
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

static int ix_finish(mr_ctx* ctx, const mr_spans* sp, mr_graph* g, IxBuild& b, const int64_t* h, bool sharded) {
    hipStream_t st = ctx->stream;
    const int32_t NT = sp->n_traces, NP = sp->n_podops;
    if (b.small && h && !h[2]) {
        g->N = (int32_t)h[0];
        g->E = h[1];
        g->T = (int32_t)h[3];
        g->nnz_sr = g->nnz_rs = h[4];
        g->cov_ready = true;
        return MR_OK;
    }
    // the general node order (sharded graphs; more call edges than the one-block path holds)
    MR_TRY(build_nodes(ctx, g, NP, b.ocnt.p, b.ofirst.p, b.ocov.p, sp->row_bits, b.gkp, b.gc.p, b.ecap, b.node_of_code,
                       nullptr, sharded));
    int64_t hh[2] = {0, 0};   // T, nnz (their scans ran before build_nodes' syncs)
    MR_TRY_HIP(ctx, hipMemcpyAsync(&hh[0], b.tpos.p + NT, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipMemcpyAsync(&hh[1], b.zoff.p + NT, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    const int32_t T = (int32_t)hh[0];
    const int64_t nnz = hh[1];
    MR_TRY(g->trace_code.alloc(ctx, T));
    MR_TRY(g->len_t.alloc(ctx, T));
    MR_TRY(g->rs_ops.alloc(ctx, nnz));
    MR_TRY(g->rs_off.alloc(ctx, T + 1));
    if (NT || sp->n_po)
        hipLaunchKernelGGL(k_ix_traces, dim3(cdiv(std::max<int64_t>(NT, sp->n_po), 256)), dim3(256), 0, st, b.tflag.p,
                           b.tpos.p, b.zoff.p, NT, sp->tlen.p, g->trace_code.p, g->len_t.p, g->rs_off.p, sp->n_po,
                           sp->po_tr.p, sp->po_off.p, sp->po_op.p, b.node_of_code.p, g->rs_ops.p);
    hipLaunchKernelGGL(k_set_last, dim3(1), dim3(1), 0, st, g->rs_off.p, T, nnz);
    MR_TRY_HIP(ctx, hipGetLastError());
    g->T = T;
    g->nnz_sr = g->nnz_rs = nnz;
    return MR_OK;
}

static int graph_build_indexed(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_mask, mr_graph* g,
                               bool sharded = false) {
    IxBuild b;
    DBuf<int64_t> dout;
    MR_TRY(dout.alloc(ctx, 8));
    MR_TRY(ix_launch(ctx, sp, d_mask, g, b, dout.p, sharded));
    int64_t h[5] = {0, 0, 0, 0, 0};   // N, E, overflow, T, nnz
    if (b.small) MR_TRY(mr_read_words(ctx, dout.p, 5, h));
    return ix_finish(ctx, sp, g, b, b.small ? h : nullptr, sharded);
}

// Both graphs of a window from the detector's states in one pass over the index (k_ix_sel_scan2,
// k_ix_stats2, k_ix_cross2, k_nodes_small2, k_ix_traces2: five launches for two graphs); sizes of
// graph g to d_out + 8 g.  det (nullable): the detector runs in the first launch
// (k_ix_detect_scan2) and writes the states to d_state.  MR_ERR_STATE when the table is past the one-pass limits (dense edge ids,
// both graphs' LDS histograms, the one-block node order): the caller builds them one by one.
int mr_ix_launch2(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_state, mr_graph* g0, mr_graph* g1, IxBuild& b0,
                  IxBuild& b1, int64_t* d_out, const DetIn* det) {
    const bool off = getenv("MR_NO_IX2") != nullptr;   // A/B knob (read per call: tests flip it)
    const int32_t NT = sp->n_traces, NP = sp->n_podops;
    const int64_t nek = sp->n_edge_keys;
    if (off || !sp->ekey.p || NP > NS_PMAX || 2 * (3 * (int64_t)NP + nek) > IX_LDS_WORDS) return MR_ERR_STATE;
    hipStream_t st = ctx->stream;
    IxBuild* b[2] = {&b0, &b1};
    mr_graph* g[2] = {g0, g1};
    IxSide2 xs;
    NsArgs2 na;
    TrOut2 to;
    for (int k = 0; k < 2; ++k) {
        IxBuild& B = *b[k];
        mr_graph* G = g[k];
        B.dense = true;
        B.small = true;
        B.ecap = (uint64_t)nek;
        B.gkp = sp->ekey.p;
        MR_TRY(B.tflag.alloc(ctx, std::max(NT, 1)));
        MR_TRY(B.tpos.alloc(ctx, (size_t)NT + 1));
        MR_TRY(B.zoff.alloc(ctx, (size_t)NT + 1));
        MR_TRY(B.ocnt.alloc(ctx, std::max(NP, 1)));
        MR_TRY(B.ofirst.alloc(ctx, std::max(NP, 1)));
        MR_TRY(B.ocov.alloc(ctx, std::max(NP, 1)));
        MR_TRY(B.gc.alloc(ctx, (size_t)std::max<int64_t>(nek, 1)));
        MR_TRY(B.node_of_code.alloc(ctx, std::max(NP, 1)));
        MR_TRY(G->node_podop.alloc(ctx, std::max(NP, 1)));
        MR_TRY(G->len_o.alloc(ctx, std::max(NP, 1)));
        MR_TRY(G->nchild.alloc(ctx, std::max(NP, 1)));
        MR_TRY(G->cov.alloc(ctx, std::max(NP, 1)));
        MR_TRY(G->ss_par.alloc(ctx, NS_EMAX));
        MR_TRY(G->ss_off.alloc(ctx, (size_t)NP + 1));
        MR_TRY(G->trace_code.alloc(ctx, std::max(NT, 1)));
        MR_TRY(G->len_t.alloc(ctx, std::max(NT, 1)));
        MR_TRY(G->rs_ops.alloc(ctx, (size_t)std::max<int64_t>(sp->n_po, 1)));
        MR_TRY(G->rs_off.alloc(ctx, (size_t)NT + 1));
        xs.g[k] = IxSide{B.tflag.p, B.ocnt.p, B.ofirst.p, B.ocov.p, B.tpos.p, B.zoff.p, B.gc.p};
        na.g[k] = NsArgs{B.gc.p, B.ocnt.p, B.ofirst.p, B.ocov.p, B.node_of_code.p, G->node_podop.p, G->len_o.p,
                         G->nchild.p, G->cov.p, G->ss_par.p, G->ss_off.p, B.tpos.p + NT, B.zoff.p + NT, G->rs_off.p,
                         d_out + 8 * k, nullptr, nullptr};
        to.g[k] = TrOut{G->trace_code.p, G->len_t.p, G->rs_ops.p, G->rs_off.p, B.node_of_code.p};
    }
    if (det) {   // the detector's states come out of the same launch (into det->state == d_state)
        const int64_t nt = std::max<int64_t>(cdiv((int64_t)NT, DB), 1);
        unsigned long long* dst = nullptr;
        uint64_t epoch = 0;
        MR_TRY(mr_dl_status(ctx, 4 * nt, &dst, &epoch));
        hipLaunchKernelGGL(k_ix_detect_scan2, dim3((unsigned)nt), dim3(DB), 0, st, *det, sp->po_off.p, NT, xs, dst,
                           epoch, NP, nek);
    } else {
        const int64_t nt = std::max<int64_t>(cdiv((int64_t)NT, SEL_TILE), 1);
        unsigned long long* dst = nullptr;
        uint64_t epoch = 0;
        MR_TRY(mr_dl_status(ctx, 4 * nt, &dst, &epoch));
        hipLaunchKernelGGL(k_ix_sel_scan2, dim3((unsigned)nt), dim3(SEL_T), 0, st, d_state, sp->tlen.p, sp->po_off.p,
                           NT, xs, dst, epoch, NP, nek);
    }
    if (NT) {
        constexpr int ix_cap = 256;   // block cap: one per CU
        const int nblk = std::max(1, std::min(ix_cap, cdiv(std::max(sp->n_po, sp->n_ed), IX_BT * IX_EPT)));
        const size_t lds = 2 * (3 * (size_t)NP + (size_t)nek) * sizeof(int32_t);
        hipLaunchKernelGGL(k_ix_stats2, dim3(nblk), dim3(IX_BT), lds, st, d_state, sp->n_po, sp->po_tr.p, sp->po_op.p,
                           sp->po_cnt.p, sp->po_first.p, sp->n_ed, sp->ed_tr.p, sp->ed_eid.p, sp->ed_cnt.p, NP,
                           (int32_t)nek, xs);
    }
    if (sp->n_xj)
        hipLaunchKernelGGL(k_ix_cross2, dim3(cdiv(sp->n_xj, 256)), dim3(256), 0, st, d_state, sp->xj_tc.p, sp->xj_tp.p,
                           sp->xj_eid.p, sp->n_xj, xs);
    hipLaunchKernelGGL(k_nodes_small2, dim3(2), dim3(NS_T), 0, st, sp->ekey.p, nek, NP, na);
    if (NT || sp->n_po)
        hipLaunchKernelGGL(k_ix_traces2, dim3(cdiv(std::max<int64_t>(NT, sp->n_po), 256)), dim3(256), 0, st, d_state, xs,
                           NT, sp->tlen.p, sp->n_po, sp->po_tr.p, sp->po_off.p, sp->po_op.p, to);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

// ---------------------------------------------------------------- the index pass of several windows
// A chunk of windows (mr_windows_batch builds 4 per auxiliary stream) in ONE launch per stage
// instead of one per window: the per-window chains of ~6 small, latency-bound launches ran back
// to back on the stream (a C2 chunk: 24 launches before its read-back), now 6.  Per stage the
// windows' arguments travel by value; a block finds its window by the launch's block offsets
// (windows without blocks in a stage repeat the next offset) and runs the single-window body with
// its index inside the window.
constexpr int IXW = 8;   // windows per batched launch
template <class A>
struct IxBatch {
    int32_t n;
    int32_t b0[IXW + 1];
    A w[IXW];
};
__device__ __forceinline__ int ixb_pick(const int32_t* b0, int32_t n) {
    const int32_t b = (int32_t)blockIdx.x;
    int k = 0;
    while (k + 1 < n && b0[k + 1] <= b) ++k;
    return k;
}
struct IxWinSel {
    DetIn d;   // (the detector-fused variant)
    const uint8_t* state;
    const int32_t* tlen;
    const int64_t* po_off;
    unsigned long long* st;   // this window's look-back status words (4 chains x its tiles)
    int64_t ecap;
    int32_t NT, NP;
    IxSide2 x;
};
struct IxWinStats {
    const uint8_t* state;
    const int32_t *po_tr, *po_op, *po_cnt, *po_first, *ed_tr, *ed_eid, *ed_cnt;
    int64_t n_po, n_ed;
    int32_t NP, n_ek;
    IxSide2 x;
};
struct IxWinCross {
    const uint8_t* state;
    const int32_t *tc, *tp, *eid;
    int64_t n;
    IxSide2 x;
};
struct IxWinNodes {
    const uint64_t* gk;
    int64_t ecap;
    int32_t NP, pad_;
    NsArgs2 a;
};
struct IxWinTraces {
    const uint8_t* state;
    const int32_t *tlen, *po_tr, *po_op;
    const int64_t* po_off;
    int64_t n_po;
    int32_t NT, pad_;
    IxSide2 x;
    TrOut2 o;
};
__global__ void __launch_bounds__(DB) k_ix_detect_b(IxBatch<IxWinSel> a) {
    __shared__ double term[DB * DCAP];
    const int k = ixb_pick(a.b0, a.n);
    (void)detect_block(a.w[k].NT, a.w[k].d, term, (int32_t)blockIdx.x - a.b0[k]);
}
__global__ void __launch_bounds__(SEL_T) k_ix_sel_scan2_b(IxBatch<IxWinSel> a, uint64_t epoch) {
    const int k = ixb_pick(a.b0, a.n);
    const IxWinSel& w = a.w[k];
    ix_sel_scan2_body(w.state, w.tlen, w.po_off, w.NT, w.x, w.st, epoch, w.NP, w.ecap, (int32_t)blockIdx.x - a.b0[k],
                      a.b0[k + 1] - a.b0[k]);
}
__global__ void __launch_bounds__(DB) k_ix_detect_scan2_b(IxBatch<IxWinSel> a, uint64_t epoch) {
    const int k = ixb_pick(a.b0, a.n);
    const IxWinSel& w = a.w[k];
    ix_detect_scan2_body(w.d, w.po_off, w.NT, w.x, w.st, epoch, w.NP, w.ecap, (int32_t)blockIdx.x - a.b0[k],
                         a.b0[k + 1] - a.b0[k]);
}
__global__ void __launch_bounds__(IX_BT) k_ix_stats2_b(IxBatch<IxWinStats> a) {
    const int k = ixb_pick(a.b0, a.n);
    const IxWinStats& w = a.w[k];
    ix_stats2_body(w.state, w.n_po, w.po_tr, w.po_op, w.po_cnt, w.po_first, w.n_ed, w.ed_tr, w.ed_eid, w.ed_cnt, w.NP,
                   w.n_ek, w.x, (int32_t)blockIdx.x - a.b0[k], a.b0[k + 1] - a.b0[k]);
}
__global__ void k_ix_cross2_b(IxBatch<IxWinCross> a) {
    const int k = ixb_pick(a.b0, a.n);
    const IxWinCross& w = a.w[k];
    const int64_t i = (int64_t)((int32_t)blockIdx.x - a.b0[k]) * blockDim.x + threadIdx.x;
    if (i >= w.n) return;
    const int sd = side_of(w.state[w.tc[i]]);
    if (sd >= 0 && side_of(w.state[w.tp[i]]) == sd) atomicAdd(&w.x.g[sd].gc[w.eid[i]], 1u);
}
__global__ void __launch_bounds__(NS_T) k_nodes_small2_b(IxBatch<IxWinNodes> a) {   // block 2k + g: window k, graph g
    const int k = (int)blockIdx.x >> 1;
    const IxWinNodes& w = a.w[k];
    const NsArgs& x = w.a.g[blockIdx.x & 1];
    nodes_small(w.gk, x.gc, w.ecap, x.ocnt, x.ofirst, w.NP, x.node_of_code, x.node_podop, x.len_o, x.nchild, x.ocov, x.cov,
                x.ss_par, x.ss_off, x.T_dev, x.nnz_dev, x.rs_off, x.out, x.u_o, x.pw, x.first_inv != 0);
}
__global__ void k_ix_traces2_b(IxBatch<IxWinTraces> a) {
    const int k = ixb_pick(a.b0, a.n);
    const IxWinTraces& w = a.w[k];
    const int64_t i = (int64_t)((int32_t)blockIdx.x - a.b0[k]) * blockDim.x + threadIdx.x;
    // (a trace is in graph sd iff its state's side is sd and it has rows -- the selection scan's
    // tflag, read from the state here: one gather less per entry; a trace with entries has rows)
    if (i < w.NT) {
        const int sd = side_of(w.state[i]);
        const int32_t len = w.tlen[i];
        if (sd >= 0 && len > 0) {
            const int32_t p = (int32_t)w.x.g[sd].tpos[i];
            w.o.g[sd].trace_code[p] = (int32_t)i;
            w.o.g[sd].len_t[p] = len;
            w.o.g[sd].rs_off[p] = w.x.g[sd].zoff[i];
        }
    }
    if (i < w.n_po) {
        const int32_t t = w.po_tr[i], op = w.po_op[i];
        const int sd = side_of(w.state[t]);
        if (sd >= 0) w.o.g[sd].rs_ops[w.x.g[sd].zoff[t] + (i - w.po_off[t])] = w.o.g[sd].node_of_code[op];
    }
}

// mr_ix_launch2 for n <= IXW windows at once (each: its table, state, graph pair, builds, size
// words); det: the windows' detector inputs -- fused into the selection launch (fuse) or a
// launch of their own before it.  MR_ERR_STATE: a window outside the one-pass limits (the caller
// then builds window by window).
int mr_ix_launch2_batch(mr_ctx* ctx, int n, const mr_spans* const* sps, uint8_t* const* d_states, mr_graph* const* g0s,
                        mr_graph* const* g1s, IxBuild* const* b0s, IxBuild* const* b1s, int64_t* const* d_outs,
                        const DetIn* dets, bool fuse) {
    if (n < 1 || n > IXW || getenv("MR_NO_IX2") != nullptr) return MR_ERR_STATE;
    for (int k = 0; k < n; ++k) {
        const mr_spans* sp = sps[k];
        if (!sp->ekey.p || sp->n_podops > NS_PMAX || 2 * (3 * (int64_t)sp->n_podops + sp->n_edge_keys) > IX_LDS_WORDS)
            return MR_ERR_STATE;
    }
    hipStream_t st = ctx->stream;
    IxBatch<IxWinSel> as{};
    IxBatch<IxWinStats> at{};
    const char* ee = getenv("MR_IX_EPT");   // (A/B knob, read per call)
    const int ept = ee ? std::max(1, atoi(ee)) : IX_EPT;   // (MR_IX_EPT forces it for every window)
    IxBatch<IxWinCross> ac{};
    IxBatch<IxWinNodes> an{};
    IxBatch<IxWinTraces> ar{};
    as.n = at.n = ac.n = an.n = ar.n = n;
    int32_t bs = 0, bt = 0, bc = 0, br = 0;
    size_t lds = 4;
    int64_t words = 0;
    std::vector<int64_t> woff((size_t)n);
    const int TP = fuse ? DB : SEL_TILE;   // traces per selection tile
    for (int k = 0; k < n; ++k) {
        const mr_spans* sp = sps[k];
        const int32_t NT = sp->n_traces, NP = sp->n_podops;
        const int64_t nek = sp->n_edge_keys;
        IxSide2 xs;
        NsArgs2 na;
        TrOut2 to;
        IxBuild* b[2] = {b0s[k], b1s[k]};
        mr_graph* g[2] = {g0s[k], g1s[k]};
        for (int j = 0; j < 2; ++j) {   // (mr_ix_launch2's buffers)
            IxBuild& B = *b[j];
            mr_graph* G = g[j];
            B.dense = true;
            B.small = true;
            B.ecap = (uint64_t)nek;
            B.gkp = sp->ekey.p;
            MR_TRY(B.tflag.alloc(ctx, std::max(NT, 1)));
            MR_TRY(B.tpos.alloc(ctx, (size_t)NT + 1));
            MR_TRY(B.zoff.alloc(ctx, (size_t)NT + 1));
            MR_TRY(B.ocnt.alloc(ctx, std::max(NP, 1)));
            MR_TRY(B.ofirst.alloc(ctx, std::max(NP, 1)));
            MR_TRY(B.ocov.alloc(ctx, std::max(NP, 1)));
            MR_TRY(B.gc.alloc(ctx, (size_t)std::max<int64_t>(nek, 1)));
            MR_TRY(B.node_of_code.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->node_podop.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->len_o.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->nchild.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->cov.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->ss_par.alloc(ctx, NS_EMAX));
            MR_TRY(G->ss_off.alloc(ctx, (size_t)NP + 1));
            MR_TRY(G->trace_code.alloc(ctx, std::max(NT, 1)));
            MR_TRY(G->len_t.alloc(ctx, std::max(NT, 1)));
            MR_TRY(G->rs_ops.alloc(ctx, (size_t)std::max<int64_t>(sp->n_po, 1)));
            MR_TRY(G->rs_off.alloc(ctx, (size_t)NT + 1));
            xs.g[j] = IxSide{B.tflag.p, B.ocnt.p, B.ofirst.p, B.ocov.p, B.tpos.p, B.zoff.p, B.gc.p};
            na.g[j] = NsArgs{B.gc.p, B.ocnt.p, B.ofirst.p, B.ocov.p, B.node_of_code.p, G->node_podop.p, G->len_o.p,
                             G->nchild.p, G->cov.p, G->ss_par.p, G->ss_off.p, B.tpos.p + NT, B.zoff.p + NT, G->rs_off.p,
                             d_outs[k] + 8 * j, nullptr, nullptr};
            to.g[j] = TrOut{G->trace_code.p, G->len_t.p, G->rs_ops.p, G->rs_off.p, B.node_of_code.p};
        }
        const int32_t nt = (int32_t)std::max<int64_t>(cdiv((int64_t)NT, TP), 1);
        woff[(size_t)k] = words;
        words += 4 * (int64_t)nt;
        as.b0[k] = bs;
        bs += nt;
        as.w[k] = IxWinSel{dets ? dets[k] : DetIn{}, d_states[k], sp->tlen.p, sp->po_off.p, nullptr, nek, NT, NP, xs};
        at.b0[k] = bt;
        const int64_t ne = std::max(sp->n_po, sp->n_ed);
        const int ek = ee ? ept : ne >= IX_EPT_BIG ? IX_EPT_BATCH : IX_EPT;
        if (NT) bt += std::max(1, std::min(256, cdiv(ne, (int64_t)IX_BT * ek)));
        lds = std::max(lds, 2 * (3 * (size_t)NP + (size_t)nek) * sizeof(int32_t));
        at.w[k] = IxWinStats{d_states[k], sp->po_tr.p, sp->po_op.p, sp->po_cnt.p, sp->po_first.p, sp->ed_tr.p, sp->ed_eid.p,
                             sp->ed_cnt.p, sp->n_po, sp->n_ed, NP, (int32_t)nek, xs};
        ac.b0[k] = bc;
        bc += (int32_t)cdiv(sp->n_xj, 256);
        ac.w[k] = IxWinCross{d_states[k], sp->xj_tc.p, sp->xj_tp.p, sp->xj_eid.p, sp->n_xj, xs};
        an.b0[k] = 2 * k;
        an.w[k] = IxWinNodes{sp->ekey.p, nek, NP, 0, na};
        ar.b0[k] = br;
        if (NT || sp->n_po) br += (int32_t)cdiv(std::max<int64_t>(NT, sp->n_po), 256);
        ar.w[k] = IxWinTraces{d_states[k], sp->tlen.p, sp->po_tr.p, sp->po_op.p, sp->po_off.p, sp->n_po, NT, 0, xs, to};
    }
    for (int k = n; k <= IXW; ++k) {   // (offsets past the last window: its end)
        if (k <= IXW) {
            as.b0[k] = bs;
            at.b0[k] = bt;
            ac.b0[k] = bc;
            an.b0[k] = 2 * n;
            ar.b0[k] = br;
        }
    }
    unsigned long long* dst = nullptr;
    uint64_t epoch = 0;
    MR_TRY(mr_dl_status(ctx, words, &dst, &epoch));
    for (int k = 0; k < n; ++k) as.w[k].st = dst + woff[(size_t)k];
    if (fuse) {
        hipLaunchKernelGGL(k_ix_detect_scan2_b, dim3(bs), dim3(DB), 0, st, as, epoch);
    } else {
        if (dets) {
            int32_t bd = 0;   // the detector's own launch: DB traces per block
            IxBatch<IxWinSel> ad = as;
            for (int k = 0; k < n; ++k) {
                ad.b0[k] = bd;
                bd += (int32_t)cdiv((int64_t)sps[k]->n_traces, DB);
            }
            for (int k = n; k <= IXW; ++k) ad.b0[k] = bd;
            if (bd) hipLaunchKernelGGL(k_ix_detect_b, dim3(bd), dim3(DB), 0, st, ad);
        }
        hipLaunchKernelGGL(k_ix_sel_scan2_b, dim3(bs), dim3(SEL_T), 0, st, as, epoch);
    }
    if (bt) hipLaunchKernelGGL(k_ix_stats2_b, dim3(bt), dim3(IX_BT), lds, st, at);
    if (bc) hipLaunchKernelGGL(k_ix_cross2_b, dim3(bc), dim3(256), 0, st, ac);
    hipLaunchKernelGGL(k_nodes_small2_b, dim3(2 * n), dim3(NS_T), 0, st, an);
    if (br) hipLaunchKernelGGL(k_ix_traces2_b, dim3(br), dim3(256), 0, st, ar);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

// ---------------------------------------------------------------- window graphs in layout order
// A window's graphs tile their traces in the table's layout order (mr_spans.lo_*: by distinct
// pod-op count, then code -- window-independent, built with the index).  The selection runs over
// that order: each selected trace's position in its graph is its rank among the graph's traces
// there (look-back scan), pinv[position] = its layout index, and its kind class is counted
// (pagerank.py:54-66's class size = the histogram of the graph's class ids).  No trace-major
// incidence, no per-graph sort by length, no kind hashing: the prepare reads each position's
// codes from the layout-ordered u16 lists (near-contiguous for a tile) and relabels them.
constexpr int LB_T = 512;                  // k_lo_build_b threads (a block: a layout range of mr_spans.lo_bstart)
constexpr int64_t LB_LDS_WORDS = 30720;   // its two graphs' histograms and the service-op thresholds (120 KB)
constexpr int32_t LB_A3MAX = 4096;        // service-op thresholds in LDS (8 B each)
bool mr_lo_fits(const mr_spans* sp) {
    return sp->indexed && sp->ekey.p && sp->n_podops <= NS_PMAX && sp->n_edge_keys <= NS_EMAX &&
           2 * (3 * (int64_t)sp->n_podops + sp->n_edge_keys) + 2 * (int64_t)sp->n_svcops <= LB_LDS_WORDS &&
           sp->n_svcops <= LB_A3MAX && sp->n_traces <= (1 << 24);
}
// Per window, in its table's layout order: the detector (anormaly_detector.py:44-84 as
// detect_block: a trace's expect summed sequentially over its service-ops in name order, T14),
// the selection of both graphs (T1 swap: state 2 -> graph 0, 1 -> graph 1: a side byte per layout
// index, k_lo_pos_b's input) and each class's count, and both graphs' per-pod-op span counts /
// first rows / coverage and per-edge-id multiplicities (get_pagerank_graph's len_o, node order
// and children multisets, preprocess_data.py:146-171) in LDS, written once per block as a partial
// row (the first row as INT_MAX - row, combined by max) that k_lo_reduce_b combines per window.
// A block is a layout range of at most LO_BT_MAX traces and LO_BE entries (mr_spans.lo_bstart):
// a thread per trace for the detector, then every wave of the block over the range's entries (a
// lane per entry, coalesced, four rounds of loads in flight), each entry's trace found from the
// traces' starts in LDS.  No block waits for another.
struct IxWinLoB {
    const int32_t *lo_tr, *lo_len, *lo_kid, *lo_first, *bstart;
    const int64_t *lo_off, *lsv_off, *le_off;
    const uint16_t *lo16, *lo_cnt;
    const uint32_t *lsv, *le;
    const long long *lo_ts, *lo_te, *lo_mx;
    const double* a3;
    const uint8_t* a3v;
    int64_t t0, t1;
    uint8_t* state;                  // by trace code (k_ix_cross2_b reads it)
    int8_t* side;                    // by layout index: 0 / 1 graph, -1 none
    unsigned long long* counts;      // detector counter shards (3 * CSH, zeroed)
    int32_t NT, NP, nek, nsvc;
    uint32_t* kcnt[2];               // kind class histograms (zeroed)
    int64_t* tot[2];                 // [T, nnz] (zeroed)
    uint32_t* rows;                  // partial rows [block][graph][cnt NP | cov NP | INT_MAX - first NP | edges nek]
};
// the build's first LDS region: both graphs' histograms, and before them (aliased) the detector's
// products of a round -- at least 2048 of them
__host__ __device__ __forceinline__ size_t lo_region0(size_t gbytes) {
    return 2 * gbytes > (size_t)2048 * 8 ? 2 * gbytes : (size_t)2048 * 8;
}
constexpr int LB_R = 4;   // entry rounds per batch (their loads in flight together)
// the block-relative trace whose entries [st[t], st[t+1]) hold entry e (st ascending, st[0] = 0,
// st[nt] = the range's entries): a division when the range's traces all have n entries (the layout
// sorts by entry count: the usual case), else a binary search in LDS
__device__ __forceinline__ int32_t lo_trace_of(uint32_t e, uint32_t n, const uint32_t* st, int32_t nt) {
    if (n > 0) return (int32_t)(e / n);
    // a fixed number of steps (LO_BT_MAX = 1024 traces): the searches of a batch's rounds are
    // independent chains the compiler can interleave (a data-dependent loop would run them one by one)
    int32_t lo = 0;
#pragma unroll
    for (int32_t step = LO_BT_MAX / 2; step >= 1; step >>= 1) {
        const int32_t mid = lo + step;
        lo = mid < nt && st[mid] <= e ? mid : lo;
    }
    return lo;
}
__global__ void __launch_bounds__(LB_T, 6) k_lo_build_b(IxBatch<IxWinLoB> a) {
    // per graph g: [cnt | cov << 32] u64 x NP, then INT_MAX - first row x NP, then edge counts x
    // nek; then the service-op thresholds (0 where a3v is false: adding +0.0 leaves expect as is)
    extern __shared__ __attribute__((aligned(16))) unsigned char lraw[];
    __shared__ uint32_t pst[LO_BT_MAX + 1], est[LO_BT_MAX + 1];   // the traces' first entries (relative)
    __shared__ int8_t ss[LO_BT_MAX];
    __shared__ unsigned long long bc[5][LB_T / WAVE];
    const int k = ixb_pick(a.b0, a.n);
    const IxWinLoB& w = a.w[k];
    const int32_t blk = (int32_t)blockIdx.x - a.b0[k];
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
    const int32_t NP = w.NP, nek = w.nek;
    const size_t gbytes = ((size_t)NP * 12 + (size_t)nek * 4 + 15) / 16 * 16;   // one graph's histograms
    const size_t reg0 = lo_region0(gbytes);   // the histograms; before them, the detector's products
    double* la3 = (double*)(lraw + reg0);
    double* prod = (double*)lraw;
    const uint32_t cap = (uint32_t)(reg0 / 8 / LB_T * LB_T);   // products per round
    for (int32_t c = tid; c < w.nsvc; c += LB_T) la3[c] = w.a3v[c] ? w.a3[c] : 0.0;
    const int32_t T0 = w.bstart[blk], nt = w.bstart[blk + 1] - T0;
    const int64_t P0 = w.lo_off[T0], Q0 = w.le_off[T0], V0 = w.lsv_off[T0];
    const uint32_t np = (uint32_t)(w.lo_off[T0 + nt] - P0), nq = (uint32_t)(w.le_off[T0 + nt] - Q0);
    const uint32_t nv = (uint32_t)(w.lsv_off[T0 + nt] - V0);
    if (tid == 0) {
        pst[nt] = np;
        est[nt] = nq;
    }
    // this thread's traces: slot s holds trace s * LB_T + tid of the range (64 consecutive per wave)
    constexpr int NS = LO_BT_MAX / LB_T;
    uint32_t va[NS], vb[NS];
    bool act[NS];
    double expect[NS];
    long long mx[NS];
    unsigned long long rows = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int32_t t = q * LB_T + tid;
        const bool valid = t < nt;
        const int64_t i = (int64_t)T0 + (valid ? t : nt - 1);   // (clamped)
        const int32_t len = w.lo_len[i];
        const long long ts = w.lo_ts[i], te = w.lo_te[i];
        mx[q] = w.lo_mx[i];
        va[q] = (uint32_t)(w.lsv_off[i] - V0);
        vb[q] = (uint32_t)(w.lsv_off[i + 1] - V0);
        const bool in = valid && len > 0 && ts >= w.t0 && te <= w.t1;
        rows += in ? (unsigned long long)len : 0ull;
        act[q] = in && mx[q] > 0;   // grouped[grouped['duration'] > 0] (preprocess_data.py:117)
        expect[q] = 0.0;
    }
    __syncthreads();   // (the thresholds in LDS)
    // the detector's expect (anormaly_detector.py:63-67), sequential in name order per trace (T14):
    // the range's service-op products staged in LDS a round at a time (coalesced loads, every load of
    // a round in flight), each lane then adding its own trace's products of the round in order --
    // the same products, the same sequential sums as a lane walking its trace alone
    for (uint32_t r0 = 0; r0 < nv; r0 += cap) {
        const uint32_t rn = min(cap, nv - r0);
        constexpr int LU = 8;
        for (uint32_t x0 = 0; x0 < rn; x0 += LU * LB_T) {
            uint32_t v[LU];
#pragma unroll
            for (int u = 0; u < LU; ++u) {
                const uint32_t x = x0 + (uint32_t)(u * LB_T + tid);
                v[u] = w.lsv[V0 + (int64_t)(r0 + min(x, rn - 1))];
            }
#pragma unroll
            for (int u = 0; u < LU; ++u) {
                const uint32_t x = x0 + (uint32_t)(u * LB_T + tid);
                if (x < rn) prod[x] = (double)(v[u] >> 16) * la3[v[u] & 0xffffu];
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NS; ++q)
            if (act[q]) {
                const uint32_t lo = max(va[q], r0), hi = min(vb[q], r0 + rn);
                for (uint32_t j = lo; j < hi; j += 8) {   // eight LDS reads in flight, then the adds in order
                    double p8[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) p8[u] = prod[min(j + u, hi - 1) - r0];
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (j + u < hi) expect[q] += p8[u];
                }
            }
        __syncthreads();
    }
    for (size_t x = (size_t)tid * 4; x < reg0; x += (size_t)LB_T * 4) *(uint32_t*)(lraw + x) = 0u;
    unsigned long long nab = 0, nno = 0, nz0 = 0, nz1 = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int32_t t = q * LB_T + tid;
        const bool valid = t < nt;
        const int64_t i = (int64_t)T0 + (valid ? t : nt - 1);   // (clamped)
        const int32_t kid0 = w.lo_kid[i], tr = w.lo_tr[i];
        const int64_t pa = w.lo_off[i], pb = w.lo_off[i + 1], ea = w.le_off[i];
        const int stt = act[q] ? ((double)mx[q] / 1000.0 > expect[q] ? 2 : 1) : 0;   // :58, :69
        const int s_ = valid ? (stt == 2 ? 0 : stt == 1 ? 1 : -1) : -1;
        if (valid) {
            w.state[tr] = (uint8_t)stt;
            w.side[i] = (int8_t)s_;
            ss[t] = (int8_t)s_;
            pst[t] = (uint32_t)(pa - P0);
            est[t] = (uint32_t)(ea - Q0);
        }
        nab += stt == 2;
        nno += stt == 1;
        if (s_ == 0) nz0 += (unsigned long long)(pb - pa);
        else if (s_ == 1) nz1 += (unsigned long long)(pb - pa);
        // kind classes are runs of the layout: one add per (run, graph) of the wave
        const int kid = valid ? kid0 : -1;
        const int kp = __shfl_up(kid, 1, WAVE);
        const bool hd = kid >= 0 && (lane == 0 || kp != kid);
        const unsigned long long H = __ballot(hd), B0 = __ballot(s_ == 0), B1 = __ballot(s_ == 1);
        if (hd) {
            const unsigned long long above = lane == WAVE - 1 ? 0ull : H & (~0ull << (lane + 1));
            const unsigned long long run = (above ? (above & (0ull - above)) - 1ull : ~0ull) & (~0ull << lane);
            const uint32_t c0 = (uint32_t)__popcll(B0 & run), c1 = (uint32_t)__popcll(B1 & run);
            if (c0) atomicAdd(&w.kcnt[0][kid], c0);
            if (c1) atomicAdd(&w.kcnt[1][kid], c1);
        }
    }
    __syncthreads();
    // the range's pod-op and join entries, each to its trace's graph.  A range of short traces (the
    // longest -- the layout sorts by count, so the last -- of <= LB_LANE pod-ops): a lane per trace
    // walks its own entries, all loads out at once, no lookups, each trace's entries rotated by its
    // index (a run of identical traces would otherwise add into the same word in the same round).
    // Else every wave over the range's entries, a lane per entry, the entry's trace looked up.
    constexpr int LB_LANE = 8;
    const bool lanewise = nt > 0 && pst[nt] - pst[nt - 1] <= (uint32_t)LB_LANE;
    if (lanewise) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int32_t t = q * LB_T + tid;
            const int sd = t < nt ? (int)ss[t] : -1;
            if (sd < 0) continue;
            unsigned char* G = lraw + (size_t)sd * gbytes;
            const uint32_t a0 = pst[t], n = pst[t + 1] - a0, rot = n ? (uint32_t)t % n : 0u;
            uint32_t pc[LB_LANE];
            int32_t fr[LB_LANE];
#pragma unroll
            for (int u = 0; u < LB_LANE; ++u) {
                const uint32_t j = (uint32_t)u + rot;
                const int64_t e = P0 + (int64_t)a0 + (u < (int)n ? (j >= n ? j - n : j) : 0u);
                pc[u] = (uint32_t)w.lo16[e] | ((uint32_t)w.lo_cnt[e] << 16);
                fr[u] = w.lo_first[e];
            }
#pragma unroll
            for (int u = 0; u < LB_LANE; ++u)
                if (u < (int)n) {
                    const uint32_t c = pc[u] & 0xffffu;
                    atomicAdd((unsigned long long*)G + c, (unsigned long long)(pc[u] >> 16) | (1ull << 32));
                    atomicMax((int32_t*)(G + (size_t)NP * 8) + c, 0x7fffffff - fr[u]);
                }
            const uint32_t b0e = est[t], m = est[t + 1] - b0e, rte = m ? (uint32_t)t % m : 0u;
            uint32_t* Ge = (uint32_t*)(G + (size_t)NP * 12);
            for (uint32_t u0 = 0; u0 < m; u0 += LB_LANE) {
                uint32_t ev[LB_LANE];
#pragma unroll
                for (int u = 0; u < LB_LANE; ++u) {
                    const uint32_t j = u0 + (uint32_t)u, jr = j + rte;
                    ev[u] = w.le[Q0 + (int64_t)b0e + (j < m ? (jr >= m ? jr - m : jr) : 0u)];
                }
#pragma unroll
                for (int u = 0; u < LB_LANE; ++u)
                    if (u0 + (uint32_t)u < m) atomicAdd(Ge + (ev[u] & 0xffffu), ev[u] >> 16);
            }
        }
    }
    const uint32_t n0 = nt ? pst[1 < nt ? 1 : nt] - pst[0] : 0u;
    const uint32_t npo = n0 > 0 && np == (uint32_t)nt * n0 ? n0 : 0u;   // (uniform: every trace n0 entries)
    constexpr int NW = LB_T / WAVE;
    const uint32_t nmax = lanewise ? 0u : max(np, nq);
    for (uint32_t b0 = (uint32_t)wv * (LB_R * WAVE); b0 < nmax; b0 += NW * LB_R * WAVE) {
        uint32_t pc[LB_R], ev[LB_R];
        int32_t fr[LB_R];
#pragma unroll
        for (int r = 0; r < LB_R; ++r) {   // (clamped: every load in bounds)
            const uint32_t o = b0 + (uint32_t)(r * WAVE + lane);
            if (b0 < np) {
                const int64_t e = P0 + (int64_t)min(o, np - 1u);
                pc[r] = (uint32_t)w.lo16[e] | ((uint32_t)w.lo_cnt[e] << 16);
                fr[r] = w.lo_first[e];
            }
            if (b0 < nq) ev[r] = w.le[Q0 + (int64_t)min(o, nq - 1u)];
        }
#pragma unroll
        for (int r = 0; r < LB_R; ++r) {
            const uint32_t o = b0 + (uint32_t)(r * WAVE + lane);
            if (o < np) {
                const int sd = ss[lo_trace_of(o, npo, pst, nt)];
                if (sd >= 0) {
                    unsigned char* G = lraw + (size_t)sd * gbytes;
                    const uint32_t c = pc[r] & 0xffffu;
                    atomicAdd((unsigned long long*)G + c, (unsigned long long)(pc[r] >> 16) | (1ull << 32));
                    atomicMax((int32_t*)(G + (size_t)NP * 8) + c, 0x7fffffff - fr[r]);
                }
            }
            if (o < nq) {
                const int sd = ss[lo_trace_of(o, 0u, est, nt)];
                if (sd >= 0)
                    atomicAdd((uint32_t*)(lraw + (size_t)sd * gbytes + (size_t)NP * 12) + (ev[r] & 0xffffu), ev[r] >> 16);
            }
        }
    }
    __syncthreads();
    {   // the detector's counts and both graphs' entry totals: per wave, per block, one add each
        unsigned long long v[5] = {nab, nno, rows, nz0, nz1};
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
            for (int q = 0; q < 5; ++q) v[q] += __shfl_xor(v[q], m, WAVE);
        if (lane == 0)
#pragma unroll
            for (int q = 0; q < 5; ++q) bc[q][wv] = v[q];
    }
    __syncthreads();
    if (tid < 5) {
        unsigned long long v = 0;
        for (int q = 0; q < NW; ++q) v += bc[tid][q];
        if (v) {
            if (tid < 3) atomicAdd(&w.counts[(size_t)(blk % CSH) * 3 + tid], v);
            else atomicAdd((unsigned long long*)&w.tot[tid - 3][1], v);
        }
    }
    // the block's histograms as its partial row (plain stores; k_lo_reduce_b combines the rows)
    const size_t rw = 3 * (size_t)NP + (size_t)nek;
    uint32_t* R = w.rows + (size_t)blk * 2 * rw;
    for (int g = 0; g < 2; ++g) {
        const unsigned char* G = lraw + (size_t)g * gbytes;
        uint32_t* Rg = R + (size_t)g * rw;
        for (int32_t c = tid; c < NP; c += LB_T) {
            const unsigned long long v = ((const unsigned long long*)G)[c];
            Rg[c] = (uint32_t)v;
            Rg[NP + c] = (uint32_t)(v >> 32);
            Rg[2 * NP + c] = ((const uint32_t*)(G + (size_t)NP * 8))[c];
        }
        for (int32_t x = tid; x < nek; x += LB_T) Rg[3 * NP + x] = ((const uint32_t*)(G + (size_t)NP * 12))[x];
    }
    __syncthreads();
}
// positions: each selected trace's rank among its graph's traces in layout order (decoupled
// look-back over the side bytes), pinv[position] = layout index, staged in LDS for coalesced
// stores; the graph sizes tot[g][0]
constexpr int LP_T = 256, LP_I = 16, LP_TILE = LP_T * LP_I;
struct IxWinLoPos {
    const int8_t* side;
    int32_t NT, pad_;
    unsigned long long* st;          // look-back words: 2 chains x the window's tiles
    int32_t* pinv[2];
    int64_t* tot[2];
};
__global__ void __launch_bounds__(LP_T) k_lo_pos_b(IxBatch<IxWinLoPos> a, uint64_t epoch) {
    __shared__ int32_t sa[2][LP_T];
    __shared__ int32_t ex[2];
    __shared__ int32_t so[2][LP_TILE];
    const int k = ixb_pick(a.b0, a.n);
    const IxWinLoPos& w = a.w[k];
    const int32_t blk = (int32_t)blockIdx.x - a.b0[k], nblk = a.b0[k + 1] - a.b0[k];
    const int tid = threadIdx.x, lane = tid & (WAVE - 1);
    const int64_t base = (int64_t)blk * LP_TILE + (int64_t)tid * LP_I;
    int8_t sd[LP_I];
    if (base + LP_I <= w.NT) {   // 16 side bytes: one load
        const uint4 v = *(const uint4*)(w.side + base);
        memcpy(sd, &v, 16);
    } else {
#pragma unroll
        for (int q = 0; q < LP_I; ++q) sd[q] = base + q < w.NT ? w.side[base + q] : (int8_t)-1;
    }
    int32_t c0 = 0, c1 = 0;
#pragma unroll
    for (int q = 0; q < LP_I; ++q) {
        c0 += sd[q] == 0;
        c1 += sd[q] == 1;
    }
    sa[0][tid] = c0;
    sa[1][tid] = c1;
    __syncthreads();
    for (int o = 1; o < LP_T; o <<= 1) {
        const int32_t v0 = tid >= o ? sa[0][tid - o] : 0, v1 = tid >= o ? sa[1][tid - o] : 0;
        __syncthreads();
        sa[0][tid] += v0;
        sa[1][tid] += v1;
        __syncthreads();
    }
    if (tid < 2 * WAVE) {   // wave g: graph g's positions
        const int g = tid / WAVE;
        const int32_t agg = sa[g][LP_T - 1];
        const int64_t e = dl_lookback_wave(w.st + (size_t)g * nblk, blk, agg, epoch);
        if (lane == 0) {
            ex[g] = (int32_t)e;
            if (blk == nblk - 1) w.tot[g][0] = e + agg;
        }
    }
    int32_t r0 = sa[0][tid] - c0, r1 = sa[1][tid] - c1;   // (block-relative)
#pragma unroll
    for (int q = 0; q < LP_I; ++q) {
        const int32_t ix = (int32_t)(base + q);
        if (sd[q] == 0) so[0][r0++] = ix;
        else if (sd[q] == 1) so[1][r1++] = ix;
    }
    __syncthreads();
    for (int g = 0; g < 2; ++g) {
        const int32_t n = sa[g][LP_T - 1], e = ex[g];
        for (int32_t x = tid; x < n; x += LP_T) w.pinv[g][e + x] = so[g][x];
    }
}
// each window's partial rows, column by column: span counts, coverage and edge multiplicities
// summed, INT_MAX - first row by max -- into the graph's words (overwritten; k_ix_cross2_b adds
// the joins across traces after)
struct IxLoRed {
    const uint32_t* rows;
    int32_t nblk, NP, nek, pad_;
    int32_t *ocnt[2], *ofinv[2], *ocov[2];
    uint32_t* gc[2];
};
__global__ void __launch_bounds__(256) k_lo_reduce_b(IxBatch<IxLoRed> a) {
    const int k = ixb_pick(a.b0, a.n);
    const IxLoRed& w = a.w[k];
    const int64_t rw = 3 * (int64_t)w.NP + w.nek;
    const int64_t col = (int64_t)((int32_t)blockIdx.x - a.b0[k]) * 256 + threadIdx.x;
    if (col >= 2 * rw) return;
    const int g = (int)(col / rw);
    const int64_t c = col - (int64_t)g * rw;
    const bool mx = c >= 2 * (int64_t)w.NP && c < 3 * (int64_t)w.NP;
    const uint32_t* p = w.rows + col;
    const size_t stride = 2 * (size_t)rw;
    uint32_t acc = 0;
    int32_t b = 0;
    for (; b + 8 <= w.nblk; b += 8) {
        uint32_t v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = p[(size_t)(b + q) * stride];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = mx ? max(acc, v[q]) : acc + v[q];
    }
    for (; b < w.nblk; ++b) {
        const uint32_t v = p[(size_t)b * stride];
        acc = mx ? max(acc, v) : acc + v;
    }
    const int32_t NP = w.NP;
    if (c < NP) w.ocnt[g][c] = (int32_t)acc;
    else if (c < 2 * (int64_t)NP) w.ocov[g][c - NP] = (int32_t)acc;
    else if (c < 3 * (int64_t)NP) w.ofinv[g][c - 2 * NP] = (int32_t)acc;
    else w.gc[g][c - 3 * NP] = acc;
}

// Per window (n <= IXW): k_lo_build_b, the rare joins across traces, the node order / P_ss / op
// constants (k_nodes_small2_b): sizes of graph j of window k to d_outs[k] + 8 j (N, E, overflow,
// T, nnz; words 5 / 6: the build's totals).  zw[k]: the window's zeroed words, lo_zero_words(sp)
// of them.  MR_ERR_STATE: a window outside the limits (the caller takes mr_ix_launch2_batch).
int64_t mr_lo_zero_words(const mr_spans* sp) {
    return 2 * ((int64_t)std::max(sp->lo_nk, 1) + 3 * (int64_t)sp->n_podops + std::max<int64_t>(sp->n_edge_keys, 1));
}
int mr_lo_launch_batch(mr_ctx* ctx, int n, const mr_spans* const* sps, mr_graph* const* g0s, mr_graph* const* g1s,
                       IxBuild* const* b0s, IxBuild* const* b1s, int64_t* const* d_outs, const DetIn* dets,
                       uint32_t* const* zw) {
    if (n < 1 || n > IXW || getenv("MR_NO_IX2") != nullptr) return MR_ERR_STATE;
    for (int k = 0; k < n; ++k)
        if (!sps[k]->lo_ok || !mr_lo_fits(sps[k])) return MR_ERR_STATE;
    hipStream_t st = ctx->stream;
    IxBatch<IxWinLoB> ab{};
    IxBatch<IxLoRed> ar{};
    IxBatch<IxWinLoPos> ap{};
    IxBatch<IxWinCross> ac{};
    IxBatch<IxWinNodes> an{};
    ab.n = ar.n = ap.n = ac.n = an.n = n;
    int32_t bb = 0, bc = 0, br = 0, bp = 0;
    int64_t rwords = 0, sbytes = 0;
    std::vector<int64_t> roff((size_t)n), soff((size_t)n);
    size_t lds = 4;
    int64_t words = 0;
    std::vector<int64_t> woff((size_t)n);
    for (int k = 0; k < n; ++k) {
        const mr_spans* sp = sps[k];
        const int32_t NT = sp->n_traces, NP = sp->n_podops;
        const int64_t nek = sp->n_edge_keys, nk = std::max(sp->lo_nk, 1);
        IxSide2 xs;
        NsArgs2 na;
        IxBuild* b[2] = {b0s[k], b1s[k]};
        mr_graph* g[2] = {g0s[k], g1s[k]};
        IxWinLoB& L = ab.w[k];
        const int64_t per = nk + 3 * (int64_t)NP + std::max<int64_t>(nek, 1);   // zeroed words per graph
        for (int j = 0; j < 2; ++j) {
            IxBuild& B = *b[j];
            mr_graph* G = g[j];
            B.dense = true;
            B.small = true;
            B.ecap = (uint64_t)nek;
            B.gkp = sp->ekey.p;
            uint32_t* z = zw[k] + j * per;
            B.kcnt = z;
            int32_t* ocnt = (int32_t*)(z + nk);
            int32_t* ofinv = ocnt + NP;
            int32_t* ocov = ofinv + NP;
            uint32_t* gc = (uint32_t*)(ocov + NP);
            MR_TRY(B.pinv.alloc(ctx, std::max(NT, 1)));
            MR_TRY(B.node_of_code.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->node_podop.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->len_o.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->nchild.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->cov.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->u_o.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->pw.alloc(ctx, std::max(NP, 1)));
            MR_TRY(G->ss_par.alloc(ctx, NS_EMAX));
            MR_TRY(G->ss_off.alloc(ctx, (size_t)NP + 1));
            xs.g[j] = IxSide{nullptr, ocnt, ofinv, ocov, nullptr, nullptr, gc};
            int64_t* out = d_outs[k] + 8 * j;
            na.g[j] = NsArgs{gc, ocnt, ofinv, ocov, B.node_of_code.p, G->node_podop.p, G->len_o.p, G->nchild.p, G->cov.p,
                             G->ss_par.p, G->ss_off.p, out + 5, out + 6, nullptr, out, G->u_o.p, G->pw.p, 1};
            ap.w[k].pinv[j] = B.pinv.p;
            ap.w[k].tot[j] = out + 5;
            L.kcnt[j] = B.kcnt;
            L.tot[j] = out + 5;
            IxLoRed& R = ar.w[k];
            R.ocnt[j] = ocnt;
            R.ofinv[j] = ofinv;
            R.ocov[j] = ocov;
            R.gc[j] = gc;
        }
        const int32_t nt = sp->lo_nblk;
        const int64_t rw = 3 * (int64_t)NP + nek;
        roff[(size_t)k] = rwords;
        rwords += (int64_t)nt * 2 * rw;
        ar.w[k].nblk = nt;
        ar.w[k].NP = NP;
        ar.w[k].nek = (int32_t)nek;
        ar.b0[k] = br;
        br += (int32_t)cdiv(2 * rw, 256);
        const int32_t npb = (int32_t)std::max<int64_t>(cdiv((int64_t)NT, LP_TILE), 1);
        woff[(size_t)k] = words;
        words += 2 * (int64_t)npb;
        ap.b0[k] = bp;
        bp += npb;
        ap.w[k].NT = NT;
        soff[(size_t)k] = sbytes;
        sbytes += ((int64_t)NT + 15) / 16 * 16;
        ab.b0[k] = bb;
        bb += nt;
        const DetIn& d = dets[k];
        L.bstart = sp->lo_bstart.p;
        L.lo_tr = sp->lo_tr.p;
        L.lo_len = sp->lo_len.p;
        L.lo_kid = sp->lo_kid.p;
        L.lo_first = sp->lo_first.p;
        L.lo_off = sp->lo_off.p;
        L.lsv_off = sp->lsv_off.p;
        L.le_off = sp->le_off.p;
        L.lo16 = sp->lo16.p;
        L.lo_cnt = sp->lo_cnt.p;
        L.lsv = sp->lsv.p;
        L.le = sp->le.p;
        L.lo_ts = sp->lo_ts.p;
        L.lo_te = sp->lo_te.p;
        L.lo_mx = sp->lo_mx.p;
        L.a3 = d.a3;
        L.a3v = d.a3v;
        L.t0 = d.t0;
        L.t1 = d.t1;
        L.state = d.state;
        L.counts = d.counts;
        L.NT = NT;
        L.NP = NP;
        L.nek = (int32_t)nek;
        L.nsvc = sp->n_svcops;
        lds = std::max(lds, lo_region0(((size_t)NP * 12 + (size_t)nek * 4 + 15) / 16 * 16) + (size_t)sp->n_svcops * 8);
        ac.b0[k] = bc;
        bc += (int32_t)cdiv(sp->n_xj, 256);
        ac.w[k] = IxWinCross{d.state, sp->xj_tc.p, sp->xj_tp.p, sp->xj_eid.p, sp->n_xj, xs};
        an.b0[k] = 2 * k;
        an.w[k] = IxWinNodes{sp->ekey.p, nek, NP, 0, na};
    }
    for (int k = n; k <= IXW; ++k) {   // (offsets past the last window: its end)
        ab.b0[k] = bb;
        ar.b0[k] = br;
        ap.b0[k] = bp;
        ac.b0[k] = bc;
        an.b0[k] = 2 * n;
    }
    unsigned long long* dst = nullptr;
    uint64_t epoch = 0;
    MR_TRY(mr_dl_status(ctx, words, &dst, &epoch));
    DBuf<uint32_t> rows;   // (stream-ordered: freed back to this context's pool after the launches)
    DBuf<int8_t> side;
    MR_TRY(rows.alloc(ctx, (size_t)std::max<int64_t>(rwords, 1)));
    MR_TRY(side.alloc(ctx, (size_t)std::max<int64_t>(sbytes, 16)));
    for (int k = 0; k < n; ++k) {
        ab.w[k].rows = rows.p + roff[(size_t)k];
        ar.w[k].rows = rows.p + roff[(size_t)k];
        ab.w[k].side = side.p + soff[(size_t)k];
        ap.w[k].side = side.p + soff[(size_t)k];
        ap.w[k].st = dst + woff[(size_t)k];
    }
    hipLaunchKernelGGL(k_lo_build_b, dim3(bb), dim3(LB_T), lds, st, ab);
    hipLaunchKernelGGL(k_lo_pos_b, dim3(bp), dim3(LP_T), 0, st, ap, epoch);
    hipLaunchKernelGGL(k_lo_reduce_b, dim3(br), dim3(256), 0, st, ar);
    if (bc) hipLaunchKernelGGL(k_ix_cross2_b, dim3(bc), dim3(256), 0, st, ac);
    hipLaunchKernelGGL(k_nodes_small2_b, dim3(2 * n), dim3(NS_T), 0, st, an);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

int mr_ix_launch(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_mask, mr_graph* g, IxBuild& b, int64_t* d_out) {
    return ix_launch(ctx, sp, d_mask, g, b, d_out, false);
}
int mr_ix_finish(mr_ctx* ctx, const mr_spans* sp, mr_graph* g, IxBuild& b, const int64_t* h) {
    MR_TRY(ix_finish(ctx, sp, g, b, h, false));
    return mr_graph_post_build(ctx, g);
}
int mr_ix_finish_unprepared(mr_ctx* ctx, const mr_spans* sp, mr_graph* g, IxBuild& b, const int64_t* h) {
    MR_TRY(ix_finish(ctx, sp, g, b, h, false));
    g->rs_is_sr = true;   // (mr_graph_post_build's fields)
    g->pr_identity = true;
    g->n_pr = g->T;
    return MR_OK;
}

// a built graph's trace-role fields and derived arrays (the K1 result is P_rs = P_sr)
int mr_graph_post_build(mr_ctx* ctx, mr_graph* g) {
    g->rs_is_sr = true;
    g->pr_identity = true;
    g->n_pr = g->T;
    PhaseTimer pt(ctx->stream, "prepare");
    MR_TRY(mr_graph_prepare(ctx, g));
    pt.mark("done");
    return MR_OK;
}

// win (nullable): [t0, t1] restricts rows to the time window on the row-level path; the indexed
// path is taken only when the window selects whole traces (uniform trace times) or is absent.
int mr_graph_build_dev(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_mask, mr_graph** out, const int64_t* win) {
    auto g = new mr_graph();
    g->ctx = ctx;
    static const bool no_index = getenv("MR_NO_INDEX") != nullptr;   // A/B knob: force the row-level path
    const bool indexed = sp->indexed && !no_index && (!win || sp->uniform_times);
    int rc = indexed ? graph_build_indexed(ctx, sp, d_mask, g) : graph_build_rows(ctx, sp, d_mask, win, g);
    if (rc == MR_OK) rc = mr_graph_post_build(ctx, g);
    if (rc != MR_OK) {
        delete g;
        return rc;
    }
    *out = g;
    return MR_OK;
}

extern "C" int mr_graph_build(mr_ctx* ctx, const mr_spans* sp, const uint8_t* trace_mask, mr_graph** out) {
    if (!ctx || !sp || !trace_mask || !out || sp->ctx != ctx) return mr_fail(ctx, MR_ERR_ARG, "mr_graph_build: bad arguments");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    DBuf<uint8_t> mask;
    MR_TRY(mask.upload(ctx, trace_mask, (size_t)sp->n_traces));
    MR_TRY(mr_graph_build_dev(ctx, sp, mask.p, out, nullptr));
    mr_handle_add(ctx, *out, [](void* h) { delete (mr_graph*)h; });
    return MR_OK;
}

extern "C" int mr_graph_build_sharded(mr_ctx* ctx, const mr_spans* sp, const uint8_t* trace_mask, mr_graph** out) {
    if (!ctx || !sp || !trace_mask || !out || sp->ctx != ctx)
        return mr_fail(ctx, MR_ERR_ARG, "mr_graph_build_sharded: bad arguments");
    if (!mr_coll_ready(ctx) && ctx->nranks != 1) return mr_fail(ctx, MR_ERR_COMM, "no collective backend");
    if (!sp->indexed) return mr_fail(ctx, MR_ERR_STATE, "span table has no per-trace index (sharded build needs it)");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    *out = nullptr;
    DBuf<uint8_t> mask;
    MR_TRY(mask.upload(ctx, trace_mask, (size_t)sp->n_traces));
    auto g = new mr_graph();
    g->ctx = ctx;
    int rc = graph_build_indexed(ctx, sp, mask.p, g, true);
    if (rc == MR_OK) {
        g->rs_is_sr = true;
        g->pr_identity = true;
        g->n_pr = g->T;
        rc = mr_graph_prepare(ctx, g);
    }
    if (rc == MR_OK) rc = hipStreamSynchronize(ctx->stream) == hipSuccess ? MR_OK : mr_fail(ctx, MR_ERR_HIP, "sync");
    if (rc != MR_OK) {
        delete g;
        return rc;
    }
    mr_handle_add(ctx, g, [](void* h) { delete (mr_graph*)h; });
    *out = g;
    return MR_OK;
}

extern "C" int mr_graph_nodes(const mr_graph* g, int32_t* node_podop, int32_t* trace_code) {
    if (!g) return MR_ERR_ARG;
    mr_ctx* ctx = g->ctx;
    if (!g->node_podop.p && g->N) return mr_fail(ctx, MR_ERR_STATE, "graph was not built from spans");
    if (node_podop && g->N) MR_TRY(g->node_podop.download(ctx, node_podop, g->N));
    if (trace_code && g->T) MR_TRY(g->trace_code.download(ctx, trace_code, g->T));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}

extern "C" int mr_graph_export(const mr_graph* g, int64_t* sr_off, int32_t* sr_ops, int32_t* len_t, int32_t* len_o,
                               int64_t* ss_off, int32_t* ss_par, int32_t* nchild) {
    if (!g) return MR_ERR_ARG;
    mr_ctx* ctx = g->ctx;
    if (sr_off) MR_TRY(g->rs_off.download(ctx, sr_off, (size_t)g->T + 1));
    if (sr_ops) MR_TRY(g->rs_ops.download(ctx, sr_ops, (size_t)g->nnz_rs));
    if (sr_ops) {   // op lists in node order (the indexed build keeps pod-op code order)
        std::vector<int64_t> off((size_t)g->T + 1);
        MR_TRY(g->rs_off.download(ctx, off.data(), off.size()));
        MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
        for (int32_t t = 0; t < g->T; ++t) std::sort(sr_ops + off[t], sr_ops + off[t + 1]);
    }
    if (len_t) MR_TRY(g->len_t.download(ctx, len_t, (size_t)g->T));
    if (len_o) MR_TRY(g->len_o.download(ctx, len_o, (size_t)g->N));
    if (ss_off) MR_TRY(g->ss_off.download(ctx, ss_off, (size_t)g->N + 1));
    if (ss_par) MR_TRY(g->ss_par.download(ctx, ss_par, (size_t)g->E));
    if (nchild) MR_TRY(g->nchild.download(ctx, nchild, (size_t)g->N));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}
