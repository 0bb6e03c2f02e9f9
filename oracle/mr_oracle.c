/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests; never linked
 * into the product).  Plain-C restatement of one MicroRank RCA window over int-coded spans,
 * parallelised with OpenMP where the reference's algorithm allows it:
 *
 *   detect   anormaly_detector.system_anomaly_detect          anormaly_detector.py:44-84
 *            + preprocess_data.get_operation_duration_data    preprocess_data.py:97-122
 *   graph    preprocess_data.get_pagerank_graph               preprocess_data.py:146-171
 *   rank     pagerank.trace_pagerank / pageRank               pagerank.py:15-130
 *   score    online_rca.calculate_spectrum_without_delay_list online_rca.py:33-152
 *
 * Semantics follow SURVEY.md §8.1 (T1-T15) exactly as the numpy oracle (oracle/oracle.py),
 * which is pinned to the reference's golden vectors; tests check this C port against both.
 * The power iteration sums each row in node/trace order (sequential), like the numpy oracle.
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- radix sort (u64 keys + u32 vals) */
static void rsort(uint64_t* k, uint32_t* v, int64_t n, int bits) {
    if (n < 2) return;
    uint64_t* kb = (uint64_t*)malloc(sizeof(uint64_t) * n);
    uint32_t* vb = v ? (uint32_t*)malloc(sizeof(uint32_t) * n) : NULL;
    uint64_t *src = k, *dst = kb;
    uint32_t *vs = v, *vd = vb;
    for (int sh = 0; sh < bits; sh += 8) {   /* stable LSD passes */
        int64_t cnt[257];
        memset(cnt, 0, sizeof cnt);
        for (int64_t i = 0; i < n; ++i) cnt[((src[i] >> sh) & 255) + 1]++;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (int64_t i = 0; i < n; ++i) {
            int64_t p = cnt[(src[i] >> sh) & 255]++;
            dst[p] = src[i];
            if (v) vd[p] = vs[i];
        }
        uint64_t* tk = src; src = dst; dst = tk;
        uint32_t* tv = vs; vs = vd; vd = tv;
    }
    if (src != k) {
        memcpy(k, src, sizeof(uint64_t) * n);
        if (v) memcpy(v, vs, sizeof(uint32_t) * n);
    }
    free(kb);
    free(vb);
}
static int nbits(uint64_t x) { int b = 0; while (b < 64 && (x >> b)) ++b; return b ? b : 1; }

/* ---------------------------------------------------------------- graph */
typedef struct {
    int32_t N, T;
    int64_t nnz, E;
    int32_t *node_podop, *trace_code;
    int64_t *sr_off; int32_t* sr_ops;      /* trace-major, node ascending */
    int64_t *op_off; int32_t* op_trs;      /* op-major, trace ascending */
    int32_t *len_t, *len_o, *nchild;
    int64_t* ss_off; int32_t* ss_par;      /* by child */
} ograph;

static void ograph_free(ograph* g) {
    free(g->node_podop); free(g->trace_code); free(g->sr_off); free(g->sr_ops); free(g->op_off); free(g->op_trs);
    free(g->len_t); free(g->len_o); free(g->nchild); free(g->ss_off); free(g->ss_par);
    memset(g, 0, sizeof *g);
}

/* preprocess_data.py:146-171 */
static void build_graph(int64_t S, const int32_t* trace, const int32_t* podop, const int64_t* span, const int64_t* parent,
                        int32_t NT, int32_t NP, const uint8_t* tmask, const int64_t* id_off, const int32_t* id_rows,
                        int64_t n_codes, ograph* g) {
    memset(g, 0, sizeof *g);
    uint8_t* sel = (uint8_t*)calloc(S ? S : 1, 1);
    int64_t Ss = 0;
    for (int64_t i = 0; i < S; ++i) if (tmask[trace[i]]) { sel[i] = 1; ++Ss; }
    int32_t* rows = (int32_t*)malloc(sizeof(int32_t) * (Ss ? Ss : 1));
    int64_t* first = (int64_t*)malloc(sizeof(int64_t) * NP);
    int32_t* ocnt = (int32_t*)calloc(NP, sizeof(int32_t));
    int32_t* tcnt = (int32_t*)calloc(NT, sizeof(int32_t));
    for (int32_t c = 0; c < NP; ++c) first[c] = INT64_MAX;
    int64_t r = 0;
    for (int64_t i = 0; i < S; ++i) if (sel[i]) {
        rows[r] = (int32_t)i;
        if (first[podop[i]] == INT64_MAX) first[podop[i]] = r;
        ocnt[podop[i]]++; tcnt[trace[i]]++;
        ++r;
    }
    /* join ParentSpanId == spanID over selected rows, traceID ignored (T11) */
    int64_t cap = 16, ne = 0;
    uint64_t* ek = (uint64_t*)malloc(sizeof(uint64_t) * cap);
    for (int64_t li = 0; li < Ss; ++li) {
        int64_t p = parent[rows[li]];
        if (p < 0 || p >= n_codes) continue;
        for (int64_t e = id_off[p]; e < id_off[p + 1]; ++e) {
            int32_t j = id_rows[e];
            if (!sel[j]) continue;
            if (ne == cap) { cap *= 2; ek = (uint64_t*)realloc(ek, sizeof(uint64_t) * cap); }
            ek[ne++] = ((uint64_t)(uint32_t)podop[j] << 32) | (uint32_t)podop[rows[li]];
        }
    }
    int32_t* nchild_c = (int32_t*)calloc(NP, sizeof(int32_t));
    uint8_t* is_par = (uint8_t*)calloc(NP, 1);
    for (int64_t i = 0; i < ne; ++i) { int32_t pc = (int32_t)(ek[i] >> 32); nchild_c[pc]++; is_par[pc] = 1; }
    rsort(ek, NULL, ne, 64);
    int64_t E = 0;
    for (int64_t i = 0; i < ne; ++i) if (i == 0 || ek[i] != ek[i - 1]) ek[E++] = ek[i];
    /* node order: parents by code, then others by first appearance (T10) */
    int32_t* node_of = (int32_t*)malloc(sizeof(int32_t) * NP);
    int32_t N = 0;
    for (int32_t c = 0; c < NP; ++c) if (is_par[c]) node_of[c] = N++;
    int64_t nq = 0;
    uint64_t* qk = (uint64_t*)malloc(sizeof(uint64_t) * (NP ? NP : 1));
    uint32_t* qv = (uint32_t*)malloc(sizeof(uint32_t) * (NP ? NP : 1));
    for (int32_t c = 0; c < NP; ++c) if (!is_par[c] && ocnt[c] > 0) { qk[nq] = (uint64_t)first[c]; qv[nq] = (uint32_t)c; ++nq; }
    rsort(qk, qv, nq, 64);
    for (int64_t i = 0; i < nq; ++i) node_of[qv[i]] = N++;
    g->N = N;
    g->node_podop = (int32_t*)malloc(sizeof(int32_t) * (N ? N : 1));
    for (int32_t c = 0; c < NP; ++c) if (is_par[c] || ocnt[c] > 0) g->node_podop[node_of[c]] = c;
    /* traces (sorted codes) */
    int32_t* tidx = (int32_t*)malloc(sizeof(int32_t) * NT);
    int32_t T = 0;
    for (int32_t c = 0; c < NT; ++c) if (tcnt[c]) tidx[c] = T++;
    g->T = T;
    g->trace_code = (int32_t*)malloc(sizeof(int32_t) * (T ? T : 1));
    g->len_t = (int32_t*)malloc(sizeof(int32_t) * (T ? T : 1));
    for (int32_t c = 0; c < NT; ++c) if (tcnt[c]) { g->trace_code[tidx[c]] = c; g->len_t[tidx[c]] = tcnt[c]; }
    g->len_o = (int32_t*)malloc(sizeof(int32_t) * (N ? N : 1));
    g->nchild = (int32_t*)malloc(sizeof(int32_t) * (N ? N : 1));
    for (int32_t n = 0; n < N; ++n) { g->len_o[n] = ocnt[g->node_podop[n]]; g->nchild[n] = nchild_c[g->node_podop[n]]; }
    /* distinct (trace, node) pairs */
    int nb = nbits((uint64_t)(N > 1 ? N - 1 : 1));
    uint64_t* pk = (uint64_t*)malloc(sizeof(uint64_t) * (Ss ? Ss : 1));
    for (int64_t li = 0; li < Ss; ++li)
        pk[li] = ((uint64_t)tidx[trace[rows[li]]] << nb) | (uint32_t)node_of[podop[rows[li]]];
    rsort(pk, NULL, Ss, nb + nbits((uint64_t)(T > 1 ? T - 1 : 1)));
    int64_t nnz = 0;
    for (int64_t i = 0; i < Ss; ++i) if (i == 0 || pk[i] != pk[i - 1]) pk[nnz++] = pk[i];
    g->nnz = nnz;
    g->sr_off = (int64_t*)calloc((size_t)T + 1, sizeof(int64_t));
    g->sr_ops = (int32_t*)malloc(sizeof(int32_t) * (nnz ? nnz : 1));
    g->op_off = (int64_t*)calloc((size_t)N + 1, sizeof(int64_t));
    g->op_trs = (int32_t*)malloc(sizeof(int32_t) * (nnz ? nnz : 1));
    const uint64_t nm = (1ull << nb) - 1;
    for (int64_t i = 0; i < nnz; ++i) {
        g->sr_off[(pk[i] >> nb) + 1]++;
        g->sr_ops[i] = (int32_t)(pk[i] & nm);
        g->op_off[(pk[i] & nm) + 1]++;
    }
    for (int32_t t = 0; t < T; ++t) g->sr_off[t + 1] += g->sr_off[t];
    for (int32_t n = 0; n < N; ++n) g->op_off[n + 1] += g->op_off[n];
    int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * (N ? N : 1));
    for (int32_t n = 0; n < N; ++n) pos[n] = g->op_off[n];
    for (int64_t i = 0; i < nnz; ++i) g->op_trs[pos[pk[i] & nm]++] = (int32_t)(pk[i] >> nb);  /* stable: traces ascending */
    /* P_ss by child */
    uint64_t* sk = (uint64_t*)malloc(sizeof(uint64_t) * (E ? E : 1));
    for (int64_t i = 0; i < E; ++i)
        sk[i] = ((uint64_t)node_of[(int32_t)(ek[i] & 0xffffffffu)] << nb) | (uint32_t)node_of[(int32_t)(ek[i] >> 32)];
    rsort(sk, NULL, E, 2 * nb);
    g->E = E;
    g->ss_off = (int64_t*)calloc((size_t)N + 1, sizeof(int64_t));
    g->ss_par = (int32_t*)malloc(sizeof(int32_t) * (E ? E : 1));
    for (int64_t i = 0; i < E; ++i) { g->ss_off[(sk[i] >> nb) + 1]++; g->ss_par[i] = (int32_t)(sk[i] & nm); }
    for (int32_t n = 0; n < N; ++n) g->ss_off[n + 1] += g->ss_off[n];
    free(sel); free(rows); free(first); free(ocnt); free(tcnt); free(ek); free(nchild_c); free(is_par); free(node_of);
    free(qk); free(qv); free(tidx); free(pk); free(pos); free(sk);
}

/* ---------------------------------------------------------------- PageRank (pagerank.py:54-130) */
static const ograph* g_cmp;
static int cmp_trace(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    const ograph* g = g_cmp;
    float wx = (float)(1.0 / g->len_t[x]), wy = (float)(1.0 / g->len_t[y]);
    int64_t nx = g->sr_off[x + 1] - g->sr_off[x], ny = g->sr_off[y + 1] - g->sr_off[y];
    if (nx != ny) return nx < ny ? -1 : 1;
    uint32_t bx, by;
    memcpy(&bx, &wx, 4); memcpy(&by, &wy, 4);
    if (nx && bx != by) return bx < by ? -1 : 1;
    for (int64_t i = 0; i < nx; ++i) {
        int32_t ox = g->sr_ops[g->sr_off[x] + i], oy = g->sr_ops[g->sr_off[y] + i];
        if (ox != oy) return ox < oy ? -1 : 1;
    }
    return x < y ? -1 : (x > y);
}

static double vmax(const double* v, int64_t n) {
    double m = -INFINITY;
    for (int64_t i = 0; i < n; ++i) { if (v[i] != v[i]) return v[i]; if (v[i] > m) m = v[i]; }
    return m;
}

/* two traces have equal P_sr columns (pagerank.py:62): same op set and fp32(1/len_t) */
static int same_column(const ograph* g, int32_t a, int32_t b) {
    int64_t na = g->sr_off[a + 1] - g->sr_off[a], nb_ = g->sr_off[b + 1] - g->sr_off[b];
    float wa = (float)(1.0 / g->len_t[a]), wb = (float)(1.0 / g->len_t[b]);
    int eq = na == nb_ && (na == 0 || wa == wb);
    for (int64_t k = 0; eq && k < na; ++k) eq = g->sr_ops[g->sr_off[a] + k] == g->sr_ops[g->sr_off[b] + k];
    return eq;
}

/* kind[t] = size of t's class of equal P_sr columns (T6), by a sort of the traces by column */
static void kinds_sorted(const ograph* g, double* kind) {
    const int32_t T = g->T;
    int32_t* ord = (int32_t*)malloc(sizeof(int32_t) * T);
    for (int32_t t = 0; t < T; ++t) ord[t] = t;
    g_cmp = g;
    qsort(ord, T, sizeof(int32_t), cmp_trace);
    for (int32_t i = 0; i < T;) {
        int32_t j = i + 1;
        while (j < T && same_column(g, ord[i], ord[j])) ++j;
        for (int32_t k = i; k < j; ++k) kind[ord[k]] = (double)(j - i);
        i = j;
    }
    free(ord);
}

static uint64_t mix64c(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* the same classes for large graphs: a 64-bit hash of each column (in parallel), a radix sort of
 * (hash, trace), and an exact check of every trace against its run's first; any collision falls
 * back to kinds_sorted */
static void kinds_hashed(const ograph* g, double* kind) {
    const int32_t T = g->T;
    uint64_t* h = (uint64_t*)malloc(sizeof(uint64_t) * T);
    uint32_t* ord = (uint32_t*)malloc(sizeof(uint32_t) * T);
#pragma omp parallel for schedule(static, 4096)
    for (int32_t t = 0; t < T; ++t) {
        float w = (float)(1.0 / g->len_t[t]);
        uint32_t wb;
        memcpy(&wb, &w, 4);
        uint64_t x = mix64c(((uint64_t)wb << 32) ^ (uint64_t)(g->sr_off[t + 1] - g->sr_off[t]));
        for (int64_t e = g->sr_off[t]; e < g->sr_off[t + 1]; ++e) x = mix64c(x ^ (uint64_t)(uint32_t)g->sr_ops[e]);
        h[t] = x;
        ord[t] = (uint32_t)t;
    }
    rsort(h, ord, T, 64);
    int collided = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(| : collided)
    for (int32_t i = 0; i < T; ++i) {
        if (i > 0 && h[i] == h[i - 1]) continue;   /* one thread per run */
        int32_t j = i + 1;
        while (j < T && h[j] == h[i]) ++j;
        for (int32_t k = i + 1; k < j; ++k) collided |= !same_column(g, (int32_t)ord[i], (int32_t)ord[k]);
        for (int32_t k = i; k < j; ++k) kind[ord[k]] = (double)(j - i);
    }
    free(h);
    free(ord);
    if (collided) kinds_sorted(g, kind);
}

static double wtime(void) {
#ifdef _OPENMP
    return omp_get_wtime();
#else
    return 0.0;
#endif
}

/* weight[N], cov[N]; returns 0 or -1 (empty graph: ValueError).  t_phase (optional): seconds of
 * [kinds + preference, iterations + weights] */
static int pagerank_core(const ograph* g, int anomaly, int iters, double* weight, int32_t* cov, double* kind_out,
                         int hashed_kinds, double* t_phase) {
    const int32_t N = g->N, T = g->T;
    if (N == 0 || T == 0) return -1;
    const double d = 0.85, alpha = 0.01;
    const double t0 = wtime();
    double* kind = (double*)malloc(sizeof(double) * T);
    if (hashed_kinds) kinds_hashed(g, kind);
    else kinds_sorted(g, kind);
    if (kind_out) memcpy(kind_out, kind, sizeof(double) * T);
    /* preference (:68-85), sequential sums in trace order (T7), stored fp32 */
    float* v = (float*)malloc(sizeof(float) * T);
    if (!anomaly) {
        double s = 0.0;
        for (int32_t t = 0; t < T; ++t) s += 1.0 / kind[t];
        for (int32_t t = 0; t < T; ++t) v[t] = (float)(1.0 / kind[t] / s);
    } else {
        double ks = 0.0, ns = 0.0;
        for (int32_t t = 0; t < T; ++t) { ks += 1.0 / kind[t]; ns += 1.0 / (double)g->len_t[t]; }
        for (int32_t t = 0; t < T; ++t) v[t] = (float)(1.0 / (kind[t] / ks * 0.5 + 1.0 / (double)g->len_t[t]) / ns * 0.5);
    }
    const float cd = (float)(1.0 - d);
    const double t1 = wtime();
    double *s = (double*)malloc(sizeof(double) * N), *r = (double*)malloc(sizeof(double) * T);
    double *s2 = (double*)malloc(sizeof(double) * N), *r2 = (double*)malloc(sizeof(double) * T);
    double *wt = (double*)malloc(sizeof(double) * T), *uo = (double*)malloc(sizeof(double) * N);
    double* pw = (double*)malloc(sizeof(double) * N);
    for (int32_t t = 0; t < T; ++t) { r[t] = 1.0 / (double)(N + T); wt[t] = (double)(float)(1.0 / g->len_t[t]); }
    for (int32_t o = 0; o < N; ++o) {
        s[o] = 1.0 / (double)(N + T);
        uo[o] = g->len_o[o] ? (double)(float)(1.0 / g->len_o[o]) : 0.0;
        pw[o] = g->nchild[o] ? (double)(float)(1.0 / g->nchild[o]) : 0.0;
    }
    /* hashed_kinds (large graphs): P_sr r as per-thread trace-range partials summed in thread order
     * (the root op is in every trace: an op-parallel loop would leave it to one thread) */
    int nthr = 1;
#ifdef _OPENMP
    if (hashed_kinds) nthr = omp_get_max_threads();
#endif
    double* part = hashed_kinds ? (double*)malloc(sizeof(double) * (size_t)N * nthr) : NULL;
    for (int it = 0; it < iters; ++it) {   /* Jacobi update (T8), max normalisation (T3) */
        if (part) {
#pragma omp parallel num_threads(nthr)
            {
                int tid = 0;
#ifdef _OPENMP
                tid = omp_get_thread_num();
#endif
                double* pp = part + (size_t)N * tid;
                memset(pp, 0, sizeof(double) * N);
                const int32_t t0_ = (int32_t)((int64_t)T * tid / nthr), t1_ = (int32_t)((int64_t)T * (tid + 1) / nthr);
                for (int32_t t = t0_; t < t1_; ++t) {
                    const double x = wt[t] * r[t];
                    for (int64_t e = g->sr_off[t]; e < g->sr_off[t + 1]; ++e) pp[g->sr_ops[e]] += x;
                }
            }
#pragma omp parallel for schedule(static, 256)
            for (int32_t o = 0; o < N; ++o) {
                double a = 0.0, b = 0.0;
                for (int k = 0; k < nthr; ++k) a += part[(size_t)N * k + o];
                for (int64_t e = g->ss_off[o]; e < g->ss_off[o + 1]; ++e) b += pw[g->ss_par[e]] * s[g->ss_par[e]];
                s2[o] = d * (a + alpha * b);
            }
        } else {
#pragma omp parallel for schedule(dynamic, 64)
            for (int32_t o = 0; o < N; ++o) {
                double a = 0.0, b = 0.0;
                for (int64_t e = g->op_off[o]; e < g->op_off[o + 1]; ++e) a += wt[g->op_trs[e]] * r[g->op_trs[e]];
                for (int64_t e = g->ss_off[o]; e < g->ss_off[o + 1]; ++e) b += pw[g->ss_par[e]] * s[g->ss_par[e]];
                s2[o] = d * (a + alpha * b);
            }
        }
#pragma omp parallel for schedule(static, 1024)
        for (int32_t t = 0; t < T; ++t) {
            double a = 0.0;
            for (int64_t e = g->sr_off[t]; e < g->sr_off[t + 1]; ++e) a += uo[g->sr_ops[e]] * s[g->sr_ops[e]];
            r2[t] = d * a + (double)(cd * v[t]);   /* (1-d)*v in float32 (T4) */
        }
        const double ms = vmax(s2, N), mr = vmax(r2, T);
        for (int32_t o = 0; o < N; ++o) s[o] = s2[o] / ms;
#pragma omp parallel for schedule(static, 4096)
        for (int32_t t = 0; t < T; ++t) r[t] = r2[t] / mr;
    }
    const double m = vmax(s, N);
    double total = 0.0;
    for (int32_t o = 0; o < N; ++o) { s[o] = s[o] / m; total += s[o]; }
    for (int32_t o = 0; o < N; ++o) {
        weight[o] = s[o] * total / (double)N;
        cov[o] = (int32_t)(g->op_off[o + 1] - g->op_off[o]);
    }
    free(kind); free(v); free(s); free(r); free(s2); free(r2); free(wt); free(uo); free(pw); free(part);
    if (t_phase) {
        t_phase[0] = t1 - t0;
        t_phase[1] = wtime() - t1;
    }
    return 0;
}

int oracle_pagerank(const ograph* g, int anomaly, int iters, double* weight, int32_t* cov, double* kind_out) {
    return pagerank_core(g, anomaly, iters, weight, cov, kind_out, 0, NULL);
}

/* ---------------------------------------------------------------- spectrum (online_rca.py:33-152) */
static double spec(int m, double ef, double nf, double ep, double np_) {
    switch (m) {
        case 0: return ef * ef / (ep + nf);
        case 1: return ef / sqrt((ep + ef) * (ef + nf));
        case 2: return ef / (ef + ep + nf);
        case 3: return 2 * ef / (2 * ef + ep + nf);
        case 4: return (ef + np_) / (ep + nf);
        case 5: return ef / (2 * ep + 2 * nf + ef + np_);
        case 6: return (2 * ef - nf - ep) / (2 * ef + nf + ep);
        case 7: return ef / (ef + nf) / (ef / (ef + nf) + ep / (ep + np_));
        case 8: return ef / (ef + nf + ep + np_);
        case 9: return (ef + np_ - ep - nf) / (ef + nf + ep + np_);
        case 10: return 2 * ef / (ef + nf + ep);
        case 11: return (ef + np_) / (ef + np_ + nf + ep);
        default: return (ef + np_) / (ef + np_ + 2 * nf + 2 * ep);
    }
}
typedef struct { double s; int32_t i; } scored;
static int cmp_scored(const void* a, const void* b) {
    const scored *x = (const scored*)a, *y = (const scored*)b;
    if (x->s > y->s) return -1;
    if (x->s < y->s) return 1;
    return x->i < y->i ? -1 : (x->i > y->i);   /* stable descending */
}

/* ---------------------------------------------------------------- one RCA window */
int oracle_rca_window(int64_t S, const int32_t* trace, const int32_t* podop, const int32_t* svcop, const int64_t* span,
                      const int64_t* parent, const int64_t* dur, const int64_t* tstart, const int64_t* tend,
                      int32_t NT, int32_t NP, int32_t NO, int64_t t0, int64_t t1, const double* a3, const uint8_t* a3v,
                      int method, int32_t top_max, int32_t* out_podop, double* out_score, int32_t* n_out,
                      int64_t* edges, int32_t* n_abn, int32_t* n_nor, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    *n_out = 0;
    /* detector (T14, T15) */
    int64_t W = 0;
    long long* tmax = (long long*)malloc(sizeof(long long) * NT);
    for (int32_t t = 0; t < NT; ++t) tmax[t] = LLONG_MIN;
    uint64_t* wk = (uint64_t*)malloc(sizeof(uint64_t) * (S ? S : 1));
    const int ob = nbits((uint64_t)(NO > 1 ? NO - 1 : 1));
    for (int64_t i = 0; i < S; ++i)
        if (tstart[i] >= t0 && tend[i] <= t1) {
            wk[W++] = ((uint64_t)(uint32_t)trace[i] << ob) | (uint32_t)svcop[i];
            if (dur[i] > tmax[trace[i]]) tmax[trace[i]] = dur[i];
        }
    if (W == 0) { free(tmax); free(wk); return -2; }
    rsort(wk, NULL, W, ob + nbits((uint64_t)(NT > 1 ? NT - 1 : 1)));
    uint8_t* state = (uint8_t*)calloc(NT, 1);
    int32_t na = 0, nn = 0;
    for (int64_t i = 0; i < W;) {
        const uint32_t t = (uint32_t)(wk[i] >> ob);
        double expect = 0.0;
        while (i < W && (uint32_t)(wk[i] >> ob) == t) {
            int64_t j = i;
            while (j < W && wk[j] == wk[i]) ++j;
            const int32_t op = (int32_t)(wk[i] & ((1ull << ob) - 1));
            if (a3v[op]) expect += (double)(j - i) * a3[op];
            i = j;
        }
        if (tmax[t] > 0) {
            const double real = (double)tmax[t] / 1000.0;
            if (real > expect) { state[t] = 2; ++na; } else { state[t] = 1; ++nn; }
        }
    }
    free(wk); free(tmax);
    *n_abn = na;
    *n_nor = nn;
    if (!na || !nn) { free(state); return 0; }
    /* spanID multimap */
    int64_t n_codes = 0;
    for (int64_t i = 0; i < S; ++i) if (span[i] + 1 > n_codes) n_codes = span[i] + 1;
    int64_t* id_off = (int64_t*)calloc((size_t)n_codes + 1, sizeof(int64_t));
    int32_t* id_rows = (int32_t*)malloc(sizeof(int32_t) * (S ? S : 1));
    for (int64_t i = 0; i < S; ++i) id_off[span[i] + 1]++;
    for (int64_t c = 0; c < n_codes; ++c) id_off[c + 1] += id_off[c];
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (n_codes ? n_codes : 1));
    memcpy(cur, id_off, sizeof(int64_t) * n_codes);
    for (int64_t i = 0; i < S; ++i) id_rows[cur[span[i]]++] = (int32_t)i;
    free(cur);
    uint8_t* m_abn = (uint8_t*)malloc(NT);
    uint8_t* m_nor = (uint8_t*)malloc(NT);
    for (int32_t t = 0; t < NT; ++t) { m_abn[t] = state[t] == 2; m_nor[t] = state[t] == 1; }
    ograph gn, ga;   /* T1: "normal" graph from the detector's abnormal list */
    build_graph(S, trace, podop, span, parent, NT, NP, m_abn, id_off, id_rows, n_codes, &gn);
    build_graph(S, trace, podop, span, parent, NT, NP, m_nor, id_off, id_rows, n_codes, &ga);
    double* wn = (double*)malloc(sizeof(double) * gn.N);
    double* wa = (double*)malloc(sizeof(double) * ga.N);
    int32_t* cn = (int32_t*)malloc(sizeof(int32_t) * gn.N);
    int32_t* ca = (int32_t*)malloc(sizeof(int32_t) * ga.N);
    oracle_pagerank(&gn, 0, 25, wn, cn, NULL);
    oracle_pagerank(&ga, 1, 25, wa, ca, NULL);
    *edges = 25 * (2 * (gn.nnz + ga.nnz) + gn.E + ga.E);
    /* spectrum over anomaly nodes then normal-only nodes */
    int32_t* pos = (int32_t*)malloc(sizeof(int32_t) * NP);
    for (int32_t c = 0; c < NP; ++c) pos[c] = -1;
    for (int32_t i = 0; i < ga.N; ++i) pos[ga.node_podop[i]] = i;
    scored* sc = (scored*)malloc(sizeof(scored) * (ga.N + gn.N));
    int32_t* code = (int32_t*)malloc(sizeof(int32_t) * (ga.N + gn.N));
    double* nw_of_a = (double*)malloc(sizeof(double) * (ga.N ? ga.N : 1));
    int32_t* nc_of_a = (int32_t*)malloc(sizeof(int32_t) * (ga.N ? ga.N : 1));
    uint8_t* both = (uint8_t*)calloc(ga.N ? ga.N : 1, 1);
    for (int32_t j = 0; j < gn.N; ++j) {
        int32_t p = pos[gn.node_podop[j]];
        if (p >= 0) { both[p] = 1; nw_of_a[p] = wn[j]; nc_of_a[p] = cn[j]; }
    }
    const double A = nn, Nl = na;   /* len(abnormal_list) = detector normals (T1) */
    int32_t n = 0;
    for (int32_t i = 0; i < ga.N; ++i) {
        double ef = wa[i] * ca[i], nf = wa[i] * (A - ca[i]), ep, np_;
        if (both[i]) { ep = nw_of_a[i] * nc_of_a[i]; np_ = nw_of_a[i] * (Nl - nc_of_a[i]); }
        else { ep = 0.0000001; np_ = 0.0000001; }
        sc[n].s = spec(method, ef, nf, ep, np_); sc[n].i = n; code[n] = ga.node_podop[i]; ++n;
    }
    for (int32_t j = 0; j < gn.N; ++j) {
        if (pos[gn.node_podop[j]] >= 0) continue;
        double ep = (1 + wn[j]) * cn[j], np_ = Nl - cn[j];
        sc[n].s = spec(method, 0.0000001, 0.0000001, ep, np_); sc[n].i = n; code[n] = gn.node_podop[j]; ++n;
    }
    for (int32_t i = 0; i < n; ++i) if (sc[i].s == 0.0) sc[i].s = 0.0;
    qsort(sc, n, sizeof(scored), cmp_scored);
    int32_t k = n < top_max + 6 ? n : top_max + 6;
    for (int32_t i = 0; i < k; ++i) { out_podop[i] = code[sc[i].i]; out_score[i] = sc[i].s; }
    *n_out = k;
    free(state); free(id_off); free(id_rows); free(m_abn); free(m_nor); free(wn); free(wa); free(cn); free(ca);
    free(pos); free(sc); free(code); free(nw_of_a); free(nc_of_a); free(both);
    ograph_free(&gn);
    ograph_free(&ga);
    return 0;
}

/* ---------------------------------------------------------------- graph + PageRank only (for tests) */
int oracle_graph_pagerank(int64_t S, const int32_t* trace, const int32_t* podop, const int64_t* span,
                          const int64_t* parent, int32_t NT, int32_t NP, const uint8_t* tmask, int anomaly,
                          int32_t* node_podop, double* weight, int32_t* cov, int32_t* n_nodes, int64_t* nnz) {
    int64_t n_codes = 0;
    for (int64_t i = 0; i < S; ++i) if (span[i] + 1 > n_codes) n_codes = span[i] + 1;
    int64_t* id_off = (int64_t*)calloc((size_t)n_codes + 1, sizeof(int64_t));
    int32_t* id_rows = (int32_t*)malloc(sizeof(int32_t) * (S ? S : 1));
    for (int64_t i = 0; i < S; ++i) id_off[span[i] + 1]++;
    for (int64_t c = 0; c < n_codes; ++c) id_off[c + 1] += id_off[c];
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (n_codes ? n_codes : 1));
    memcpy(cur, id_off, sizeof(int64_t) * n_codes);
    for (int64_t i = 0; i < S; ++i) id_rows[cur[span[i]]++] = (int32_t)i;
    free(cur);
    ograph g;
    build_graph(S, trace, podop, span, parent, NT, NP, tmask, id_off, id_rows, n_codes, &g);
    *n_nodes = g.N;
    *nnz = g.nnz;
    int rc = oracle_pagerank(&g, anomaly, 25, weight, cov, NULL);
    if (rc == 0) memcpy(node_podop, g.node_podop, sizeof(int32_t) * g.N);
    free(id_off); free(id_rows);
    ograph_free(&g);
    return rc;
}

/* ---------------------------------------------------------------- a graph given as incidence lists
 * trace_pagerank (pagerank.py:15-130) of a graph built elsewhere (bench.py's C4 CPU baseline: the
 * same synthetic graph the GPU ranks).  sr_off/sr_ops: trace-major distinct ops (ascending);
 * ss_off/ss_par: parents by child.  The op-major copy is built before the clock starts.
 * nthreads 0: OpenMP default.  t_phase[2]: seconds of kinds + preference, iterations + weights. */
int oracle_incidence_pagerank(int32_t N, int32_t T, const int64_t* sr_off, const int32_t* sr_ops, const int32_t* len_t,
                              const int32_t* len_o, const int64_t* ss_off, const int32_t* ss_par,
                              const int32_t* nchild, int anomaly, int iters, int nthreads, double* weight,
                              int32_t* cov, double* t_phase) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    ograph g;
    memset(&g, 0, sizeof g);
    g.N = N;
    g.T = T;
    g.nnz = sr_off[T];
    g.E = ss_off[N];
    g.sr_off = (int64_t*)sr_off;
    g.sr_ops = (int32_t*)sr_ops;
    g.len_t = (int32_t*)len_t;
    g.len_o = (int32_t*)len_o;
    g.nchild = (int32_t*)nchild;
    g.ss_off = (int64_t*)ss_off;
    g.ss_par = (int32_t*)ss_par;
    g.op_off = (int64_t*)calloc((size_t)N + 1, sizeof(int64_t));
    g.op_trs = (int32_t*)malloc(sizeof(int32_t) * (g.nnz ? g.nnz : 1));
    for (int64_t e = 0; e < g.nnz; ++e) g.op_off[sr_ops[e] + 1]++;
    for (int32_t o = 0; o < N; ++o) g.op_off[o + 1] += g.op_off[o];
    int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * (N ? N : 1));
    memcpy(pos, g.op_off, sizeof(int64_t) * N);
    for (int32_t t = 0; t < T; ++t)
        for (int64_t e = sr_off[t]; e < sr_off[t + 1]; ++e) g.op_trs[pos[sr_ops[e]]++] = t;
    free(pos);
    int rc = pagerank_core(&g, anomaly, iters, weight, cov, NULL, 1, t_phase);
    free(g.op_off);
    free(g.op_trs);
    return rc;
}
