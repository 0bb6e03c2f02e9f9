/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Driver that runs the C restatement (mr_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 "race detection / sanitizers"):
 * tests/test_c_oracle.py dumps a window's int-coded spans to a file, runs this binary, and
 * compares its output with the unsanitised library's.  Any ASan/UBSan report aborts (nonzero exit).
 *
 * Input file (little endian): int64 S, int32 NT, NP, NO, int32 pad, int64 t0, t1, then the
 * columns trace[S] podop[S] svcop[S] (int32), span[S] parent[S] dur[S] tstart[S] tend[S] (int64),
 * a3[NO] (float64), a3v[NO] (uint8).
 * Output: "n_abn n_nor n_out edges" then one "code score(hex)" line per ranked op.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int oracle_rca_window(int64_t S, const int32_t* trace, const int32_t* podop, const int32_t* svcop, const int64_t* span,
                      const int64_t* parent, const int64_t* dur, const int64_t* tstart, const int64_t* tend,
                      int32_t NT, int32_t NP, int32_t NO, int64_t t0, int64_t t1, const double* a3, const uint8_t* a3v,
                      int method, int32_t top_max, int32_t* out_podop, double* out_score, int32_t* n_out,
                      int64_t* edges, int32_t* n_abn, int32_t* n_nor, int nthreads);

static void* rd(FILE* f, size_t n, size_t sz) {
    void* p = malloc(n * sz + 1);
    if (!p || fread(p, sz, n, f) != n) { fprintf(stderr, "short read\n"); exit(3); }
    return p;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int64_t S, t0, t1;
    int32_t hdr[4];
    if (fread(&S, 8, 1, f) != 1 || fread(hdr, 4, 4, f) != 4 || fread(&t0, 8, 1, f) != 1 || fread(&t1, 8, 1, f) != 1)
        return 3;
    const int32_t NT = hdr[0], NP = hdr[1], NO = hdr[2];
    int32_t* trace = rd(f, S, 4);
    int32_t* podop = rd(f, S, 4);
    int32_t* svcop = rd(f, S, 4);
    int64_t* span = rd(f, S, 8);
    int64_t* parent = rd(f, S, 8);
    int64_t* dur = rd(f, S, 8);
    int64_t* ts = rd(f, S, 8);
    int64_t* te = rd(f, S, 8);
    double* a3 = rd(f, NO, 8);
    uint8_t* a3v = rd(f, NO, 1);
    fclose(f);
    int32_t codes[11], n_out = 0, na = 0, nn = 0;
    double scores[11];
    int64_t edges = 0;
    const int rc = oracle_rca_window(S, trace, podop, svcop, span, parent, dur, ts, te, NT, NP, NO, t0, t1, a3, a3v, 0, 5,
                                     codes, scores, &n_out, &edges, &na, &nn, 2);
    if (rc != 0) { printf("rc %d\n", rc); return 0; }
    printf("%d %d %d %lld\n", na, nn, n_out, (long long)edges);
    for (int i = 0; i < n_out; ++i) printf("%d %a\n", codes[i], scores[i]);
    free(trace); free(podop); free(svcop); free(span); free(parent); free(dur); free(ts); free(te); free(a3); free(a3v);
    return 0;
}
