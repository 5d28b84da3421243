/*
 * oracle/san_check.c -- TEST INFRASTRUCTURE: a self-check of the C restatement
 * (nw_oracle.c) meant to be built with host sanitizers (tests/test_sanitizers.py):
 *   -fsanitize=address,undefined : every oracle entry point on small ragged
 *                                  shapes, including the empty ones;
 *   -fsanitize=thread            : the idxarray-mt restatement (the only
 *                                  threaded code, idxarray-mt.cpp:4-70) on 2-4
 *                                  threads, checked against the serial fill.
 * Exit status 0 = all consistent; each inconsistency prints one line and exits 1.
 * Usage: san_check [all|threads]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void nw_oracle_fill(const int8_t *, int64_t, const int8_t *, int64_t, int32_t, int32_t, int32_t,
                    int32_t *, int64_t);
int32_t nw_oracle_score(const int8_t *, int64_t, const int8_t *, int64_t, int32_t, int32_t, int32_t,
                        int32_t *, int32_t *, uint64_t *, uint64_t *);
void nw_oracle_fill_idxarray(const int8_t *, int64_t, const int8_t *, int64_t, int32_t, int32_t,
                             int32_t, int32_t *, int);
void nw_oracle_band_layout(int64_t, int, int, int64_t *, int64_t *);
void nw_oracle_fill_band(const int8_t *, int64_t, const int8_t *, int64_t, int32_t, int32_t, int32_t,
                         int, int, const int32_t *, int32_t *);
void nw_oracle_colband_layout(int64_t, int, int, int64_t *, int64_t *);
void nw_oracle_fill_colband(const int8_t *, const int8_t *, int64_t, int32_t, int32_t, int32_t,
                            int64_t, int64_t, const int32_t *, int32_t *);
void nw_oracle_synth(uint64_t, int64_t, int8_t *);
void nw_oracle_sw_fill(const int8_t *, int64_t, const int8_t *, int64_t, int32_t, int32_t, int32_t,
                       int32_t *);
int32_t nw_oracle_sw_best(const int8_t *, int64_t, const int8_t *, int64_t, int32_t, int32_t, int32_t,
                          int64_t *, int64_t *);
int64_t nw_oracle_sw_traceback(const int8_t *, int64_t, const int8_t *, int64_t, int32_t, int32_t,
                               int32_t, const int32_t *, int64_t, int64_t, uint8_t *, int64_t,
                               int64_t *, int64_t *);

#define FAIL(...) do { printf(__VA_ARGS__); printf("\n"); exit(1); } while (0)

static const int32_t kSchemes[3][3] = {{1, 0, -1}, {1, -1, -1}, {2, -1, -2}};

static int32_t *full(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2, const int32_t *sc) {
    int32_t *t = malloc(sizeof(int32_t) * (size_t)((n1 + 1) * (n2 + 1)));
    nw_oracle_fill(s1, n1, s2, n2, sc[0], sc[1], sc[2], t, n1 + 1);
    return t;
}

static void check_threads(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2, const int32_t *sc,
                          const int32_t *t) {
    const size_t cells = (size_t)((n1 + 1) * (n2 + 1));
    int32_t *u = malloc(sizeof(int32_t) * cells);
    for (int th = 2; th <= 4; ++th) {
        memset(u, 0x5a, sizeof(int32_t) * cells);
        nw_oracle_fill_idxarray(s1, n1, s2, n2, sc[0], sc[1], sc[2], u, th);
        if (memcmp(t, u, sizeof(int32_t) * cells) != 0)
            FAIL("idxarray %lldx%lld threads=%d differs from the serial fill", (long long)n1, (long long)n2, th);
    }
    free(u);
}

static void check_all(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2, const int32_t *sc,
                      const int32_t *t) {
    const int64_t nc = n1 + 1, nr = n2 + 1;
    /* score-only with rows/cols/checksums */
    int32_t *lr = malloc(sizeof(int32_t) * (size_t)nc), *lc = malloc(sizeof(int32_t) * (size_t)nr);
    uint64_t *rs = malloc(sizeof(uint64_t) * (size_t)nr), *rw = malloc(sizeof(uint64_t) * (size_t)nr);
    int32_t sc_ = nw_oracle_score(s1, n1, s2, n2, sc[0], sc[1], sc[2], lr, lc, rs, rw);
    if (sc_ != t[n2 * nc + n1]) FAIL("score %lldx%lld", (long long)n1, (long long)n2);
    if (memcmp(lr, t + n2 * nc, sizeof(int32_t) * (size_t)nc)) FAIL("last row");
    for (int64_t i = 0; i < nr; ++i) {
        uint64_t s = 0, w = 0;
        for (int64_t j = 0; j < nc; ++j) {
            s += (uint64_t)(int64_t)t[i * nc + j];
            w += (uint64_t)(int64_t)t[i * nc + j] * (uint64_t)(j + 1);
        }
        if (lc[i] != t[i * nc + n1] || rs[i] != s || rw[i] != w) FAIL("row %lld checksums", (long long)i);
    }
    /* row bands (mpi-horz) and column bands (mpi-vert) reassemble the table */
    for (int P = 1; P <= 4; ++P) {
        if (nr >= P) {
            const int32_t *halo = NULL;
            int32_t *prev = NULL;
            for (int r = 0; r < P; ++r) {
                int64_t rows, start;
                nw_oracle_band_layout(n2, P, r, &rows, &start);
                int32_t *b = malloc(sizeof(int32_t) * (size_t)(rows * nc));
                nw_oracle_fill_band(s1, n1, s2, n2, sc[0], sc[1], sc[2], P, r, halo, b);
                if (memcmp(b, t + start * nc, sizeof(int32_t) * (size_t)(rows * nc)))
                    FAIL("row band P=%d r=%d", P, r);
                free(prev);
                prev = b;
                halo = b + (rows - 1) * nc;
            }
            free(prev);
        }
        if (nc >= P) {
            int32_t *left = NULL;
            for (int r = 0; r < P; ++r) {
                int64_t cols, start;
                nw_oracle_colband_layout(n1, P, r, &cols, &start);
                int32_t *b = malloc(sizeof(int32_t) * (size_t)(cols * nr));
                nw_oracle_fill_colband(s1, s2, n2, sc[0], sc[1], sc[2], start, cols, left, b);
                for (int64_t i = 0; i < nr; ++i)
                    if (memcmp(b + i * cols, t + i * nc + start, sizeof(int32_t) * (size_t)cols))
                        FAIL("column band P=%d r=%d row %lld", P, r, (long long)i);
                free(left);
                left = malloc(sizeof(int32_t) * (size_t)nr);
                for (int64_t i = 0; i < nr; ++i) left[i] = b[i * cols + cols - 1];
                free(b);
            }
            free(left);
        }
    }
    /* Smith-Waterman: full table vs linear-memory best cell, traceback replay */
    int32_t *w = malloc(sizeof(int32_t) * (size_t)(nc * nr));
    nw_oracle_sw_fill(s1, n1, s2, n2, sc[0], sc[1], sc[2], w);
    int64_t ei, ej, bi, bj;
    int32_t best = nw_oracle_sw_best(s1, n1, s2, n2, sc[0], sc[1], sc[2], &ei, &ej);
    if (best != w[ei * nc + ej]) FAIL("sw best");
    uint8_t *ops = malloc((size_t)(n1 + n2 + 1));
    int64_t k = nw_oracle_sw_traceback(s1, n1, s2, n2, sc[0], sc[1], sc[2], w, ei, ej, ops, n1 + n2 + 1, &bi, &bj);
    if (k < 0) FAIL("sw traceback %lld", (long long)k);
    int64_t i = bi, j = bj;
    int32_t v = 0;
    for (int64_t x = 0; x < k; ++x) {
        if (ops[x] == 0) { v += s1[j] == s2[i] ? sc[0] : sc[1]; ++i; ++j; }
        else { v += sc[2]; if (ops[x] == 1) ++i; else ++j; }
    }
    if (i != ei || j != ej || v != best) FAIL("sw traceback replay");
    free(ops); free(w); free(lr); free(lc); free(rs); free(rw);
}

int main(int argc, char **argv) {
    const int threads_only = argc > 1 && strcmp(argv[1], "threads") == 0;
    static const int64_t shapes[][2] = {{0, 0}, {0, 5}, {7, 0}, {1, 1}, {3, 17}, {64, 63},
                                        {129, 65}, {200, 31}, {257, 300}};
    for (size_t q = 0; q < sizeof(shapes) / sizeof(shapes[0]); ++q) {
        const int64_t n1 = shapes[q][0], n2 = shapes[q][1];
        int8_t *s1 = malloc((size_t)n1 + 1), *s2 = malloc((size_t)n2 + 1);
        nw_oracle_synth(11 + q, n1, s1);
        nw_oracle_synth(97 + q, n2, s2);
        for (int s = 0; s < 3; ++s) {
            int32_t *t = full(s1, n1, s2, n2, kSchemes[s]);
            if (threads_only) check_threads(s1, n1, s2, n2, kSchemes[s], t);
            else check_all(s1, n1, s2, n2, kSchemes[s], t);
            free(t);
        }
        free(s1);
        free(s2);
    }
    printf("ok\n");
    return 0;
}
