/*
 * ac_oracle.c -- CPU restatement of errorCount (approx_counter.cpp:531-601).
 * TEST INFRASTRUCTURE ONLY -- see ac_oracle.h.  PARITY UNPINNED.
 *
 * Build: oracle/Makefile  (gcc -O2 -fopenmp -shared).
 */
#include "ac_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* int2dna (approx_counter.cpp:70-78): base i of the k-mer (i = 0 first) sits at
 * bits 2*(k-1-i) .. 2*(k-1-i)+1 of the value. */
static void decode_kmer(uint64_t kmer, uint32_t k, uint8_t* out) {
    for (uint32_t i = 0; i < k; ++i) out[i] = (uint8_t)((kmer >> (2u * (k - 1u - i))) & 3u);
}

static int valid_k(uint32_t k) { return k >= 2 && k <= 32; } /* main 781-783 */

/* ------------------------------------------------------------------------ */
/* (1) Plain DP.  D[0][j] = 0 (free start in the text), D[i][0] = i, answer   */
/*     min_j D[k][j] for j = 0..n (j = 0 is the empty substring).            */
/* ------------------------------------------------------------------------ */
static int dp_distance(const uint8_t* p, uint32_t m, const uint8_t* t, uint32_t n, int cap) {
    int col[33];
    for (uint32_t i = 0; i <= m; ++i) col[i] = (int)i;
    int best = col[m];
    for (uint32_t j = 1; j <= n; ++j) {
        int diag = col[0]; /* D[0][j-1] */
        col[0] = 0;
        for (uint32_t i = 1; i <= m; ++i) {
            int up = col[i]; /* D[i][j-1] */
            int sub = diag + ((t[j - 1] >= 4 || t[j - 1] != p[i - 1]) ? 1 : 0);
            int del = up + 1;          /* text char unmatched          */
            int ins = col[i - 1] + 1;  /* pattern char unmatched       */
            int v = sub < del ? sub : del;
            v = v < ins ? v : ins;
            diag = up;
            col[i] = v;
        }
        if (col[m] < best) best = col[m];
    }
    return best < cap ? best : cap;
}

int oracle_distance_dp(uint64_t kmer, uint32_t k, const uint8_t* text, uint32_t n, int cap) {
    if (!valid_k(k)) return -1;
    uint8_t p[32];
    decode_kmer(kmer, k, p);
    return dp_distance(p, k, text, n, cap);
}

int oracle_count_dp(uint32_t k, const uint64_t* kmers, uint32_t n_kmers, const uint8_t* bases,
                    const uint64_t* offset, const uint32_t* length, uint32_t n_windows,
                    uint64_t* counts) {
    if (!valid_k(k)) return 1;
    for (uint32_t c = 0; c < n_kmers; ++c) {
        uint8_t p[32];
        decode_kmer(kmers[c], k, p);
        uint64_t total = 0;
        for (uint32_t w = 0; w < n_windows; ++w) {
            int d = dp_distance(p, k, bases + offset[w], length[w], 3);
            total += (uint64_t)(3 - d);
        }
        counts[c] = total;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* (2) Myers 1999 bit-vector search, one 64-bit word (k <= 32).  min score    */
/*     over all text columns, starting from score = k (empty substring).      */
/*     OpenMP over candidates, schedule(dynamic) like approx_counter.cpp:567. */
/* ------------------------------------------------------------------------ */
static int myers_distance(const uint64_t peq[5], uint32_t m, const uint8_t* t, uint32_t n, int cap) {
    const uint64_t hib = 1ull << (m - 1);
    uint64_t pv = (m == 64) ? ~0ull : ((1ull << m) - 1ull), mv = 0;
    int score = (int)m, best = (int)m;
    for (uint32_t j = 0; j < n; ++j) {
        const uint64_t eq = peq[t[j] < 4 ? t[j] : 4];
        const uint64_t xv = eq | mv;
        const uint64_t xh = (((eq & pv) + pv) ^ pv) | eq;
        uint64_t ph = mv | ~(xh | pv);
        uint64_t mh = pv & xh;
        if (ph & hib) ++score;
        else if (mh & hib) --score;
        ph <<= 1;
        mh <<= 1;
        pv = mh | ~(xv | ph);
        mv = ph & xv;
        if (score < best) best = score;
    }
    return best < cap ? best : cap;
}

int oracle_count_myers(uint32_t k, const uint64_t* kmers, uint32_t n_kmers, const uint8_t* bases,
                       const uint64_t* offset, const uint32_t* length, uint32_t n_windows,
                       uint64_t* counts, int n_threads) {
    if (!valid_k(k)) return 1;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
#pragma omp parallel for schedule(dynamic)
    for (long c = 0; c < (long)n_kmers; ++c) {
        uint8_t p[32];
        uint64_t peq[5] = {0, 0, 0, 0, 0};
        decode_kmer(kmers[c], k, p);
        for (uint32_t i = 0; i < k; ++i) peq[p[i]] |= 1ull << i;
        uint64_t total = 0;
        for (uint32_t w = 0; w < n_windows; ++w)
            total += (uint64_t)(3 - myers_distance(peq, k, bases + offset[w], length[w], 3));
        counts[c] = total;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* (3) SeqAn 2.4 find<0,2>(delegate, index, needle, EditDistance()) restated */
/*     (approx_counter.cpp:586).  The bidirectional FM index */
/*     iterator is replaced by the explicit occurrence set of the text string */
/*     matched so far; goDown(iter, dir) = extend every occurrence by one     */
/*     character on the right (dir=RIGHT) or on the left.  Strings never span */
/*     two windows (StringSet sentinels).  'N' is a text character of the     */
/*     Dna5 index alphabet that never equals a needle character.              */
/* ------------------------------------------------------------------------ */
enum { RIGHT = 1, LEFT = 0 };
#define NBLOCKS 4

typedef struct { uint32_t w, s, e; } occ_t; /* window w, text [s, e) */

typedef struct {
    const uint8_t* bases;
    const uint64_t* offset;
    const uint32_t* length;
    uint32_t n_windows;
    const uint8_t* needle;
    int k;
    int strict;
    /* current scheme */
    int pi[NBLOCKS], lo[NBLOCKS], up[NBLOCKS], blen[NBLOCKS];
    uint8_t* hits; /* per window: bit e = reported with e errors (tcount[e]) */
} sim_t;

typedef struct { occ_t* v; size_t n; int root; } occset_t;

static occset_t extend(const sim_t* S, const occset_t* in, int c, int dir) {
    occset_t out = {NULL, 0, 0};
    size_t cap = 0;
#define PUSH(W, A, B)                                                        \
    do {                                                                     \
        if (out.n == cap) {                                                  \
            cap = cap ? 2 * cap : 64;                                        \
            out.v = (occ_t*)realloc(out.v, cap * sizeof(occ_t));             \
        }                                                                    \
        out.v[out.n].w = (W); out.v[out.n].s = (A); out.v[out.n].e = (B);    \
        ++out.n;                                                             \
    } while (0)
    if (in->root) {
        for (uint32_t w = 0; w < S->n_windows; ++w) {
            const uint8_t* t = S->bases + S->offset[w];
            for (uint32_t p = 0; p < S->length[w]; ++p)
                if ((int)(t[p] < 4 ? t[p] : 4) == c) PUSH(w, p, p + 1);
        }
    } else {
        for (size_t i = 0; i < in->n; ++i) {
            const occ_t o = in->v[i];
            const uint8_t* t = S->bases + S->offset[o.w];
            if (dir == RIGHT) {
                if (o.e < S->length[o.w] && (int)(t[o.e] < 4 ? t[o.e] : 4) == c) PUSH(o.w, o.s, o.e + 1);
            } else {
                if (o.s > 0 && (int)(t[o.s - 1] < 4 ? t[o.s - 1] : 4) == c) PUSH(o.w, o.s - 1, o.e);
            }
        }
    }
#undef PUSH
    return out;
}

static void report(sim_t* S, const occset_t* occ, int errors) {
    if (occ->root) { /* whole index: every read (only reachable for k <= 2) */
        for (uint32_t w = 0; w < S->n_windows; ++w) S->hits[w] |= (uint8_t)(1u << errors);
        return;
    }
    for (size_t i = 0; i < occ->n; ++i) S->hits[occ->v[i].w] |= (uint8_t)(1u << errors);
}

static int dir_of_block(const sim_t* S, int b) { return (b == 0 || S->pi[b] > S->pi[b - 1]) ? RIGHT : LEFT; }

static void search(sim_t* S, const occset_t* occ, int lp, int rp, int e, int b, int dir);

/* _optimalSearchSchemeDeletion: the block is complete; either hand over to the
 * next block (the last block stays, so the next call sees `done`), or, while
 * errors remain in this block, extend the text by any character (+1 error). */
static void deletion_mode(sim_t* S, const occset_t* occ, int lp, int rp, int e, int b, int dir) {
    const int max_left = S->up[b] - e;
    const int min_left = S->lo[b] > e ? S->lo[b] - e : 0;
    if (min_left == 0) {
        const int b2 = (b + 1 < NBLOCKS) ? b + 1 : NBLOCKS - 1;
        search(S, occ, lp, rp, e, b2, dir_of_block(S, b2));
    }
    const int complete = (lp == 0 && rp == S->k + 1);
    if (max_left > 0 && !(S->strict && complete)) {
        for (int c = 0; c < 5; ++c) {
            occset_t o2 = extend(S, occ, c, dir);
            if (o2.n) deletion_mode(S, &o2, lp, rp, e + 1, b, dir);
            free(o2.v);
        }
    }
}

/* _optimalSearchSchemeExact: match the rest of block b exactly. */
static void exact(sim_t* S, const occset_t* occ, int lp, int rp, int e, int b, int dir) {
    occset_t cur = *occ, tmp;
    int owned = 0;
    while (rp - lp - 1 < S->blen[b]) {
        const int nc = (dir == RIGHT) ? S->needle[rp - 1] : S->needle[lp - 1];
        tmp = extend(S, &cur, nc, dir);
        if (owned) free(cur.v);
        cur = tmp;
        owned = 1;
        if (!cur.n) { free(cur.v); return; }
        if (dir == RIGHT) ++rp; else --lp;
    }
    if (b + 1 < NBLOCKS) search(S, &cur, lp, rp, e, b + 1, dir_of_block(S, b + 1));
    else search(S, &cur, lp, rp, e, b, dir); /* done -> report */
    if (owned) free(cur.v);
}

/* _optimalSearchSchemeChildren: every text character extending the current
 * string: match/mismatch (consumes one needle char) and deletion (does not). */
static void children(sim_t* S, const occset_t* occ, int lp, int rp, int e, int b, int dir) {
    const int matched = rp - lp - 1;
    const int nc = (dir == RIGHT) ? S->needle[rp - 1] : S->needle[lp - 1];
    const int lp2 = lp - (dir == LEFT), rp2 = rp + (dir == RIGHT);
    for (int c = 0; c < 5; ++c) {
        occset_t o2 = extend(S, occ, c, dir);
        if (!o2.n) { free(o2.v); continue; }
        const int delta = (c != nc) ? 1 : 0; /* N (4) never equals */
        if (matched + 1 == S->blen[b]) deletion_mode(S, &o2, lp2, rp2, e + delta, b, dir);
        else search(S, &o2, lp2, rp2, e + delta, b, dir);
        search(S, &o2, lp, rp, e + 1, b, dir); /* deletion */
        free(o2.v);
    }
}

/* _optimalSearchScheme */
static void search(sim_t* S, const occset_t* occ, int lp, int rp, int e, int b, int dir) {
    const int max_left = S->up[b] - e;
    const int min_left = S->lo[b] > e ? S->lo[b] - e : 0;
    if (lp == 0 && rp == S->k + 1) { /* done */
        if (min_left == 0) report(S, occ, e);
        return;
    }
    const int matched = rp - lp - 1;
    if (max_left == 0 && matched != S->blen[b]) {
        exact(S, occ, lp, rp, e, b, dir);
        return;
    }
    if (max_left <= 0) return; /* unreachable for well-formed schemes */
    /* insertion: consume a needle char without a text char */
    {
        const int pos = (dir == RIGHT) ? rp - 1 : lp - 1;
        const int forbid = S->strict && (pos == 0 || pos == S->k - 1);
        if (!forbid) {
            const int lp2 = lp - (dir == LEFT), rp2 = rp + (dir == RIGHT);
            if (matched + 1 == S->blen[b]) deletion_mode(S, occ, lp2, rp2, e + 1, b, dir);
            else search(S, occ, lp2, rp2, e + 1, b, dir);
        }
    }
    children(S, occ, lp, rp, e, b, dir);
}

/* OptimalSearchSchemes<0, 2>: three searches over four blocks (pi, L, U). */
static const int SCHEMES[3][3][NBLOCKS] = {
    {{2, 1, 3, 4}, {0, 0, 1, 1}, {0, 0, 2, 2}},
    {{3, 2, 1, 4}, {0, 0, 0, 0}, {0, 1, 1, 2}},
    {{4, 3, 2, 1}, {0, 0, 0, 2}, {0, 1, 2, 2}},
};

int oracle_count_scheme(uint32_t k, const uint64_t* kmers, uint32_t n_kmers, const uint8_t* bases,
                        const uint64_t* offset, const uint32_t* length, uint32_t n_windows,
                        uint64_t* counts, uint8_t* levels, int strict) {
    if (!valid_k(k)) return 1;
    sim_t S;
    memset(&S, 0, sizeof S);
    S.bases = bases; S.offset = offset; S.length = length; S.n_windows = n_windows;
    S.k = (int)k; S.strict = strict;
    S.hits = (uint8_t*)calloc(n_windows ? n_windows : 1, 1);
    uint8_t needle[32];
    S.needle = needle;
    /* block lengths in needle order: floor(k/4) + (i < k mod 4) */
    int bl[NBLOCKS];
    for (int i = 0; i < NBLOCKS; ++i) bl[i] = (int)(k / NBLOCKS) + (i < (int)(k % NBLOCKS) ? 1 : 0);
    for (uint32_t c = 0; c < n_kmers; ++c) {
        decode_kmer(kmers[c], k, needle);
        memset(S.hits, 0, n_windows);
        for (int s = 0; s < 3; ++s) {
            int cum = 0, start = 0;
            for (int b = 0; b < NBLOCKS; ++b) {
                S.pi[b] = SCHEMES[s][0][b];
                S.lo[b] = SCHEMES[s][1][b];
                S.up[b] = SCHEMES[s][2][b];
                cum += bl[S.pi[b] - 1];
                S.blen[b] = cum;
            }
            for (int i = 0; i < S.pi[0] - 1; ++i) start += bl[i];
            occset_t root = {NULL, 0, 1};
            search(&S, &root, start, start + 1, 0, 0, RIGHT);
        }
        uint64_t total = 0;
        for (uint32_t w = 0; w < n_windows; ++w) {
            const uint8_t h = S.hits[w];
            total += (uint64_t)((h & 1) + ((h >> 1) & 1) + ((h >> 2) & 1)); /* vectorSum x3, 590-593 */
            if (levels) levels[(size_t)c * n_windows + w] = h;
        }
        counts[c] = total;
    }
    free(S.hits);
    return 0;
}
