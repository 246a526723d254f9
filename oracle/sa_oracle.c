/* TEST INFRASTRUCTURE ONLY — CPU checker; see sa_oracle.h for the contract and who may call it.
 *
 * A deliberately plain restatement of the reference's O(mn) full-matrix algorithms: row-major
 * int32 matrices of (m+1)x(n+1), a byte match cache, scalar loops in the reference's order and
 * its exact comparison / tie rules.  Integer overflow wraps (-fwrapv), like the compiled
 * reference does in practice; scorings that overflow are outside parity anyway.
 */
#include "sa_oracle.h"

#include <limits.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define IDX(i, j) ((size_t)(i) * (size_t)(n + 1) + (size_t)(j))

static inline int32_t max2(int32_t a, int32_t b) { return a > b ? a : b; }
static inline int32_t max3(int32_t a, int32_t b, int32_t c) { return max2(max2(a, b), c); }
static inline int32_t max4(int32_t a, int32_t b, int32_t c, int32_t d) { return max2(max3(a, b, c), d); }

/* cacheAllMatches (e.g. SASmithWaterman.h:20-45): Matches[i*n+j] = match(Seq1[i], Seq2[j]). */
static uint8_t* match_cache(const uint8_t* s1, int m, const uint8_t* s2, int n, const uint8_t* lut) {
    uint8_t* mt = (uint8_t*)malloc((size_t)m * (size_t)n + 1);
    if (!mt) return NULL;
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j)
            mt[(size_t)i * n + j] = lut ? (lut[s1[i] * 256 + s2[j]] != 0) : (s1[i] == s2[j]);
    return mt;
}

/* Diagonal candidate exactly as the fill computes it (SASmithWaterman.h:95-100 / :128-131). */
static inline int32_t diag_term(int32_t hd, int v, const oracle_scoring* sc) {
    if (sc->allow_mismatch) return hd + (v ? sc->match : sc->mismatch);
    return v ? hd + sc->match : INT_MIN;
}

typedef struct {
    uint8_t* ops;
    int cap, n;
    int overflow;
} opbuf;

static inline void put(opbuf* b, uint8_t op) {
    if (b->n < b->cap) b->ops[b->n] = op; else b->overflow = 1;
    b->n++;
}

/* Expand an op stream + forceGlobal (SequenceAlignment.h:156-189) into three strings. */
static int expand(const uint8_t* s1, int m, const uint8_t* s2, int n, const uint8_t* ops, int nops,
                  int end_i, int end_j, int force_global, int fg_i, int fg_j, int fg_ei, int fg_ej,
                  char* row0, char* bars, char* row1, int cap, int* out_len) {
    /* Build the local part in reverse (traceback order), then emit forward. */
    int local = 0;
    for (int k = 0; k < nops; ++k) local += (ops[k] == 'X') ? 2 : 1;
    int front = force_global ? fg_i + fg_j : 0;
    int back = force_global ? (m - fg_ei) + (n - fg_ej) : 0;
    int len = front + local + back;
    *out_len = len;
    if (!row0) return 0;
    if (len > cap) return -1;
    int p = 0;
    if (force_global) {
        for (int k = 0; k < fg_i; ++k, ++p) { row0[p] = (char)s1[k]; bars[p] = ' '; row1[p] = '-'; }
        for (int k = 0; k < fg_j; ++k, ++p) { row0[p] = '-'; bars[p] = ' '; row1[p] = (char)s2[k]; }
    }
    /* Walk the traceback to recover the positions each op consumed, writing from the back. */
    int q = p + local;
    int i = end_i, j = end_j;
    for (int k = 0; k < nops; ++k) {
        uint8_t op = ops[k];
        if (op == 'M' || op == 'S') {
            --q; row0[q] = (char)s1[i - 1]; bars[q] = op == 'M' ? '|' : ' '; row1[q] = (char)s2[j - 1];
            --i; --j;
        } else if (op == 'X') {
            /* push_front(Seq1,Blank) then push_front(Blank,Seq2): forward order (-,s2),(s1,-) */
            --q; row0[q] = (char)s1[i - 1]; bars[q] = ' '; row1[q] = '-';
            --q; row0[q] = '-'; bars[q] = ' '; row1[q] = (char)s2[j - 1];
            --i; --j;
        } else if (op == 'U' || op == 'u') {
            --q; row0[q] = (char)s1[i - 1]; bars[q] = ' '; row1[q] = '-';
            if (op == 'U') --i;
        } else { /* 'L' / 'l' */
            --q; row0[q] = '-'; bars[q] = ' '; row1[q] = (char)s2[j - 1];
            if (op == 'L') --j;
        }
    }
    p += local;
    if (force_global) {
        for (int k = fg_ei; k < m; ++k, ++p) { row0[p] = (char)s1[k]; bars[p] = ' '; row1[p] = '-'; }
        for (int k = fg_ej; k < n; ++k, ++p) { row0[p] = '-'; bars[p] = ' '; row1[p] = (char)s2[k]; }
    }
    return 0;
}

/* ---------------------------------------------------------------- Smith-Waterman (linear) */
static int align_sw(const oracle_scoring* sc, const uint8_t* s1, int m, const uint8_t* s2, int n,
                    const uint8_t* mt, oracle_result* res, opbuf* ob) {
    (void)s1; (void)s2;
    int32_t* H = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m + 1) * (size_t)(n + 1));
    if (!H) return -2;
    const int32_t G = sc->gap;
    for (int i = 0; i <= m; ++i) H[IDX(i, 0)] = 0;            /* SASmithWaterman.h:68-71 */
    for (int j = 0; j <= n; ++j) H[IDX(0, j)] = 0;            /* :74-77 */
    int32_t best = INT_MIN;
    int maxr = 0, maxc = 0;                                   /* members default to 0 (:14-15) */
    for (int i = 1; i <= m; ++i)
        for (int j = 1; j <= n; ++j) {
            int v = mt[(size_t)(i - 1) * n + (j - 1)];
            int32_t h = max4(diag_term(H[IDX(i - 1, j - 1)], v, sc), H[IDX(i - 1, j)] + G,
                             H[IDX(i, j - 1)] + G, 0);        /* :95-104 */
            H[IDX(i, j)] = h;
            if (h >= best) { best = h; maxr = i; maxc = j; }  /* :110-115, last row-major max */
        }
    /* buildResult :220-339 */
    int i = maxr, j = maxc;
    if (m == 0 || n == 0) { i = 0; j = 0; }
    while (i > 0 || j > 0) {
        if (i == 0 || j == 0) break;
        int v = mt[(size_t)(i - 1) * n + (j - 1)];
        int32_t s = max2(diag_term(H[IDX(i - 1, j - 1)], v, sc), 0);
        if (H[IDX(i, j)] == s) {
            if (s == 0) break;
            put(ob, (v || sc->allow_mismatch) ? (v ? 'M' : 'S') : 'X');
            --i; --j;
            continue;
        }
        if (i > 0 && H[IDX(i, j)] == H[IDX(i - 1, j)] + G) {
            if (H[IDX(i - 1, j)] + G <= 0) break;
            put(ob, 'U'); --i;
        } else {
            if (H[IDX(i, j - 1)] + G <= 0) break;
            put(ob, 'L'); --j;
        }
    }
    res->score = (m == 0 || n == 0) ? INT_MIN : best;
    res->end_i = maxr; res->end_j = maxc;
    res->start_i = i; res->start_j = j;
    free(H);
    return 0;
}

/* ------------------------------------------------------------- Needleman-Wunsch (linear) */
static int align_nw(const oracle_scoring* sc, const uint8_t* s1, int m, const uint8_t* s2, int n,
                    const uint8_t* mt, oracle_result* res, opbuf* ob) {
    (void)s1; (void)s2;
    int32_t* H = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m + 1) * (size_t)(n + 1));
    if (!H) return -2;
    const int32_t G = sc->gap;
    for (int i = 0; i <= m; ++i) H[IDX(i, 0)] = (int32_t)((uint32_t)i * (uint32_t)G);  /* :59-60 */
    for (int j = 0; j <= n; ++j) H[IDX(0, j)] = (int32_t)((uint32_t)j * (uint32_t)G);  /* :61-62 */
    for (int i = 1; i <= m; ++i)
        for (int j = 1; j <= n; ++j) {
            int v = mt[(size_t)(i - 1) * n + (j - 1)];
            H[IDX(i, j)] = max3(diag_term(H[IDX(i - 1, j - 1)], v, sc), H[IDX(i - 1, j)] + G,
                                H[IDX(i, j - 1)] + G);         /* :73-78 */
        }
    int i = m, j = n;                                          /* buildResult :167 */
    while (i > 0 || j > 0) {
        if (i > 0 && j > 0) {
            int v = mt[(size_t)(i - 1) * n + (j - 1)];
            if (H[IDX(i, j)] == diag_term(H[IDX(i - 1, j - 1)], v, sc)) {
                put(ob, (v || sc->allow_mismatch) ? (v ? 'M' : 'S') : 'X');
                --i; --j;
                continue;
            }
        }
        if (i > 0 && H[IDX(i, j)] == H[IDX(i - 1, j)] + G) { put(ob, 'U'); --i; }
        else { put(ob, 'L'); --j; }
    }
    res->score = H[IDX(m, n)];
    res->end_i = m; res->end_j = n;
    res->start_i = 0; res->start_j = 0;
    free(H);
    return 0;
}

/* --------------------------------------------------------------------- Gotoh (affine) */
static int align_gotoh(int local, const oracle_scoring* sc, int m, int n, const uint8_t* mt,
                       oracle_result* res, opbuf* ob) {
    size_t cells = (size_t)(m + 1) * (size_t)(n + 1);
    int32_t* M = (int32_t*)malloc(sizeof(int32_t) * cells);
    int32_t* X = (int32_t*)malloc(sizeof(int32_t) * cells); /* Ix: vertical gap (consumes Seq1) */
    int32_t* Y = (int32_t*)malloc(sizeof(int32_t) * cells); /* Iy: horizontal gap (consumes Seq2) */
    if (!M || !X || !Y) { free(M); free(X); free(Y); return -2; }
    const int32_t GO = sc->gap_open, GE = sc->gap_extend;
    for (int i = 0; i <= m; ++i) {   /* LG :77-82, GG :75-80 */
        M[IDX(i, 0)] = local ? 0 : (i < 1 ? 0 : (int32_t)((uint32_t)GO + (uint32_t)i * (uint32_t)GE));
        X[IDX(i, 0)] = -10000;
        Y[IDX(i, 0)] = -10000;
    }
    for (int j = 0; j <= n; ++j) {   /* LG :85-90, GG :83-88 */
        M[IDX(0, j)] = local ? 0 : (j < 1 ? 0 : (int32_t)((uint32_t)GO + (uint32_t)j * (uint32_t)GE));
        X[IDX(0, j)] = -10000;
        Y[IDX(0, j)] = -10000;
    }
    int32_t best = INT_MIN;
    int maxr = 0, maxc = 0;
    for (int i = 1; i <= m; ++i)
        for (int j = 1; j <= n; ++j) {
            int32_t x = max2(M[IDX(i - 1, j)] + GO + GE, X[IDX(i - 1, j)] + GE);   /* :108-112 */
            int32_t y = max2(M[IDX(i, j - 1)] + GO + GE, Y[IDX(i, j - 1)] + GE);   /* :115-119 */
            int v = mt[(size_t)(i - 1) * n + (j - 1)];
            int32_t d = diag_term(M[IDX(i - 1, j - 1)], v, sc);
            int32_t h = local ? max4(d, x, y, 0) : max3(d, x, y);                    /* :122-130 */
            X[IDX(i, j)] = x; Y[IDX(i, j)] = y; M[IDX(i, j)] = h;
            if (local && h >= best) { best = h; maxr = i; maxc = j; }                /* :133-138 */
        }
    int rc = 0;
    int type = 0;
    int i, j;
    if (local) {
        /* SALocalGotoh.h buildResult :275-473 */
        i = maxr; j = maxc;
        while (i > 0 || j > 0) {
            if (i <= 0 || j <= 0) break;
            if (type == 0) {
                int v = mt[(size_t)(i - 1) * n + (j - 1)];
                int32_t s = max2(diag_term(M[IDX(i - 1, j - 1)], v, sc), 0);
                if (M[IDX(i, j)] == s) {
                    if (s <= 0) break;
                    put(ob, (v || sc->allow_mismatch) ? (v ? 'M' : 'S') : 'X');
                    --i; --j;
                    continue;
                }
            }
            {
                int32_t mup = max2(M[IDX(i - 1, j)] + GO + GE, 0);
                int32_t xup = X[IDX(i - 1, j)] + GE;
                if (X[IDX(i, j)] == xup && type == 1) { put(ob, 'U'); --i; continue; }
                if (X[IDX(i, j)] == mup && type == 1) {
                    if (mup <= 0) { put(ob, 'u'); break; }
                    put(ob, 'U'); type = 0; --i; continue;
                }
                if (M[IDX(i, j)] == X[IDX(i, j)] && type == 0) { type = 1; continue; }
            }
            {
                int32_t mleft = max2(M[IDX(i, j - 1)] + GO + GE, 0);
                int32_t yleft = Y[IDX(i, j - 1)] + GE;
                if (Y[IDX(i, j)] == yleft && type == 2) { put(ob, 'L'); --j; continue; }
                if (Y[IDX(i, j)] == mleft && type == 2) {
                    if (mleft <= 0) { put(ob, 'l'); break; }
                    put(ob, 'L'); type = 0; --j; continue;
                }
                if (M[IDX(i, j)] == Y[IDX(i, j)] && type == 0) { type = 2; continue; }
            }
            rc = -3; /* the reference loops forever here (undefined scoring); outside parity */
            break;
        }
        (void)best;
        res->score = M[IDX(maxr, maxc)]; /* harness reads Matrix[MaxRow][MaxCol] */
        res->end_i = maxr; res->end_j = maxc;
    } else {
        /* SAGlobalGotoh.h buildResult :235-422 */
        i = m; j = n;
        while (i > 0 || j > 0) {
            if (i > 0 && j > 0 && type == 0) {
                int v = mt[(size_t)(i - 1) * n + (j - 1)];
                if (M[IDX(i, j)] == diag_term(M[IDX(i - 1, j - 1)], v, sc)) {
                    put(ob, (v || sc->allow_mismatch) ? (v ? 'M' : 'S') : 'X');
                    --i; --j;
                    continue;
                }
            }
            if (i > 0) {
                if (j == 0) { put(ob, 'U'); --i; continue; }
                int32_t mup = M[IDX(i - 1, j)] + GO + GE;
                int32_t xup = X[IDX(i - 1, j)] + GE;
                if (X[IDX(i, j)] == xup && type == 1) { put(ob, 'U'); --i; continue; }
                if (X[IDX(i, j)] == mup && type == 1) { put(ob, 'U'); type = 0; --i; continue; }
                if (M[IDX(i, j)] == X[IDX(i, j)] && type == 0) { type = 1; continue; }
            }
            if (j > 0) {
                if (i == 0) { put(ob, 'L'); --j; continue; }
                int32_t mleft = M[IDX(i, j - 1)] + GO + GE;
                int32_t yleft = Y[IDX(i, j - 1)] + GE;
                if (Y[IDX(i, j)] == yleft && type == 2) { put(ob, 'L'); --j; continue; }
                if (Y[IDX(i, j)] == mleft && type == 2) { put(ob, 'L'); type = 0; --j; continue; }
                if (M[IDX(i, j)] == Y[IDX(i, j)] && type == 0) { type = 2; continue; }
            }
            rc = -3;
            break;
        }
        res->score = M[IDX(m, n)];
        res->end_i = m; res->end_j = n;
    }
    res->start_i = i; res->start_j = j;
    free(M); free(X); free(Y);
    return rc;
}

/* ------------------------------------------------------- Hirschberg (SAHirschberg.h) */
/* match(Seq1[i], Seq2[j]) by position: bytes through the LUT / equality, or (generic-Ty form)
 * the caller's m x n match matrix mt -- what the reference's MatchFnTy returns per cell
 * (SAHirschberg.h:74, :90; SAMyersMiller.h:24-37 caches the same per recursion). */
typedef struct {
    const uint8_t *s1, *s2, *lut;
    const uint8_t* mt;       /* NULL: byte symbols */
    int n;                   /* row length of mt */
} pos_match;

static inline int match_at(const pos_match* p, int i, int j) {
    if (p->mt) return p->mt[(size_t)i * (size_t)p->n + (size_t)j] != 0;
    return p->lut ? p->lut[p->s1[i] * 256 + p->s2[j]] != 0 : p->s1[i] == p->s2[j];
}

/* the match cache of the sub-block [a0, a0+m) x [b0, b0+n) */
static uint8_t* match_block(const pos_match* p, int a0, int m, int b0, int n) {
    uint8_t* mt = (uint8_t*)malloc((size_t)m * (size_t)n + 1);
    if (!mt) return NULL;
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) mt[(size_t)i * n + j] = (uint8_t)match_at(p, a0 + i, b0 + j);
    return mt;
}

typedef struct {
    const oracle_scoring* sc;
    pos_match pm;
    int32_t *F, *A, *C;      /* FinalScore, ScoreAux, ScoreCache (n+1 each), :174-178 */
    uint8_t* fwd;            /* forward-order op list of the whole alignment */
    int nf;
    int err;
} hb_ctx;

/* NWScore (:11-100): last row of NW over Seq1[a0..a0+alen) x Seq2[b0..b0+blen), each read
 * forwards or (rev) backwards, into h->F[0..blen]. */
static void hb_nwscore(hb_ctx* h, int a0, int alen, int arev, int b0, int blen, int brev) {
    const int32_t G = h->sc->gap, MA = h->sc->match;
    const int allow = h->sc->allow_mismatch;
    const int32_t MI = allow ? h->sc->mismatch : INT_MIN;
    int32_t *F = h->F, *A = h->A;
    F[0] = 0;
    for (int j = 1; j <= blen; ++j) F[j] = F[j - 1] + G;
    for (int i = 1; i <= alen; ++i) {
        const int ai = arev ? a0 + alen - i : a0 + i - 1;
        A[0] = F[0] + G;
        for (int j = 1; j <= blen; ++j) {
            const int bj = brev ? b0 + blen - j : b0 + j - 1;
            const int v = match_at(&h->pm, ai, bj);
            const int32_t sub = allow ? F[j - 1] + (v ? MA : MI) : (v ? F[j - 1] + MA : MI);
            A[j] = max3(sub, F[j] + G, A[j - 1] + G);
        }
        int32_t* t = F; F = A; A = t;
    }
    h->F = F; h->A = A;
}

static void hb_put(hb_ctx* h, uint8_t op) { h->fwd[h->nf++] = op; }

/* HirschbergRec (:102-163) over s1[a0..a0+alen) x s2[b0..b0+blen); appends forward ops. */
static void hb_rec(hb_ctx* h, int a0, int alen, int b0, int blen) {
    if (h->err) return;
    if (alen == 0) {
        for (int k = 0; k < blen; ++k) hb_put(h, 'L');   /* Entry(Blank, Char) */
    } else if (blen == 0) {
        for (int k = 0; k < alen; ++k) hb_put(h, 'U');   /* Entry(Char, Blank) */
    } else if (alen == 1 || blen == 1) {
        /* NeedlemanWunschSA::getAlignment on the two views, spliced at the end (:119-126) */
        uint8_t* mt = match_block(&h->pm, a0, alen, b0, blen);
        uint8_t* tb = (uint8_t*)malloc((size_t)(alen + blen) + 1);
        if (!mt || !tb) { free(mt); free(tb); h->err = -2; return; }
        opbuf ob = {tb, alen + blen + 1, 0, 0};
        oracle_result r;
        if (align_nw(h->sc, NULL, alen, NULL, blen, mt, &r, &ob)) h->err = -2;
        for (int k = ob.n - 1; k >= 0; --k) hb_put(h, tb[k]);   /* traceback order -> forward */
        free(mt); free(tb);
    } else {
        const int mid = alen / 2;
        hb_nwscore(h, a0, mid, 0, b0, blen, 0);
        memcpy(h->C, h->F, sizeof(int32_t) * (size_t)(blen + 1));          /* swap into ScoreCache */
        hb_nwscore(h, a0 + mid, alen - mid, 1, b0, blen, 1);
        int mid2 = 0;
        int32_t best = INT_MIN;
        for (int i = 0; i < blen; ++i) {                                  /* :138-149, i < size */
            const int32_t sc = h->C[i] + h->F[blen - i];
            if (sc >= best) { best = sc; mid2 = i; }
        }
        hb_rec(h, a0, mid, b0, mid2);
        hb_rec(h, a0 + mid, alen - mid, b0 + mid2, blen - mid2);
    }
}

static int align_hirschberg(const oracle_scoring* sc, const pos_match* pm, int m, int n, oracle_result* res,
                            opbuf* ob) {
    hb_ctx h;
    memset(&h, 0, sizeof(h));
    h.sc = sc; h.pm = *pm;
    h.F = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1) * 3);
    h.fwd = (uint8_t*)malloc((size_t)(m + n) + 1);
    if (!h.F || !h.fwd) { free(h.F); free(h.fwd); return -2; }
    h.A = h.F + (n + 1);
    h.C = h.A + (n + 1);
    int32_t* base = h.F;
    hb_nwscore(&h, 0, m, 0, 0, n, 0);                   /* score: NW H[m][n] */
    res->score = h.F[n];
    hb_rec(&h, 0, m, 0, n);
    for (int k = h.nf - 1; k >= 0; --k) put(ob, h.fwd[k]);   /* back to traceback order */
    res->end_i = m; res->end_j = n;
    res->start_i = 0; res->start_j = 0;
    free(base);
    free(h.fwd);
    return h.err;
}

/* ----------------------------------------------------- Myers–Miller (SAMyersMiller.h) */
typedef struct {
    const oracle_scoring* sc;
    pos_match pm;
    int32_t *C, *D, *Cr, *Dr;   /* CC, DD (:167-168) and RR, SS (:242-243), n+1 each */
    uint8_t* fwd;               /* forward-order op list of the whole alignment */
    int nf;
    int top_done;
    int32_t score;              /* the top call's optimum (see align_myers_miller) */
} mm_ctx;

/* The forward sweep of buildResultRec (:172-238) over Seq1[a0..a0+alen) x Seq2[b0..b0+blen), each
 * read forwards or (rev) backwards, with row-0 gap open t0 (tb).  Read backwards with t0 = te it
 * is the reverse sweep (:247-313) in reversed coordinates: RR[j] = C[blen-j], SS[j] = D[blen-j]. */
static void mm_sweep(mm_ctx* h, int a0, int alen, int rev, int b0, int blen, int32_t t0, int32_t* C, int32_t* D) {
    const int32_t g = h->sc->gap_open, x = h->sc->gap_extend, MA = h->sc->match;
    const int allow = h->sc->allow_mismatch;
    const int32_t MI = allow ? h->sc->mismatch : INT_MIN;
    int32_t t = g;
    C[0] = 0;
    for (int j = 1; j <= blen; ++j) { t += x; C[j] = t; D[j] = t + g; }   /* :183-188 */
    t = t0;
    for (int i = 1; i <= alen; ++i) {
        const int ai = rev ? a0 + alen - i : a0 + i - 1;
        int32_t s = C[0];
        t += x;
        int32_t c = t;
        C[0] = c;
        int32_t e = t + g;
        for (int j = 1; j <= blen; ++j) {
            const int bj = rev ? b0 + blen - j : b0 + j - 1;
            e = (e > c + g ? e : c + g) + x;
            D[j] = (D[j] > C[j] + g ? D[j] : C[j] + g) + x;
            const int v = match_at(&h->pm, ai, bj);
            const int32_t diag = (allow || v) ? s + (v ? MA : MI) : INT_MIN;   /* :218-232 */
            c = max3(D[j], e, diag);
            s = C[j];
            C[j] = c;
        }
    }
    D[0] = C[0];   /* :238 (and SS[N] = RR[N], :313) */
}

static void mm_put(mm_ctx* h, uint8_t op) { h->fwd[h->nf++] = op; }

/* buildResultRec (:44-397) over s1[a0..a0+M) x s2[b0..b0+N) with boundary gap opens tb, te;
 * appends forward-order ops. */
static void mm_rec(mm_ctx* h, int a0, int M, int b0, int N, int32_t tb, int32_t te) {
    const int32_t g = h->sc->gap_open, x = h->sc->gap_extend, MA = h->sc->match;
    const int allow = h->sc->allow_mismatch;
    const int32_t MI = allow ? h->sc->mismatch : INT_MIN;
    const int top = !h->top_done;
    h->top_done = 1;
    if (N == 0) {                                                     /* :57-66 */
        for (int k = 0; k < M; ++k) mm_put(h, 'U');
        if (top) h->score = M > 0 ? tb + x * M : 0;
    } else if (M == 0) {                                              /* :67-74 */
        for (int k = 0; k < N; ++k) mm_put(h, 'L');
        if (top) h->score = g + x * N;
    } else if (M == 1) {                                              /* :75-160 */
        const int32_t base = (tb > te ? tb : te) + x + (g + x * N);
        int32_t best = INT_MIN;
        int index = 0;
        for (int j = 1; j <= N; ++j) {
            const int v = match_at(&h->pm, a0, b0 + j - 1);
            int32_t t = base;
            if (allow || v) {
                const int32_t via = g + x * (j - 1) + (v ? MA : MI) + g + x * (N - j);
                if (via > t) t = via;
            }
            if (t > best) { best = t; index = j; }
        }
        for (int j = 1; j <= N; ++j) {
            if (j == index) {
                const int v = match_at(&h->pm, a0, b0 + j - 1);
                if (!allow && !v) {          /* :141-147: (a, Blank) then (Blank, b) */
                    mm_put(h, 'U');
                    mm_put(h, 'L');
                } else {
                    mm_put(h, v ? 'M' : 'S');  /* :148-152 */
                }
            } else {
                mm_put(h, 'L');
            }
        }
        if (top) h->score = best;
    } else {
        const int mid = M / 2;
        mm_sweep(h, a0, mid, 0, b0, N, tb, h->C, h->D);
        mm_sweep(h, a0 + mid, M - mid, 1, b0, N, te, h->Cr, h->Dr);
        int index = 0, type2 = 0;
        int32_t best = INT_MIN;
        for (int j = 0; j <= N; ++j) {                                /* :320-340 */
            const int32_t c1 = h->C[j] + h->Cr[N - j];
            const int32_t c2 = h->D[j] + h->Dr[N - j] - g;
            const int32_t t = c1 > c2 ? c1 : c2;
            if (t > best) { best = t; index = j; type2 = !(c1 > c2); }
        }
        if (top) h->score = best;
        if (!type2) {                                                 /* :358-374 */
            mm_rec(h, a0, mid, b0, index, tb, g);
            mm_rec(h, a0 + mid, M - mid, b0 + index, N - index, g, te);
        } else {                                                      /* :375-395 */
            mm_rec(h, a0, mid - 1, b0, index, tb, 0);
            mm_put(h, 'U');
            mm_put(h, 'U');
            mm_rec(h, a0 + mid + 1, M - mid - 1, b0 + index, N - index, 0, te);
        }
    }
}

/* MyersMillerSA::getAlignment (:412-420): buildResultRec(.., M, N, GapOpen, GapOpen).  The
 * reference exposes no score; res->score is the optimum the top call computes (its midpoint
 * maximum :320-340, the M == 1 maximum :81-124, or the boundary value of an empty side). */
static int align_myers_miller(const oracle_scoring* sc, const pos_match* pm, int m, int n, oracle_result* res,
                              opbuf* ob) {
    mm_ctx h;
    memset(&h, 0, sizeof(h));
    h.sc = sc; h.pm = *pm;
    int32_t* base = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1) * 4);
    h.fwd = (uint8_t*)malloc((size_t)(m + n) + 1);
    if (!base || !h.fwd) { free(base); free(h.fwd); return -2; }
    h.C = base; h.D = base + (n + 1); h.Cr = base + 2 * (n + 1); h.Dr = base + 3 * (n + 1);
    mm_rec(&h, 0, m, 0, n, sc->gap_open, sc->gap_open);
    for (int k = h.nf - 1; k >= 0; --k) put(ob, h.fwd[k]);   /* back to traceback order */
    res->score = h.score;
    res->end_i = m; res->end_j = n;
    res->start_i = 0; res->start_j = 0;
    free(base);
    free(h.fwd);
    return 0;
}

/* SALocalGotoh.h:484-488: these three size pairs discard the Gotoh result and run
 * StaticFuncs::useNW (StaticFuncs.h:12-25) with the same (affine) ScoringSystem. */
static int lg_size_hack(int m, int n) {
    return (m == 314 && n == 288) || (m == 60 && n == 57) || (m == 61 && n == 58);
}

int oracle_align(int algo, const oracle_scoring* sc, const uint8_t* s1, int m, const uint8_t* s2,
                 int n, const uint8_t* lut, oracle_result* res, uint8_t* ops, int ops_cap,
                 char* row0, char* bars, char* row1, int cap) {
    if (algo == OR_LOCAL_GOTOH && lg_size_hack(m, n)) algo = OR_NW;
    if (algo == OR_HIRSCHBERG || algo == OR_MYERS_MILLER) {
        opbuf hb = {ops, ops_cap, 0, 0};
        memset(res, 0, sizeof(*res));
        const pos_match pm = {s1, s2, lut, NULL, n};
        int rc = algo == OR_HIRSCHBERG ? align_hirschberg(sc, &pm, m, n, res, &hb)
                                       : align_myers_miller(sc, &pm, m, n, res, &hb);
        res->nops = hb.n;
        if (rc) return rc;
        if (hb.overflow) return -1;
        int len = 0;
        int e = expand(s1, m, s2, n, ops, hb.n, m, n, 0, 0, 0, m, n, row0, bars, row1, cap, &len);
        res->len = len;
        return e;
    }
    uint8_t* mt = match_cache(s1, m, s2, n, lut);
    if (!mt) return -2;
    opbuf ob = {ops, ops_cap, 0, 0};
    memset(res, 0, sizeof(*res));
    int rc;
    switch (algo) {
        case OR_SW: rc = align_sw(sc, s1, m, s2, n, mt, res, &ob); break;
        case OR_NW: rc = align_nw(sc, s1, m, s2, n, mt, res, &ob); break;
        case OR_LOCAL_GOTOH: rc = align_gotoh(1, sc, m, n, mt, res, &ob); break;
        default: rc = align_gotoh(0, sc, m, n, mt, res, &ob); break;
    }
    free(mt);
    res->nops = ob.n;
    if (rc) return rc;
    if (ob.overflow) return -1;
    int fg = (algo == OR_SW || algo == OR_LOCAL_GOTOH);
    int len = 0;
    int e = expand(s1, m, s2, n, ops, ob.n, res->end_i, res->end_j, fg, res->start_i, res->start_j,
                   res->end_i, res->end_j, row0, bars, row1, cap, &len);
    res->len = len;
    return e;
}

/* ------------------------------------------------------------------ CPU baseline (port) */
typedef struct {
    const oracle_scoring* sc;
    const uint8_t *s1, *s2;
    const uint64_t *o1, *o2;
    int npairs;
    int32_t* out;
    volatile int next;
    pthread_mutex_t mu;
    int err;
    int algo;                 /* oracle_batch: algorithm, full results and op streams */
    oracle_result* res;
    uint8_t* ops;             /* pair p's ops at o1[p] + o2[p] + p */
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* J = (batch_job*)arg;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        int p = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (p >= J->npairs) break;
        int m = (int)(J->o1[p + 1] - J->o1[p]), n = (int)(J->o2[p + 1] - J->o2[p]);
        const uint8_t* a = J->s1 + J->o1[p];
        const uint8_t* b = J->s2 + J->o2[p];
        int cap = m + n + 2;
        uint8_t* ops = (uint8_t*)malloc((size_t)cap);
        char* r = (char*)malloc((size_t)cap * 3);
        oracle_result res;
        int rc = (ops && r) ? oracle_align(J->algo, J->sc, a, m, b, n, NULL, &res, ops, cap, r, r + cap,
                                           r + 2 * cap, cap)
                            : -2;
        if (J->out) J->out[p] = rc ? INT_MIN : res.score;
        if (J->res) {
            J->res[p] = res;
            memcpy(J->ops + J->o1[p] + J->o2[p] + p, ops, (size_t)res.nops);
        }
        if (rc) J->err = rc;
        free(ops); free(r);
    }
    return NULL;
}

int oracle_sw_batch(const oracle_scoring* sc, const uint8_t* s1cat, const uint64_t* off1,
                    const uint8_t* s2cat, const uint64_t* off2, int npairs, int threads,
                    int32_t* out_score) {
    if (threads < 1) threads = 1;
    batch_job J;
    J.sc = sc; J.s1 = s1cat; J.s2 = s2cat; J.o1 = off1; J.o2 = off2;
    J.npairs = npairs; J.out = out_score; J.next = 0; J.err = 0;
    J.algo = OR_SW; J.res = NULL; J.ops = NULL;
    pthread_mutex_init(&J.mu, NULL);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    if (!th) return -2;
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, batch_worker, &J);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&J.mu);
    return J.err;
}

/* Full results and op streams of a batch (test infrastructure: the GPU parity tests' checker at
 * large sizes), `threads` host threads, pair p's ops at off1[p] + off2[p] + p. */
int oracle_batch(int algo, const oracle_scoring* sc, const uint8_t* s1cat, const uint64_t* off1,
                 const uint8_t* s2cat, const uint64_t* off2, int npairs, int threads,
                 oracle_result* res, uint8_t* ops) {
    if (threads < 1) threads = 1;
    batch_job J;
    J.sc = sc; J.s1 = s1cat; J.s2 = s2cat; J.o1 = off1; J.o2 = off2;
    J.npairs = npairs; J.out = NULL; J.next = 0; J.err = 0;
    J.algo = algo; J.res = res; J.ops = ops;
    pthread_mutex_init(&J.mu, NULL);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    if (!th) return -2;
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, batch_worker, &J);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&J.mu);
    return J.err;
}

/* Score and end cell only, linear space: SW (SASmithWaterman.h:89-117) with byte equality as
 * the match fn -- the same recurrence, border and last row-major maximum as align_sw above, two
 * rows instead of the full matrix, so whole north-star batches can be checked on the host.
 * out[3p..3p+2] = (MaxScore, MaxRow, MaxCol); an empty side gives (INT_MIN, 0, 0). */
typedef struct {
    const oracle_scoring* sc;
    const uint8_t *s1, *s2;
    const uint64_t *o1, *o2;
    int npairs;
    int32_t* out;
    volatile int next;
    pthread_mutex_t mu;
} score_job;

static void sw_score_one(const oracle_scoring* sc, const uint8_t* a, int m, const uint8_t* b, int n,
                         int32_t* row, int32_t* out) {
    const int32_t G = sc->gap, MA = sc->match, MI = sc->mismatch;
    const int allow = sc->allow_mismatch;
    int32_t best = INT_MIN;
    int bi = 0, bj = 0;
    for (int j = 0; j <= n; ++j) row[j] = 0;
    for (int i = 1; i <= m; ++i) {
        int32_t diag = 0, left = 0;            /* H[i-1][0] and H[i][0] */
        const uint8_t ai = a[i - 1];
        for (int j = 1; j <= n; ++j) {
            const int32_t up = row[j];
            const int v = ai == b[j - 1];
            int32_t d = v ? diag + MA : (allow ? diag + MI : INT_MIN);
            int32_t h = d;
            if (up + G > h) h = up + G;
            if (left + G > h) h = left + G;
            if (h < 0) h = 0;
            diag = up;
            row[j] = h;
            left = h;
            if (h >= best) { best = h; bi = i; bj = j; }
        }
    }
    if (m == 0 || n == 0) { best = INT_MIN; bi = 0; bj = 0; }
    out[0] = best; out[1] = bi; out[2] = bj;
}

/* sw_score_one on 8 pairs of equal shape at once, lane l = pair l: the same recurrence, row-major
 * order and ">=" maximum per lane, written so the compiler vectorises the lane loop (the batch
 * checker of the 10,000 x 4096^2 headline would otherwise take minutes).  Pinned against
 * sw_score_one by tests/test_oracle_golden.py. */
#define SW8 8
typedef int32_t sw_v8 __attribute__((vector_size(32)));
typedef uint8_t sw_v8b __attribute__((vector_size(8)));
#define SW_AVX2 __attribute__((target("avx2")))
SW_AVX2 static inline sw_v8 sw_sel(sw_v8 mask, sw_v8 a, sw_v8 b) { return (mask & a) | (~mask & b); }
SW_AVX2 static void sw_score_x8(const oracle_scoring* sc, const uint8_t* const* a, const uint8_t* const* b, int m,
                        int n, sw_v8* rows, uint8_t* bt, int32_t* out) {
    const sw_v8 G = (sw_v8){0} + sc->gap, MA = (sw_v8){0} + sc->match, MI = (sw_v8){0} + sc->mismatch;
    const sw_v8 zero = (sw_v8){0}, neg = zero + INT_MIN;
    const int allow = sc->allow_mismatch;
    sw_v8 best = neg, bi = zero, bj = zero;
    for (int j = 0; j < n; ++j)
        for (int l = 0; l < SW8; ++l) bt[(size_t)j * SW8 + l] = b[l][j];
    for (int j = 0; j <= n; ++j) rows[j] = zero;
    for (int i = 1; i <= m; ++i) {
        sw_v8 diag = zero, left = zero, ai;
        for (int l = 0; l < SW8; ++l) ai[l] = a[l][i - 1];
        const sw_v8 iv = zero + i;
        for (int j = 1; j <= n; ++j) {
            sw_v8b bb;
            memcpy(&bb, bt + (size_t)(j - 1) * SW8, SW8);
            const sw_v8 bv = __builtin_convertvector(bb, sw_v8);
            const sw_v8 up = rows[j];
            const sw_v8 dx = allow ? diag + MI : neg;
            sw_v8 h = sw_sel(ai == bv, diag + MA, dx);
            const sw_v8 u = up + G, lf = left + G;
            h = sw_sel(u > h, u, h);
            h = sw_sel(lf > h, lf, h);
            h = sw_sel(h < zero, zero, h);
            diag = up;
            rows[j] = h;
            left = h;
            const sw_v8 take = h >= best;
            best = sw_sel(take, h, best);
            bi = sw_sel(take, iv, bi);
            bj = sw_sel(take, zero + j, bj);
        }
    }
    for (int l = 0; l < SW8; ++l) {
        const int e = m == 0 || n == 0;
        out[3 * l] = e ? INT_MIN : best[l];
        out[3 * l + 1] = e ? 0 : bi[l];
        out[3 * l + 2] = e ? 0 : bj[l];
    }
}

static void* score_worker(void* arg) {
    score_job* J = (score_job*)arg;
    int32_t* row = NULL;
    uint8_t* bt = NULL;
    int cap = -1;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const int p0 = J->next;
        J->next += SW8;
        pthread_mutex_unlock(&J->mu);
        if (p0 >= J->npairs) break;
        const int p1 = p0 + SW8 <= J->npairs ? p0 + SW8 : J->npairs;
        const int m = (int)(J->o1[p0 + 1] - J->o1[p0]), n = (int)(J->o2[p0 + 1] - J->o2[p0]);
        int same = p1 - p0 == SW8, nmax = 0;
        for (int p = p0; p < p1; ++p) {
            const int mp = (int)(J->o1[p + 1] - J->o1[p]), np = (int)(J->o2[p + 1] - J->o2[p]);
            same = same && mp == m && np == n;
            nmax = np > nmax ? np : nmax;
        }
        if (nmax > cap) {
            free(row);
            free(bt);
            row = (int32_t*)aligned_alloc(32, sizeof(int32_t) * ((size_t)nmax + 1) * SW8);
            bt = (uint8_t*)malloc((size_t)nmax * SW8 + 1);
            cap = nmax;
        }
        if (same && __builtin_cpu_supports("avx2")) {
            const uint8_t* a[SW8];
            const uint8_t* b[SW8];
            for (int l = 0; l < SW8; ++l) { a[l] = J->s1 + J->o1[p0 + l]; b[l] = J->s2 + J->o2[p0 + l]; }
            sw_score_x8(J->sc, a, b, m, n, (sw_v8*)row, bt, J->out + 3 * (size_t)p0);
        } else {
            for (int p = p0; p < p1; ++p)
                sw_score_one(J->sc, J->s1 + J->o1[p], (int)(J->o1[p + 1] - J->o1[p]), J->s2 + J->o2[p],
                             (int)(J->o2[p + 1] - J->o2[p]), row, J->out + 3 * (size_t)p);
        }
    }
    free(row);
    free(bt);
    return NULL;
}

int oracle_sw_score_batch(const oracle_scoring* sc, const uint8_t* s1cat, const uint64_t* off1,
                          const uint8_t* s2cat, const uint64_t* off2, int npairs, int threads,
                          int32_t* out) {
    if (threads < 1) threads = 1;
    score_job J;
    J.sc = sc; J.s1 = s1cat; J.s2 = s2cat; J.o1 = off1; J.o2 = off2;
    J.npairs = npairs; J.out = out; J.next = 0;
    pthread_mutex_init(&J.mu, NULL);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    if (!th) return -2;
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, score_worker, &J);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&J.mu);
    return 0;
}

/* Generic-Ty form (test infrastructure): the same aligners driven by a caller-supplied m x n
 * match matrix (mt[i*n + j] != 0 iff match(Seq1[i], Seq2[j]), the reference's cacheAllMatches)
 * instead of byte symbols; results and op stream only.  SW, NW, LocalGotoh (size hack included),
 * GlobalGotoh, HirschbergSA and MyersMillerSA. */
int oracle_align_matrix(int algo, const oracle_scoring* sc, int m, int n, const uint8_t* mt_in,
                        oracle_result* res, uint8_t* ops, int ops_cap) {
    if (algo == OR_LOCAL_GOTOH && lg_size_hack(m, n)) algo = OR_NW;
    if (algo == OR_HIRSCHBERG || algo == OR_MYERS_MILLER) {
        opbuf hb = {ops, ops_cap, 0, 0};
        memset(res, 0, sizeof(*res));
        const pos_match pm = {NULL, NULL, NULL, mt_in, n};
        int rc = algo == OR_HIRSCHBERG ? align_hirschberg(sc, &pm, m, n, res, &hb)
                                       : align_myers_miller(sc, &pm, m, n, res, &hb);
        res->nops = hb.n;
        if (rc) return rc;
        return hb.overflow ? -1 : 0;
    }
    uint8_t* mt = (uint8_t*)malloc((size_t)m * (size_t)n + 1);
    if (!mt) return -2;
    for (size_t k = 0; k < (size_t)m * (size_t)n; ++k) mt[k] = mt_in[k] != 0;
    opbuf ob = {ops, ops_cap, 0, 0};
    memset(res, 0, sizeof(*res));
    int rc;
    switch (algo) {
        case OR_SW: rc = align_sw(sc, NULL, m, NULL, n, mt, res, &ob); break;
        case OR_NW: rc = align_nw(sc, NULL, m, NULL, n, mt, res, &ob); break;
        case OR_LOCAL_GOTOH: rc = align_gotoh(1, sc, m, n, mt, res, &ob); break;
        default: rc = align_gotoh(0, sc, m, n, mt, res, &ob); break;
    }
    free(mt);
    res->nops = ob.n;
    if (rc) return rc;
    return ob.overflow ? -1 : 0;
}
