/*
 * cpg_oracle.c — CPU restatement of CpGIslandFinder's hot path (see cpg_oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY (the checker and the CPU baseline).  PARITY UNPINNED: no
 * reference build, no reference tests or golden vectors exist.
 *
 * Every function cites the reference line it follows.  Java semantics reproduced:
 *   - int arithmetic wraps (done in uint32_t, then reinterpreted),
 *   - double arithmetic in source order (IEEE binary64, round-to-nearest-even),
 *   - Math.log is taken as the C library log (Java allows 1 ulp; documented in
 *     DESIGN.md — the GPU path shares the host-computed constants).
 */
#include "cpg_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* CpGIslandFinder.java:155-173 */
void orc_initial_model(cpg_model* m) {
    static const double pi[8] = {0.05, 0.05, 0.05, 0.05, 0.2, 0.2, 0.2, 0.2};
    static const double a[8][8] = {
        {0.170, 0.274, 0.426, 0.120, 0.0025, 0.0025, 0.0025, 0.0025},
        {0.170, 0.358, 0.274, 0.188, 0.0025, 0.0025, 0.0025, 0.0025},
        {0.161, 0.329, 0.375, 0.125, 0.0025, 0.0025, 0.0025, 0.0025},
        {0.079, 0.345, 0.384, 0.182, 0.0025, 0.0025, 0.0025, 0.0025},
        {0.0025, 0.0025, 0.0025, 0.0025, 0.300, 0.205, 0.275, 0.210},
        {0.0025, 0.0025, 0.0025, 0.0025, 0.393, 0.137, 0.088, 0.372},
        {0.0025, 0.0025, 0.0025, 0.0025, 0.248, 0.246, 0.288, 0.208},
        {0.0025, 0.0025, 0.0025, 0.0025, 0.177, 0.239, 0.282, 0.292}};
    memcpy(m->pi, pi, sizeof pi);
    memcpy(m->a, a, sizeof a);
    memset(m->b, 0, sizeof m->b);
    for (int i = 0; i < 8; ++i) m->b[i][i % 4] = 1.0;
}

/* :114-123 / :240-249 */
static inline int sym_of(uint8_t ch) {
    switch (ch) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return -1;
    }
}

/* :112-145.  `count` is a Java int: the chunk test (count != 0 && count % 0x10000 == 0)
 * is evaluated after EVERY character, so a non-ACGT character read while count sits on a
 * multiple emits another chunk from the (empty) list: DenseVector(0x10000) all 0.0 = 'A'.
 * At 2^32 bases `count` wraps to 0 and the test is skipped: the list keeps its 65,536
 * bases, grows to 131,072 by the next multiple, and there `inputVector.set(65536, …)`
 * (:133-134) throws — the training run dies at the valid byte that brings count to
 * 2^32 + 65,536 (*crash_byte; returns the symbols of the chunks written before it).
 * count0: the Java `count` before the first byte (test hook: a stream that has already
 * read and committed count0 bases; a multiple of 65,536 below 2^32). */
int64_t orc_ingest_train_at(const uint8_t* txt, int64_t n, uint8_t* syms, int64_t cap,
                            uint32_t count0, int64_t* crash_byte) {
    uint32_t count = count0;         /* Java int, wraps */
    int64_t listlen = 0, out = 0;
    *crash_byte = -1;
    uint8_t* list = (uint8_t*)malloc(2 * CPG_TRAIN_CHUNK);   /* one skipped test at most */
    for (int64_t k = 0; k < n; ++k) {
        int v = sym_of(txt[k]);
        if (v != -1) {
            list[listlen++] = (uint8_t)v;
            count++;
        }
        if (count != 0 && (count & 0xFFFFu) == 0) {
            if (listlen > CPG_TRAIN_CHUNK) { *crash_byte = k; break; }   /* set(65536) */
            if (out + CPG_TRAIN_CHUNK > cap) { free(list); return -1; }
            memset(syms + out, 0, CPG_TRAIN_CHUNK);          /* new DenseVector: zeros */
            memcpy(syms + out, list, (size_t)listlen);        /* :133-135 */
            out += CPG_TRAIN_CHUNK;
            listlen = 0;                                      /* :136 */
        }
    }
    free(list);
    return out;                       /* tail (count % 65536 bases) never written */
}

int64_t orc_ingest_train(const uint8_t* txt, int64_t n, uint8_t* syms, int64_t cap) {
    int64_t cb;
    const int64_t r = orc_ingest_train_at(txt, n, syms, cap, 0u, &cb);
    return cb >= 0 ? -2 : r;
}

/* :238-259.  At 2^32 bases `count` wraps to 0 and the test is skipped: the list keeps its
 * 2^20 bases and keeps growing; at the next multiple the loop copies get(0..2^20-1) — the
 * held chunk — and clear() drops the 2^20 bases read after the wrap.  No exception; the
 * chunks after it are shifted (their `chunk` index counts decoded chunks, :287).  A
 * non-ACGT byte read while count == 0 fires nothing.  count0 as for the training reader
 * (a multiple of 2^20 below 2^32). */
int64_t orc_ingest_decode_at(const uint8_t* txt, int64_t n, uint8_t* syms, int64_t cap,
                             uint32_t count0, int* crash, int64_t* crash_byte) {
    uint32_t count = count0;
    int64_t listlen = 0, out = 0;
    *crash = 0;
    *crash_byte = -1;
    uint8_t* list = (uint8_t*)malloc(2 * CPG_DECODE_CHUNK);  /* one skipped test at most */
    for (int64_t k = 0; k < n; ++k) {
        int v = sym_of(txt[k]);
        if (v != -1) {
            list[listlen++] = (uint8_t)v;
            count++;
        }
        if (count != 0 && (count & 0xFFFFFu) == 0) {
            if (listlen < CPG_DECODE_CHUNK) {              /* get(i) on a short list */
                *crash = 1;
                *crash_byte = k;
                break;
            }
            if (out + CPG_DECODE_CHUNK > cap) { free(list); return -1; }
            memcpy(syms + out, list, CPG_DECODE_CHUNK);     /* get(0 .. 2^20-1) */
            out += CPG_DECODE_CHUNK;
            listlen = 0;                                     /* clear(): drops the rest */
        }
    }
    free(list);
    return out;
}

int64_t orc_ingest_decode(const uint8_t* txt, int64_t n, uint8_t* syms, int64_t cap,
                          int* crash) {
    int64_t cb;
    return orc_ingest_decode_at(txt, n, syms, cap, 0u, crash, &cb);
}

/* Mahout HmmAlgorithms.viterbiAlgorithm(sequence, delta, phi, model, obs, scaled=true),
 * called through HmmEvaluator.decode(trainedModel, testSequence, true) (:260). */
double orc_viterbi8(const cpg_model* m, const uint8_t* obs, int64_t T, int32_t* states_out) {
    double dprev[8], dcur[8];
    uint8_t* phi = (uint8_t*)malloc((size_t)(T > 1 ? T - 1 : 1) * 8);
    for (int i = 0; i < 8; ++i) dprev[i] = log(m->pi[i] * m->b[i][obs[0]]);
    for (int64_t t = 1; t < T; ++t) {
        for (int i = 0; i < 8; ++i) {
            /* Mahout's induction starts from candidate j = 0, not from a
             * sentinel: when every candidate is -inf (pi = 0 for both live states at t = 0)
             * delta stays -inf, maxState stays 0 and the final argmax leaves state 0 */
            int maxState = 0;
            double maxProb = dprev[0] + log(m->a[0][i]);
            for (int j = 1; j < 8; ++j) {
                double prob = dprev[j] + log(m->a[j][i]);
                if (prob > maxProb) { maxProb = prob; maxState = j; }
            }
            dcur[i] = maxProb + log(m->b[i][obs[t]]);
            phi[(t - 1) * 8 + i] = (uint8_t)maxState;
        }
        memcpy(dprev, dcur, sizeof dcur);
    }
    double maxProb = -INFINITY;
    states_out[T - 1] = 0;                          /* Java int[] starts zeroed */
    for (int i = 0; i < 8; ++i)
        if (dprev[i] > maxProb) { maxProb = dprev[i]; states_out[T - 1] = i; }
    for (int64_t t = T - 2; t >= 0; --t) states_out[t] = phi[t * 8 + states_out[t + 1]];
    free(phi);
    return maxProb;
}

/* SURVEY.md Appendix A.2, 2-state form: live states at t are o_t (+) and o_t+4 (-);
 * the + predecessor (index o_{t-1}) is visited before the - one (o_{t-1}+4), so ties go
 * to '+'; adding log(1.0) = +0.0 is exact.  Requires a deterministic emission matrix. */
double orc_viterbi2(const cpg_model* m, const uint8_t* obs, int64_t T, uint8_t* sign_out) {
    double L[4][4][4];   /* [p][b][k]  k: 0 = +->+, 1 = -->+, 2 = +->-, 3 = -->- */
    for (int p = 0; p < 4; ++p)
        for (int b = 0; b < 4; ++b) {
            L[p][b][0] = log(m->a[p][b]);
            L[p][b][1] = log(m->a[p + 4][b]);
            L[p][b][2] = log(m->a[p][b + 4]);
            L[p][b][3] = log(m->a[p + 4][b + 4]);
        }
    uint8_t* bp = (uint8_t*)malloc((size_t)(T > 1 ? T : 1));
    double P = log(m->pi[obs[0]] * m->b[obs[0]][obs[0]]);
    double M = log(m->pi[obs[0] + 4] * m->b[obs[0] + 4][obs[0]]);
    for (int64_t t = 1; t < T; ++t) {
        const double* l = L[obs[t - 1]][obs[t]];
        double cpp = P + l[0], cmp = M + l[1], cpm = P + l[2], cmm = M + l[3];
        int bP = cmp > cpp, bM = cmm > cpm;     /* 1: predecessor is '-' */
        P = (bP ? cmp : cpp) + 0.0;
        M = (bM ? cmm : cpm) + 0.0;
        bp[t] = (uint8_t)(bP | (bM << 1));
    }
    int s = (M > P) ? 0 : 1;                   /* + first: '-' wins only when strictly > */
    double best = s ? P : M;
    for (int64_t t = T - 1; t >= 0; --t) {
        sign_out[t] = (uint8_t)s;
        if (t > 0) s = s ? !(bp[t] & 1) : !(bp[t] & 2);
    }
    free(bp);
    return best;
}

/* SURVEY.md Appendix A.3 — Rabiner-rescaled forward-backward (MAHOUT-627 "rescaling"
 * mapper, unvendored; convention unpinned).  Accumulates expected counts. */
void orc_estep8(const cpg_model* m, const uint8_t* obs, int64_t T, cpg_counts_f64* acc) {
    double* al = (double*)malloc((size_t)T * 8 * sizeof(double));
    double* c = (double*)malloc((size_t)T * sizeof(double));
    double s = 0.0;
    for (int i = 0; i < 8; ++i) { al[i] = m->pi[i] * m->b[i][obs[0]]; s += al[i]; }
    c[0] = 1.0 / s;
    for (int i = 0; i < 8; ++i) al[i] *= c[0];
    for (int64_t t = 1; t < T; ++t) {
        double* ap = al + (t - 1) * 8;
        double* at = al + t * 8;
        s = 0.0;
        for (int j = 0; j < 8; ++j) {
            double x = 0.0;
            for (int i = 0; i < 8; ++i) x += ap[i] * m->a[i][j];
            at[j] = x * m->b[j][obs[t]];
            s += at[j];
        }
        c[t] = 1.0 / s;
        for (int j = 0; j < 8; ++j) at[j] *= c[t];
    }
    double ll = 0.0;
    for (int64_t t = 0; t < T; ++t) ll -= log(c[t]);
    acc->loglik += ll;

    double bn[8], bc[8];
    for (int i = 0; i < 8; ++i) bc[i] = 1.0;                  /* beta_{T-1} = 1 */
    for (int64_t t = T - 1; t >= 0; --t) {
        const double* at = al + t * 8;
        /* gamma_t */
        double den = 0.0;
        for (int k = 0; k < 8; ++k) den += at[k] * bc[k];
        for (int i = 0; i < 8; ++i) {
            double g = (at[i] * bc[i]) / den;
            acc->emit[i][obs[t]] += g;
            if (t == 0) acc->init[i] += g;
        }
        if (t == 0) break;
        /* beta_{t-1} and xi_{t-1} (needs alpha_{t-1}, a, b(o_t), beta_t) */
        const double* ap = al + (t - 1) * 8;
        double num[8][8];
        double dx = 0.0;
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 8; ++j) {
                num[i][j] = ((ap[i] * m->a[i][j]) * m->b[j][obs[t]]) * bc[j];
                dx += num[i][j];
            }
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 8; ++j) acc->trans[i][j] += num[i][j] / dx;
        for (int i = 0; i < 8; ++i) {
            double x = 0.0;
            for (int j = 0; j < 8; ++j) x += (m->a[i][j] * m->b[j][obs[t]]) * bc[j];
            bn[i] = x * c[t];
        }
        memcpy(bc, bn, sizeof bn);
    }
    free(al);
    free(c);
}

/* Reducer (MAHOUT-627, unvendored): sum of stripes then row normalisation. */
void orc_normalize(const cpg_counts_f64* c, cpg_model* out) {
    double s = 0.0;
    for (int i = 0; i < 8; ++i) s += c->init[i];
    for (int i = 0; i < 8; ++i) out->pi[i] = c->init[i] / s;
    for (int i = 0; i < 8; ++i) {
        double r = 0.0, e = 0.0;
        for (int j = 0; j < 8; ++j) r += c->trans[i][j];
        for (int j = 0; j < 8; ++j) out->a[i][j] = c->trans[i][j] / r;
        for (int k = 0; k < 4; ++k) e += c->emit[i][k];
        for (int k = 0; k < 4; ++k) out->b[i][k] = c->emit[i][k] / e;
    }
}

/* SURVEY.md §8 a6 (build-defined): state s_t = o_t + (sign_t ? 0 : 4). */
void orc_count_labelled(const uint8_t* obs, const uint8_t* sign, int64_t n,
                        int64_t chunk_len, cpg_counts_i64* acc) {
    int64_t nch = n / chunk_len;
    for (int64_t ch = 0; ch < nch; ++ch) {
        const uint8_t* o = obs + ch * chunk_len;
        const uint8_t* g = sign + ch * chunk_len;
        int sp = o[0] + (g[0] ? 0 : 4);
        acc->init[sp]++;
        acc->emit[sp][o[0]]++;
        acc->mono[o[0]]++;
        for (int64_t t = 1; t < chunk_len; ++t) {
            int s = o[t] + (g[t] ? 0 : 4);
            acc->trans[sp][s]++;
            acc->emit[s][o[t]]++;
            acc->dinuc[o[t - 1]][o[t]]++;
            acc->mono[o[t]]++;
            sp = s;
        }
    }
}

/* CpGIslandFinder.java:262-339 (state reset per chunk :262-268; int arithmetic). */
int64_t orc_islands(const int32_t* states, int64_t T, int32_t chunk, cpg_island* out,
                    int64_t cap) {
    int32_t beg = 0, cCount = 0, gCount = 0, cgCount = 0, islandLen = 0;
    int inIsland = 0, atC = 0;
    int64_t n = 0;
    /* chunk*0x100000 (int, wraps); for other chunk lengths: chunk*T */
    const uint32_t base = (uint32_t)chunk * (uint32_t)T;
    for (int64_t i = 0; i < T; ++i) {
        int32_t val = states[i];
        if (inIsland) {
            if (val == 4 || val == 5 || val == 6 || val == 7) {
                inIsland = 0;
                int32_t end = (int32_t)(i - 1);
                double ccnt = cCount, gcnt = gCount;
                double cgcontent = (ccnt + gcnt) / (double)islandLen;
                double oeratio = 0.0;
                if (cCount != 0 && gCount != 0) {
                    int32_t prod = (int32_t)((uint32_t)cgCount * (uint32_t)islandLen);
                    oeratio = (double)prod / (ccnt * gcnt);
                }
                if (cgcontent > 0.5 && oeratio > 0.6) {
                    if (n < cap) {
                        out[n].beg1 = (int32_t)((uint32_t)beg + base + 1u);
                        out[n].end1 = (int32_t)((uint32_t)end + base + 1u);
                        out[n].len = islandLen;
                        out[n].chunk = chunk;
                        out[n].cg = cgcontent;
                        out[n].oe = oeratio;
                    }
                    n++;
                }
            } else {
                islandLen++;
                if (val == 2) { gCount++; if (atC) cgCount++; }
                if (val == 1) { cCount++; atC = 1; } else atC = 0;
            }
        } else {
            if (val == 0 || val == 1 || val == 2 || val == 3) {
                inIsland = 1;
                islandLen = 1;
                cgCount = 0;
                beg = (int32_t)i;
                if (val == 1) { cCount = 1; atC = 1; } else cCount = 0;   /* atC kept */
                gCount = (val == 2) ? 1 : 0;
            }
        }
    }
    return n;                    /* an island still open at the chunk end is dropped */
}

/* java.util.Formatter %f: the digits of the shortest decimal that round-trips
 * (FloatingDecimal), rounded HALF_UP to 6 fraction digits, root locale. */
static int java_fixed6(double x, char* buf, int cap) {
    if (x != x) return snprintf(buf, cap, "NaN");
    if (isinf(x)) return snprintf(buf, cap, x > 0 ? "Infinity" : "-Infinity");
    char tmp[64];
    int prec;
    for (prec = 1; prec <= 17; ++prec) {
        snprintf(tmp, sizeof tmp, "%.*e", prec - 1, x);
        if (strtod(tmp, NULL) == x) break;
    }
    /* tmp = [-]d.ddddde[+-]XX */
    int neg = tmp[0] == '-';
    char* p = tmp + neg;
    char digits[32];
    int nd = 0;
    for (; *p && *p != 'e'; ++p)
        if (*p >= '0' && *p <= '9') digits[nd++] = *p;
    int exp10 = atoi(p + 1);          /* value = d1.d2d3... x 10^exp10 */
    /* fixed representation: integer part digits = exp10+1 */
    char fixed[400];
    int fl = 0, point;
    if (exp10 >= 0) {
        for (int k = 0; k <= exp10; ++k) fixed[fl++] = k < nd ? digits[k] : '0';
        point = fl;
        for (int k = exp10 + 1; k < nd; ++k) fixed[fl++] = digits[k];
    } else {
        fixed[fl++] = '0';
        point = fl;
        for (int k = 0; k < -exp10 - 1; ++k) fixed[fl++] = '0';
        for (int k = 0; k < nd; ++k) fixed[fl++] = digits[k];
    }
    while (fl < point + 7) fixed[fl++] = '0';
    /* HALF_UP at 6 fraction digits */
    int keep = point + 6;
    int up = fixed[keep] >= '5';
    fl = keep;
    if (up) {
        int k = keep - 1;
        for (; k >= 0; --k) {
            if (fixed[k] == '9') fixed[k] = '0';
            else { fixed[k]++; break; }
        }
        if (k < 0) { memmove(fixed + 1, fixed, (size_t)fl); fixed[0] = '1'; fl++; point++; }
    }
    int w = 0;
    if (neg && w < cap) buf[w++] = '-';
    for (int k = 0; k < fl && w < cap - 1; ++k) {
        if (k == point) buf[w++] = '.';
        buf[w++] = fixed[k];
    }
    buf[w] = 0;
    return w;
}

int orc_format_island(const cpg_island* r, char* buf, int cap) {
    char a[400], b[400];
    java_fixed6(r->cg, a, sizeof a);
    java_fixed6(r->oe, b, sizeof b);
    return snprintf(buf, cap, "%d %d %d %s %s\n", r->beg1, r->end1, r->len, a, b);
}
