// CPU simulation of the walk's block resolve (design tool, not product code).
//
// The walk of k_emu_walk (csrc/lgcn_exact.hip) re-runs every block whose chain value cannot be
// translated as the reference's 256-step fma chain. This program measures, on real hub rows of
// the C3 graph (tools/sim/gen_hub.py), how a parallel resolve would do instead:
//   * guess the binade of every step's exact sum z_j = a_{j-1} + p_j from a double prefix sum;
//   * step increments q_j = RN_{ulp(b_j)}(p_j) (one fma with C = 1.5 * 2^b_j), as integers in
//     units of the window's finest ulp, and one prefix scan;
//   * an exact check per step (a_{j-1} a multiple of ulp(b_j), the result inside binade b_j
//     with a one-ulp margin, no possible tie, |p_j| small against 2^b_j); the first failing
//     step is taken by the reference's fma and the rest of the block shifted by the change.
// Every block's end value (and every intermediate value) is compared bitwise with the
// sequential chain. Prints the distribution of fix steps per resolved block.
//
//   gcc -O2 -o /tmp/resolve_sim tools/sim/resolve_sim.c -lm && /tmp/resolve_sim /tmp/hub/row0_l1.bin
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define B 256

static int binade(float f) {  // floor(log2|f|) for normal f; -1000 for 0/subnormal
    uint32_t u;
    memcpy(&u, &f, 4);
    int E = (u >> 23) & 255;
    if (E == 0) return -1000;
    return E - 127;
}
static int lsb_exp(float f) {
    uint32_t b;
    memcpy(&b, &f, 4);
    int E = (b >> 23) & 255;
    uint32_t M = b & 0x7fffff;
    if (E == 0) return -149 + __builtin_ctz(M);
    return E - 150 + __builtin_ctz(M | 0x800000);
}
static int lsb_prod(float v, float x) { return (v != 0 && x != 0) ? lsb_exp(v) + lsb_exp(x) : -100000; }

typedef struct {
    long blocks, failed, fixes, setups, hist[64], wins, zero_or_span, exceed;
    long fix_div, fix_bin, fix_tie, fix_big, sub64, sub32, sub16, ucross;
} Stats;

// resolve block: v, x (n steps), start value a (exact). Returns end value; traj gets every value.
static float resolve(const float* v, const float* x, int n, float a, float* traj, Stats* st,
                     int* nfix_out) {
    int j0 = 0, nfix = 0;
    while (j0 < n) {
        st->setups++;
        // guesses from the double prefix (exact products, accurate sums)
        int bj[B];
        double S = a;
        int emin = binade(a) > -1000 ? binade(a) : 1000, emax = binade(a) > -1000 ? binade(a) : -1000;
        int jw = n;
        for (int j = j0; j < n; ++j) {
            S += (double)v[j] * (double)x[j];
            int e;
            if (S == 0.0) { jw = j; break; }
            frexp(S, &e);
            bj[j] = e - 1;
            int lo = emin < bj[j] ? emin : bj[j], hi = emax > bj[j] ? emax : bj[j];
            if (hi - lo > 6 || bj[j] < -126) { jw = j; break; }
            emin = lo, emax = hi;
        }
        if (jw == j0) {  // no window: one sequential step
            st->zero_or_span++;
            a = fmaf(v[j0], x[j0], a);
            traj[j0] = a;
            ++j0;
            ++nfix;
            continue;
        }
        st->wins++;
        // increments in units U = 2^(emin - 23)
        int64_t inc[B], A[B + 1];
        int bad[B];
        for (int j = j0; j < jw; ++j) {
            const int b = bj[j];
            // RN_G(p), G = ulp(b): TwoProduct hi + lo = p exactly; a large product is hi (a
            // multiple of G) plus RN_G(lo); a small one goes through C in binade b
            const float hi = v[j] * x[j];
            const float lo = fmaf(v[j], x[j], -hi);
            const float P2 = ldexpf(1.f, b);
            double qd;
            int big;
            if (fabsf(hi) >= P2) {
                const float C = ldexpf(1.5f, b);
                const float r = (lo + C) - C;
                big = !(fabsf(lo) < ldexpf(1.f, b - 1));
                qd = ldexp((double)hi, 23 - b) + ldexp((double)r, 23 - b);
            } else {
                const float G = ldexpf(1.f, b - 23);
                const float C = hi > 0 ? P2 : 2 * P2 - 2 * G;
                const float R = fmaf(v[j], x[j], C) - C;
                big = hi == 0.f || fabsf(hi) > P2 - 4 * G;
                qd = ldexp((double)R, 23 - b);
            }
            const int tie = lsb_prod(v[j], x[j]) == b - 24;
            bad[j] = big ? 1 : tie ? 2 : 0;
            inc[j] = big ? 0 : ((int64_t)qd << (b - emin));
        }
        // prefix (exclusive start A[j0] = a / U)
        int64_t Astart = (int64_t)ldexp((double)a, 23 - emin);
        int j = j0;
        int64_t cur = Astart, shift = 0;
        // the GPU version: one scan, then a loop over failing steps (check in parallel on the
        // shifted prefix). Here sequentially, counting the fix steps.
        for (j = j0; j < jw; ++j) {
            const int b = bj[j];
            const int64_t G = (int64_t)1 << (b - emin);
            const int64_t lo = ((int64_t)1 << (b - emin + 23)) + G;
            const int64_t hi = ((int64_t)1 << (b - emin + 24)) - G;
            int fail = bad[j];
            if (!fail && (cur % G) != 0) fail = 3;
            int64_t nx = cur + inc[j];
            int64_t m = nx < 0 ? -nx : nx;
            if (!fail && (m < lo || m > hi)) fail = 4;
            if (fail) {
                // the reference's fma
                nfix++;
                if (fail == 1) st->fix_big++;
                else if (fail == 2) st->fix_tie++;
                else if (fail == 3) st->fix_div++;
                else st->fix_bin++;
                float ap = (float)ldexp((double)cur, emin - 23);
                float an = fmaf(v[j], x[j], ap);
                int be = binade(an);
                if (an != 0.f && (be < emin || be > emax + 1)) {  // left the window's units
                    traj[j] = an;
                    a = an;
                    ++j;
                    goto next_round;
                }
                nx = (int64_t)ldexp((double)an, 23 - emin);
                if ((double)nx != ldexp((double)an, 23 - emin)) {
                    traj[j] = an;
                    a = an;
                    ++j;
                    goto next_round;
                }
            }
            cur = nx;
            traj[j] = (float)ldexp((double)cur, emin - 23);
        }
        a = (float)ldexp((double)cur, emin - 23);
    next_round:
        j0 = j;
        (void)shift;
    }
    *nfix_out = nfix;
    return a;
}


static int bexp_of(float f) { uint32_t u; memcpy(&u, &f, 4); return (u >> 23) & 255; }
static uint32_t bits_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

typedef struct { long ok, rounds, seq_steps, end_span, end_multi, end_big, end_tie, end_res, end_verify, ucs, hist[8]; } V3;

// one parallel round over steps [j0, n) from the exact value a (the value before step j0):
// returns the first step not proven (n: all done); traj[j0 .. ret) are exact
static int round_v4(const float* v, const float* x, int n, int j0, float a, float* traj, V3* st) {
    int be[B], uc[B];
    int32_t inc[B], dodd[B];
    float hi[B];
    const int ba = bexp_of(a);
    if (a != 0.f && ba == 0) return j0;
    float P = 0.f;
    for (int j = j0; j < n; ++j) {
        hi[j] = v[j] * x[j];
        P += hi[j];
        be[j] = bexp_of(a + P);
    }
    // window: cumulative binade span <= 6, normal, finite
    int emin = a != 0.f ? ba : 1000, emax = a != 0.f ? ba : -1000;
    int w = n;
    for (int j = j0; j < n; ++j) {
        const int lo = emin < be[j] ? emin : be[j], hi_ = emax > be[j] ? emax : be[j];
        if (lo < 1 || hi_ - lo > 6 || hi_ > 253) { w = j; st->end_span++; break; }
        emin = lo, emax = hi_;
    }
    if (w == j0) return j0;
    const int eu = emin;
    // up-crossings: one level, one binade up; the first other one ends the window
    int level = -1;
    for (int j = j0; j < w; ++j) {
        const int ep = j > j0 ? be[j - 1] : (a != 0.f ? ba : 0);
        uc[j] = ep > 0 && be[j] > ep;
        if (uc[j]) {
            if (be[j] != ep + 1 || (level >= 0 && level != be[j])) { w = j; st->end_multi++; break; }
            level = be[j];
            st->ucs++;
        }
    }
    for (int j = j0; j < w; ++j) {
        const int b = be[j];
        const float lo = fmaf(v[j], x[j], -hi[j]);
        if (lo == 0.f && hi[j] != 0.f) { w = j; st->end_tie++; break; }
        const uint32_t hb = bits_of(hi[j]);
        if (((hb >> 23) & 255) >= (uint32_t)b) {
            // |hi| >= 2^b: hi is a multiple of G; RN_G(p) = hi + RN_G(lo)
            const int eh = (hb >> 23) & 255;
            if (eh > b + 6) { w = j; st->end_big++; break; }
            const int32_t mh = (int32_t)(((hb & 0x7fffffu) | 0x800000u) << (eh - b));
            const uint32_t cl = (bits_of(lo) & 0x80000000u) ? ((((uint32_t)b + 1) << 23) - 2u) : ((uint32_t)b << 23);
            const float Fl = from_bits(cl) + lo;
            if ((bits_of(Fl) >> 23) != (uint32_t)b) { w = j; st->end_big++; break; }
            const int32_t ql = (int32_t)(bits_of(Fl) - cl);
            inc[j] = ((hb >> 31) ? -mh : mh) + ql;
            inc[j] <<= (b - eu);
        } else {
            // |p| < 2^b: C in binade b on the side that keeps C + p inside it
            const uint32_t cb = (hb >> 31) ? ((((uint32_t)b + 1) << 23) - 2u) : ((uint32_t)b << 23);
            const float F = fmaf(v[j], x[j], from_bits(cb));
            if ((bits_of(F) >> 23) != (uint32_t)b) { w = j; st->end_big++; break; }
            inc[j] = (int32_t)(bits_of(F) - cb) << (b - eu);
        }
        dodd[j] = 0;
        if (uc[j]) {
            const uint32_t sgn = bits_of(hi[j]) & 0x80000000u;
            const uint32_t cob = (((uint32_t)b << 23) - 1u) | sgn;
            const float Fo = fmaf(v[j], x[j], from_bits(cob));
            if ((bits_of(Fo) >> 23) != (cob >> 23)) { w = j; st->end_big++; break; }
            const int32_t t = (int32_t)((bits_of(Fo) & 0x7fffffffu) - ((uint32_t)b << 23));
            dodd[j] = ((sgn ? -(2 * t + 1) : (2 * t + 1)) << (b - 1 - eu)) - inc[j];
        }
    }
    const int32_t A0 = a == 0.f ? 0
        : (int32_t)(((bits_of(a) & 0x7fffffu) | 0x800000u) << (ba - eu)) * ((bits_of(a) >> 31) ? -1 : 1);
    int32_t prev[B], cs[B];
    int odd[B];
    int32_t s_ = A0;
    for (int j = j0; j < w; ++j) { prev[j] = s_; s_ += inc[j]; cs[j] = s_; }
    int xlast = 0;
    int32_t C = 0;
    for (int j = j0; j < w; ++j) {
        odd[j] = 0;
        if (uc[j]) {
            const int b = be[j];
            const int32_t Gm = (1 << (b - eu)) - 1, half = 1 << (b - 1 - eu);
            const int32_t r = prev[j] & Gm;
            if (r != 0 && r != half) { w = j; st->end_res++; break; }
            odd[j] = (r == half) ^ xlast;
            xlast = r == half;
        }
        prev[j] += C;
        if (odd[j]) C += dodd[j];
        cs[j] += C;
    }
    for (int j = j0; j < w; ++j) {
        const int b = be[j];
        const int32_t Gm = (1 << (b - eu)) - 1;
        const int32_t want = odd[j] ? (1 << (b - 1 - eu)) : 0;
        const uint32_t m = cs[j] < 0 ? (uint32_t)-cs[j] : (uint32_t)cs[j];
        const int msb = m ? 31 - __builtin_clz(m) : -1;
        if ((prev[j] & Gm) != want || msb != b - eu + 23 || m == (1u << (b - eu + 23))) {
            st->end_verify++;
            w = j;
            break;
        }
        traj[j] = (float)ldexp((double)cs[j], eu - 150);
    }
    return w;
}

static float resolve_v3(const float* v, const float* x, int n, float a, float* traj, V3* st) {
    int j0 = 0, rounds = 0;
    while (j0 < n) {
        ++rounds;
        const int w = round_v4(v, x, n, j0, a, traj, st);
        if (w > j0) a = traj[w - 1];
        if (w >= n) break;
        // step w by the reference's fma, then a new round
        traj[w] = a = fmaf(v[w], x[w], a);
        st->seq_steps++;
        j0 = w + 1;
    }
    st->rounds += rounds;
    st->hist[rounds < 7 ? rounds : 7]++;
    if (rounds == 1) st->ok++;
    return a;
}

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    FILE* f = fopen(argv[1], "rb");
    int hdr[2];
    if (fread(hdr, 4, 2, f) != 2) return 1;
    const int n = hdr[0], d = hdr[1];
    float* v = malloc(sizeof(float) * n);
    float* X = malloc(sizeof(float) * (size_t)n * d);
    if (fread(v, 4, n, f) != (size_t)n || fread(X, 4, (size_t)n * d, f) != (size_t)n * d) return 1;
    fclose(f);
    const int ncols = argc > 2 ? atoi(argv[2]) : d;
    float* xc = malloc(sizeof(float) * n);
    float* tr = malloc(sizeof(float) * n);
    float* tr2 = malloc(sizeof(float) * B);
    Stats st;
    memset(&st, 0, sizeof st);
    long mism = 0, mism3 = 0;
    V3 s3;
    memset(&s3, 0, sizeof s3);
    for (int c = 0; c < ncols; ++c) {
        for (int j = 0; j < n; ++j) xc[j] = X[(size_t)j * d + c];
        float a = 0.f;
        for (int j = 0; j < n; ++j) tr[j] = a = fmaf(v[j], xc[j], a);
        // blocks
        float start = 0.f;
        for (int b0 = 0; b0 < n; b0 += B) {
            const int nb = n - b0 < B ? n - b0 : B;
            st.blocks++;
            // translatable: trajectory stays in the start binade with a 132-ulp slack
            const int e = binade(start);
            int ok = e > -1000;
            if (ok) {
                const double u = ldexp(1.0, e - 23);
                const double lo = ldexp(1.0, e) + 132 * u, hi = ldexp(1.0, e + 1) - 132 * u;
                for (int j = b0; j < b0 + nb && ok; ++j) {
                    const double m = fabs((double)tr[j]);
                    ok = m >= lo && m <= hi;
                }
                const double m0 = fabs((double)start);
                ok = ok && m0 >= lo && m0 <= hi;
            }
            if (!ok) {
                st.failed++;
                for (int sb = 16; sb <= 64; sb *= 2) {
                    for (int s0 = b0; s0 < b0 + nb; s0 += sb) {
                        const float s_start = s0 == 0 ? 0.f : tr[s0 - 1];
                        const int es = binade(s_start);
                        int sok = es > -1000;
                        if (sok) {
                            const double u = ldexp(1.0, es - 23);
                            const double lo = ldexp(1.0, es) + 4 * u, hi = ldexp(1.0, es + 1) - 4 * u;
                            for (int j = s0; j < s0 + sb && j < b0 + nb && sok; ++j) {
                                const double m = fabs((double)tr[j]);
                                sok = m >= lo && m <= hi;
                            }
                        }
                        if (!sok) { if (sb == 64) st.sub64++; else if (sb == 32) st.sub32++; else st.sub16++; }
                    }
                }
                {
                    float pv = start;
                    for (int j = b0; j < b0 + nb; ++j) {
                        if (binade(tr[j]) > binade(pv)) st.ucross++;
                        pv = tr[j];
                    }
                }
                int nfix = 0;
                float endv = resolve(v + b0, xc + b0, nb, start, tr2, &st, &nfix);
                st.fixes += nfix;
                st.hist[nfix < 63 ? nfix : 63]++;
                for (int j = 0; j < nb; ++j)
                    if (memcmp(&tr2[j], &tr[b0 + j], 4)) { mism++; break; }
                if (memcmp(&endv, &tr[b0 + nb - 1], 4)) mism++;
                {
                    float e3 = resolve_v3(v + b0, xc + b0, nb, start, tr2, &s3);
                    for (int j = 0; j < nb; ++j)
                        if (memcmp(&tr2[j], &tr[b0 + j], 4)) {
                            if (mism3 < 3) fprintf(stderr, "mismatch block at %d step %d: got %a want %a (prev %a)\n", b0, j, tr2[j], tr[b0+j], j ? tr[b0+j-1] : start);
                            mism3++; break; }
                    if (memcmp(&e3, &tr[b0 + nb - 1], 4)) mism3++;
                }
            }
            start = tr[b0 + nb - 1];
        }
    }
    printf("%s: n=%d cols=%d blocks=%ld failed=%ld (%.1f%%) mismatches=%ld\n", argv[1], n, ncols,
           st.blocks, st.failed, 100.0 * st.failed / st.blocks, mism);
    printf("  per failed block: setups %.2f, fix steps %.2f (div %.2f bin %.2f tie %.3f big %.3f), "
           "no-window steps %.2f\n",
           (double)st.setups / st.failed, (double)st.fixes / st.failed,
           (double)st.fix_div / st.failed, (double)st.fix_bin / st.failed,
           (double)st.fix_tie / st.failed, (double)st.fix_big / st.failed,
           (double)st.zero_or_span / st.failed);
    printf("  failing sub-blocks per failed block: of 64 %.2f/4, of 32 %.2f/8, of 16 %.2f/16; up-crossings %.2f\n",
           (double)st.sub64 / st.failed, (double)st.sub32 / st.failed, (double)st.sub16 / st.failed,
           (double)st.ucross / st.failed);
    printf("  v4: mismatches %ld, one round %.1f%%, rounds/failed block %.2f, seq steps %.2f; window ends per failed block: span %.2f multi %.2f big %.3f tie %.3f res %.3f verify %.3f; ucs %.2f; rounds hist",
           mism3, 100.0 * s3.ok / st.failed, (double)s3.rounds / st.failed, (double)s3.seq_steps / st.failed,
           (double)s3.end_span / st.failed, (double)s3.end_multi / st.failed, (double)s3.end_big / st.failed,
           (double)s3.end_tie / st.failed, (double)s3.end_res / st.failed, (double)s3.end_verify / st.failed,
           (double)s3.ucs / st.failed);
    for (int k = 1; k < 8; ++k) printf(" %d:%ld", k, s3.hist[k]);
    printf("\n");
    printf("  fix-step histogram:");
    for (int k = 0; k < 64; ++k)
        if (st.hist[k]) printf(" %d:%ld", k, st.hist[k]);
    printf("\n");
    return 0;
}
