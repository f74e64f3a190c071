/*
 * sbz_oracle.c — CPU restatement (plain C) of the sBayes likelihood.
 *
 * TEST INFRASTRUCTURE ONLY.  Built into oracle/liboracle.so and used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.  The
 * product path (contact_zones_amd) never links or calls it.
 *
 * Restates, per (site, feature) cell and in the reference's operation order:
 *   lh_c        one-hot gathers            sbayes/model.py:324-328, 387-390, 427-431
 *   NA -> 1     all components             sbayes/model.py:247
 *   w_norm      w[f,c]*has[s,c] / ((w0*h0 + w1*h1) + w2*h2)   sbayes/model.py:451-452
 *   mixture     log((w0*l0 + w1*l1) + w2*l2)                   sbayes/model.py:175-176
 *   source      log(w_src * l_src), -inf if any w_src == 0      sbayes/model.py:177-184
 * and reduces the N*F log values with numpy's pairwise summation
 * (numpy/_core/src/umath/loops_utils.h.src, PW_BLOCKSIZE 128, 8 accumulators)
 * so that the final sum follows np.sum's association order.
 *
 * Compile with -ffp-contract=off: numpy never fuses multiply-adds.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#define SBZ_NONE 255

static double pairwise_sum(const double *a, long n)
{
    if (n < 8) {
        double res = -0.0;
        for (long i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
    }
}

/* Per-cell log values into vals[N*F]; returns 1 if a selected source weight is 0. */
static int cell_logs(int N, int F, int S, int inheritance,
                     const int8_t *obs, const uint8_t *fam_of_site, const uint8_t *zone_of_site,
                     const double *w, const double *pg, const double *pz, const double *pf,
                     const uint8_t *source, double *vals)
{
    const int C = inheritance ? 3 : 2;
    int zero_weight = 0;
    for (int s = 0; s < N; s++) {
        const int z = zone_of_site[s];
        const int fam = fam_of_site[s];
        const double hz = (z != SBZ_NONE) ? 1.0 : 0.0;
        const double hf = (inheritance && fam != SBZ_NONE) ? 1.0 : 0.0;
        for (int f = 0; f < F; f++) {
            const int x = obs[(long)s * F + f];
            const int na = x < 0;
            double l[3], wc[3], nw[3];
            l[0] = na ? 1.0 : pg[(long)f * S + x];
            l[1] = na ? 1.0 : (hz != 0.0 ? pz[((long)z * F + f) * S + x] : 0.0);
            l[2] = 0.0;
            if (inheritance)
                l[2] = na ? 1.0 : (hf != 0.0 ? pf[((long)fam * F + f) * S + x] : 0.0);
            wc[0] = w[(long)f * C + 0] * 1.0;
            wc[1] = w[(long)f * C + 1] * hz;
            double sum = wc[0] + wc[1];
            if (inheritance) {
                wc[2] = w[(long)f * C + 2] * hf;
                sum = sum + wc[2];
            }
            for (int c = 0; c < C; c++) nw[c] = wc[c] / sum;
            double v;
            if (source == NULL) {
                double cell = nw[0] * l[0] + nw[1] * l[1];
                if (inheritance) cell = cell + nw[2] * l[2];
                v = log(cell);
            } else {
                const int c = source[(long)s * F + f];
                if (nw[c] == 0.0) zero_weight = 1;
                v = log(nw[c] * l[c]);
            }
            vals[(long)s * F + f] = v;
        }
    }
    return zero_weight;
}

/* Log-likelihood of one chain.  source == NULL selects the mixture branch. */
double oracle_loglik(int N, int F, int S, int Z, int Fam, int inheritance,
                     const int8_t *obs, const uint8_t *fam_of_site, const uint8_t *zone_of_site,
                     const double *w, const double *pg, const double *pz, const double *pf,
                     const uint8_t *source)
{
    (void)Z; (void)Fam;
    double *vals = (double *)malloc(sizeof(double) * (size_t)N * (size_t)F);
    if (!vals) return NAN;
    int zero_weight = cell_logs(N, F, S, inheritance, obs, fam_of_site, zone_of_site,
                                w, pg, pz, pf, source, vals);
    /* np.sum(..) over a contiguous array: identity 0.0 plus the pairwise sum */
    double r = 0.0 + pairwise_sum(vals, (long)N * F);
    free(vals);
    if (source != NULL && zero_weight) return -INFINITY;
    return r;
}

/* B chains; per-chain arrays stacked contiguously (layouts as in include/sbz.h). */
void oracle_loglik_batch(int B, int N, int F, int S, int Z, int Fam, int inheritance,
                         const int8_t *obs, const uint8_t *fam_of_site,
                         const uint8_t *zone_of_site, const double *w, const double *pg,
                         const double *pz, const double *pf, const uint8_t *source,
                         double *out)
{
    const int C = inheritance ? 3 : 2;
    for (int b = 0; b < B; b++) {
        out[b] = oracle_loglik(
            N, F, S, Z, Fam, inheritance, obs, fam_of_site, zone_of_site + (long)b * N,
            w + (long)b * F * C, pg + (long)b * F * S, pz + (long)b * Z * F * S,
            pf ? pf + (long)b * Fam * F * S : NULL,
            source ? source + (long)b * N * F : NULL);
    }
}
