// sbz_mh_src.hip — the MH sampler with SAMPLE_SOURCE = true on CDNA4 (gfx950).
//
// MCMCGenerative.step (sbayes/sampling/mcmc_generative.py:282-351) with the operators the
// reference uses when every observation carries its mixture component ("source",
// mcmc_setup.py:80-87, zone_sampling.py:180-406):
//   shrink_zone / grow_zone / swap_zone with source resampling (:704-933; warm-up :1328-1574):
//       log q_back += sum log posterior[current source] (current sample), then every source is
//       redrawn from the new sample's posterior and log q += sum log posterior[new source]
//       (gibbs_sample_sources(as_gibbs=False), :180-220).  ZoneMCMCWarmup passes as_gibbs=True
//       whatever it is given (:1293-1296), so its zone moves carry log q = -inf: accepted.
//   gibbs_sample_sources   (:180-215)  every source redrawn (sample_categorical,
//                                      preprocessing.py:321-348)
//   gibbs_sample_weights   (:222-331)  Dirichlet(1 + source counts) per feature; with inheritance
//                                      a Beta draw for one weight ratio (the per-feature accept
//                                      draw is made and overridden, :325-327: always the new ones)
//   gibbs_sample_p_global  (:334-357)  40 % of the features, Dirichlet(prior counts + counts)
//   gibbs_sample_p_zones   (:359-379)  one zone, every feature, Dirichlet(1 + counts)
//   gibbs_sample_p_families(:381-406)  one family, 40 % of the features
//   gibbsish_sample_zones  (:619-702)  one zone's available sites resampled in / out from their
//                                      marginal likelihoods, then their sources redrawn
//                                      (site_subset = available); weight 0 in the reference's own
//                                      operator table (mcmc_setup.py:77)
// The Gibbs operators return Q_GIBBS (log q = -inf): always accepted.
//
// One workgroup of NW waves (8 by default) runs one chain.  The chain's sources (N x F bytes,
// current and candidate), zone assignment and counters live in LDS for the whole launch where they
// fit, in HBM by position with per-chain count tables otherwise (the table-pass kernel, cfg5);
// every operator is a few lane-parallel passes over the N*F observations (per observation: the normalised weights and
// component likelihoods in the reference's operation order, the posterior, the categorical draw,
// the source-branch log-likelihood log(w_src * lh_src), model.py:177-184).  Draws come from the
// replay tape (the reference's own decisions) or from Philox: uniform decisions from the wave's
// stream, per-observation / per-feature draws from per-lane streams.
#include <cmath>
#include <cstdint>
#include <type_traits>

#include "sbz_mh_common.h"

namespace sbz {


namespace {

// The component likelihoods and normalised weights of observation (s, f) (update_component_
// likelihoods model.py:230-249 with NA -> 1 for every component; normalize_weights :436-452).
template <int C>
__device__ __forceinline__ void obs_terms(const MhArgs &a, const double *w, const double *pg,
                                          const double *pz, const double *pf, int f, int x, int zc,
                                          int fc, double (&l)[3], double (&wn)[3]) {
    const int S = a.S, F = a.F, Z = a.Z;
    const bool na = x >= S;
    const int xc = na ? 0 : x;
    const bool hz = zc < Z;
    const bool hf = (C == 3) && fc > 0;
    const double w0 = ldp(w + (size_t)f * C) * 1.0;
    const double w1 = ldp(w + (size_t)f * C + 1) * (hz ? 1.0 : 0.0);
    double sum = w0 + w1, w2 = 0.0;
    if (C == 3) {
        w2 = ldp(w + (size_t)f * C + 2) * (hf ? 1.0 : 0.0);
        sum = sum + w2;
    }
    wn[0] = w0 / sum;
    wn[1] = w1 / sum;
    wn[2] = C == 3 ? w2 / sum : 0.0;
    l[0] = na ? 1.0 : ldp(pg + (size_t)f * S + xc);
    l[1] = na ? 1.0 : (hz ? ldp(pz + ((size_t)zc * F + f) * S + xc) : 0.0);
    l[2] = (C == 3) ? (na ? 1.0 : (hf ? ldp(pf + ((size_t)(fc - 1) * F + f) * S + xc) : 0.0)) : 0.0;
}

// normalize(lh * w) (zone_sampling.py:202), then sample_categorical: argmax(u < cumsum(p)), 0 if
// no entry exceeds u (preprocessing.py:335-338).  Returns the component; p[] the posterior.
template <int C>
__device__ __forceinline__ int posterior_draw(const double (&l)[3], const double (&wn)[3], double u,
                                              double (&p)[3]) {
    const double x0 = l[0] * wn[0], x1 = l[1] * wn[1], x2 = C == 3 ? l[2] * wn[2] : 0.0;
    double sum = x0 + x1;
    if (C == 3) sum = sum + x2;
    p[0] = x0 / sum;
    p[1] = x1 / sum;
    p[2] = C == 3 ? x2 / sum : 0.0;
    const double c0 = p[0], c1 = c0 + p[1], c2 = c1 + p[2];
    return u < c0 ? 0 : (u < c1 ? 1 : ((C == 3 && u < c2) ? 2 : 0));
}

}  // namespace

// ---- Feature-table passes (the sources in HBM, TB).  One pass over the N * F observations: each
// wave takes whole features (f = wave, wave + NW, ...), with a table, a parameter column and a
// count block of its own in LDS, and no block barrier until the pass ends.  Per feature the wave
// loads the parameter column, normalises the weights (normalize_weights, model.py:436-452) and
// builds the table of the three component terms t_k = l_k * w_norm_k of every (zone class, family
// class, state) cell kind (obs_terms' operations: the source branch's factors, model.py:177-184,
// and the unnormalised posterior of gibbs_sample_sources, zone_sampling.py:200-202); then each
// lane takes 32 positions of the feature (8 dwords of observation / source bytes, coalesced), and
// a cell costs one table read, a compare chain and one product.  A resample draw with Philox
// uniforms compares u * s against the partial sums of the terms (s = their sum: the categorical
// distribution of the reference's u < cumsum(t / s), sample_categorical preprocessing.py:335-338,
// without its divisions); a tape replay takes the reference's own quotients and partial sums per
// cell, so its draws are the reference's bit for bit.  A source byte is always written and read
// back by the same thread.  The pass also counts the new sources per (component row, state) and
// per (class, component) into the chain's count table in HBM, from which the Gibbs parameter
// operators take their Dirichlet counts and their log-likelihood change without a pass of their
// own.  Each wave loads the next feature's column and observation (source) words while it works on
// the current one.
constexpr int TB_NCH = 8;  // 256-position chunks per feature: the passes take Np <= 2048
struct TbDims {
    int E;     // table entries per feature: (Z + 1) zone classes x FamC family classes x (S + 1) states
    int FamC;  // family classes (Fam + 1 with inheritance, else 1)
    int NL;    // column values loaded per feature: the C raw weights, then p_global, p_zones, p_families
    int NCOL;  // doubles per column: w_norm [4][3], raw weights [3], the parameters
    int CTP;   // counters per feature: p_global [S], p_zones [Z][S], p_families [Fam][S], classes [4][3]
    int WOFF;  // offset of the class counters [h][k] (h = has_zone | has_family << 1)
};
__host__ __device__ inline TbDims tb_dims(int S, int Z, int Fam, int C) {
    TbDims t;
    const int Fm = C == 3 ? Fam : 0;
    t.FamC = Fm + 1;
    t.E = (Z + 1) * t.FamC * (S + 1);
    t.NL = C + S * (1 + Z + Fm);
    t.NCOL = 15 + S * (1 + Z + Fm);
    t.WOFF = S * (1 + Z + Fm);
    t.CTP = t.WOFF + 12;
    return t;
}
// LDS of the pass (from the pass region's 16-B aligned base): per wave a table [E + 1][3] doubles
// (entry E: the padding positions' neutral entry), a column [NCOL] doubles and a count block
// [CTP] ints (`wave` bytes apart), then the per-position class words [Np] and the table entries'
// (state, zone class, family class) [E]
struct TbLayout {
    size_t wave, col, kcnt, pinfo, ed, end;
};
__host__ __device__ inline TbLayout tb_layout(const TbDims &t, int Np, int nw) {
    TbLayout L;
    L.col = ((size_t)(t.E + 1) * 24 + 15) & ~(size_t)15;
    L.kcnt = L.col + (((size_t)t.NCOL * 8 + 15) & ~(size_t)15);
    L.wave = L.kcnt + (((size_t)t.CTP * 4 + 15) & ~(size_t)15);
    L.pinfo = (size_t)nw * L.wave;
    L.ed = L.pinfo + (size_t)Np * 4;
    L.end = L.ed + (((size_t)t.E * 4 + 15) & ~(size_t)15);
    return L;
}
// the table passes apply: at most 8 chunks of 256 positions, three column values and three counters
// per lane
__host__ __device__ inline bool tb_fits(const TbDims &t, int Np) {
    return Np <= 256 * TB_NCH && t.NL <= 3 * 64 && t.CTP <= 3 * 64 && t.E <= 65535 - 256;
}

// LDS bytes of the redraw scratch (redraw_rows / weight gammas: draws [F][max(S, 2)] doubles,
// per-feature tape offsets and counter ranks [F] ints, two totals)
__host__ __device__ inline size_t redraw_bytes(size_t F, size_t S) { return F * (S > 2 ? S : 2) * 8 + 2 * F * 4 + 8; }

size_t mh_src_lds_bytes(const sbz_dims &d, int C, bool hbm_sources, bool geo, bool stage, bool tb, int Np, int nw) {
    const size_t N = d.n_sites, F = d.n_features, S = d.n_states, Z = d.n_zones;
    const size_t cnt = F * (S > (size_t)C ? S : (size_t)C);
    const size_t head = MH_SRC_MAX_WAVES * 2 * (8 + 4) + cnt * 4 + ((Z + 1) & ~(size_t)1) * 4 + MH_STAT_INTS * 4 +
                        ((N + 1) & ~(size_t)1) * 2 +
                        (hbm_sources ? 0 : ((N * F + 15) & ~(size_t)15) * 2) + ((N + 15) & ~(size_t)15) +
                        ((F + 15) & ~(size_t)15) + (geo ? 16 + geo_scratch_bytes((int)N) : 0);
    if (tb) {
        // the operator CDF, then one region that holds the redraw scratch or the pass buffers
        const TbDims t = tb_dims((int)S, (int)Z, d.n_families, C);
        const size_t pass = tb_layout(t, Np, nw).end, rd = redraw_bytes(F, S);
        return head + 16 + SBZ_N_OPS * 8 + 16 + (pass > rd ? pass : rd);
    }
    return head + 16 + redraw_bytes(F, S) + 8 + SBZ_N_OPS * 8 +
           // staged parameters: normalised weights [F][4][3], p_global, p_zones, p_families
           (stage ? 16 + (12 * F + (1 + Z + (C == 3 ? (size_t)d.n_families : 0)) * F * S) * 8 + N * F + N : 0);
}

// LDS bytes of the staged constant tables (a.cstage): 'counts' prior and Gibbs prior counts of
// p_global / p_families where set, applicable states [F][S] and their counts [F] as bytes
size_t mh_src_const_bytes(const sbz_dims &d, int C, bool alg, bool alf, bool gcg, bool gcf) {
    const size_t FS = (size_t)d.n_features * d.n_states, Fam = C == 3 ? (size_t)d.n_families : 0;
    return 16 + 8 * FS * ((alg ? 1 : 0) + (gcg ? 1 : 0) + Fam * ((alf ? 1 : 0) + (gcf ? 1 : 0))) + FS +
           (size_t)d.n_features + 16;
}

// table passes: timing ablations of diagnostic builds (bit 1 no count atomics, 4 no table build, 8 a
// constant uniform, 16 no log-likelihood product; results invalid)
#ifndef SBZ_TB_ABL
#define SBZ_TB_ABL 0
#endif
// table passes: stage cycle stamps of diagnostic builds (SBZ_TB_STAMP=1): per chain, the shader
// cycles of each pipeline stage summed over the launch replace the first 16 entries of the ll trace
// (wave 0: 0..7, the last wave: 8..15; results invalid)
#ifndef SBZ_TB_STAMP
#define SBZ_TB_STAMP 0
#endif
// A/B knobs: the log-likelihood pass reads only the selected component's weight and likelihood
// (SBZ_SRC_LL1), and the N * F passes are unrolled SBZ_SRC_UNR cells deep
#ifndef SBZ_SRC_LL1
#define SBZ_SRC_LL1 1
#endif
#ifndef SBZ_SRC_UNR
#define SBZ_SRC_UNR 1
#endif
// Philox Gibbs draws in flight per thread (gamma_fill slots): p_* redraws, weights
#ifndef SBZ_RB_REDRAW
#define SBZ_RB_REDRAW 4
#endif
#ifndef SBZ_RB_WEIGHTS
#define SBZ_RB_WEIGHTS 2
#endif

namespace {

// (p, f) of position-major cell i = f * Np + p, advanced by NT cells per step
struct PosWalk {
    int p, f, dP, dF, Np;
    __device__ __forceinline__ void next() {
        p += dP;
        f += dF;
        if (p >= Np) {
            p -= Np;
            f++;
        }
    }
};

// (s, f) of cell c = s * F + f, advanced by NT cells per step
struct CellWalk {
    int s, f, dS, dF, F;
    __device__ __forceinline__ void next() {
        f += dF;
        s += dS;
        if (f >= F) {
            f -= F;
            s++;
        }
    }
};

// ---- The feature-table pass (TbDims), a function of its own: its phase loop gets its own register
// allocation instead of sharing the sampler kernel's (inlined, its in-flight loads met spill
// reloads and waits).  LDS arrays come in as local-address-space pointers (cast back to generic
// ones inside, where the compiler infers ds_* accesses from the casts).
// (global arrays likewise come in as global-address-space pointers: a generic one would make its
// loads flat loads, which a barrier's lgkmcnt wait waits for)
template <class T>
using lds_ptr = __attribute__((address_space(3))) T *;
template <class T>
using gbl_ptr = __attribute__((address_space(1))) T *;
struct TbPassArgs {
    int N, F, S, Z, Np, xs8;
    TbDims td;
    gbl_ptr<const int> perm;
    gbl_ptr<const uint8_t> famc, obs_fm;
    lds_ptr<uint8_t> zos;
    lds_ptr<unsigned char> base;  // the pass region (tb_layout)
    lds_ptr<double> red;
    lds_ptr<int> redi;
    gbl_ptr<const double> w, pg, pz, pf;  // the chain's parameters
    gbl_ptr<const uint8_t> sv;
    gbl_ptr<uint8_t> dst;
    gbl_ptr<int> ct;
    gbl_ptr<const double> tape;
    int64_t pos0, len;
    uint32_t key0, key1;
    uint64_t chain, ctr;
    uint64_t *stamps;  // SBZ_TB_STAMP builds
};
struct TbPassOut {
    double ll;
    int err, bad;
    long long err_val;
};
// the per-cell uniforms of a Philox resample pass: xoroshiro128+ seeded per thread and pass from
// one Philox block keyed (seed; thread, counter, chain, 0xFD tag) — a stream no LaneRng / site
// stream shares; each 64-bit output gives two cells their uniforms, its high and its low 32 bits
// (w 2^-32: a 3-way categorical draw needs no finer grid)
struct Xoro {
    uint64_t s0, s1;
    __device__ __forceinline__ uint64_t next() {
        const uint64_t r = s0 + s1;
        const uint64_t t = s1 ^ s0;
        s0 = ((s0 << 24) | (s0 >> 40)) ^ t ^ (t << 16);
        s1 = (t << 37) | (t >> 27);
        return r;
    }
};
__device__ __forceinline__ double u32u(uint32_t w) { return (double)w * 0x1p-32; }
// per-thread sum of logs as one log: mantissas multiplied, exponents added (exact for any factor)
struct TbLogAcc {
    double m = 1.0;
    int e = 0;
    __device__ __forceinline__ double value() const { return flog(m) + (double)e * LN2; }
};

// The Philox Gibbs gammas of a redraw, a function of its own so that its loops get their own
// registers (inlined, the sampler kernel's live state spilled around them).  buf[t] holds item t's
// alpha (< 0: no draw, 0 returned) on entry and its gamma on exit, t < n; thread tid takes the
// items t = tid + i NT.  Item t is the Philox stream (key; block j0 + b, counter word, chain, c3):
// mode 0 (p_* redraws): item (f, j) = (t / S, t % S), counter ctr0 + frank[f], c3 tag lane j, j0 0;
// mode 1 (weights): counter ctr0, tag 0xFFF, j0 = t << 8.
// - integer alpha = m <= GB_NMAX: -log(u_1 ... u_m), the u's four per block from block j0 (K items
//   at a time);
// - otherwise Marsaglia-Tsang (boosted by u^(1/alpha) below 1, block j0 + 255), round r of an item
//   on block j0 + 16 + r (a 53-bit and a 32-bit uniform for the Box-Muller normal, a 32-bit
//   acceptance uniform), at most 64 rounds (then d, as LaneRng::gamma).  Each thread keeps K items
//   in flight (their dependent f64 chains overlap) and refills a slot from its own queue as soon
//   as the slot's item accepts, so a wave runs about (its items / K) x 1.03 rounds plus the tail
//   of its slowest lane, not the slowest lane's rounds for every batch.
// A draw depends only on its item's stream: not on K, NT or the order the slots take the items.
template <int K, int NT>
__device__ __noinline__ void gamma_fill(lds_ptr<double> bufp, int n, int S, lds_ptr<const int> frankp, uint32_t key0,
                                        uint32_t key1, uint32_t chain, uint64_t ctr0, int mode) {
    double *buf = (double *)bufp;
    const int *frank = (const int *)frankp;
    const int tid = (int)threadIdx.x;
    auto stream = [&](int t, uint32_t &j0, uint32_t &bs, uint32_t &c3) {
        if (mode == 0) {
            const int f = t / S, j = t - f * S;
            const uint64_t cr = ctr0 + (uint64_t)frank[f];
            j0 = 0;
            bs = (uint32_t)cr;
            c3 = (uint32_t)(cr >> 32) ^ ((uint32_t)(j + 1) << 24);
        } else {
            j0 = (uint32_t)t << 8;
            bs = (uint32_t)ctr0;
            c3 = (uint32_t)(ctr0 >> 32) ^ (0xFFFu << 20);
        }
    };
    for (int c0 = 0; c0 < n; c0 += 64 * NT) {  // chunks of at most 64 items per thread
        const int cn = min(n - c0, 64 * NT);
        uint64_t mt = 0;  // the thread's Marsaglia-Tsang items of the chunk: bit i <-> c0 + tid + i NT
        // 1. the product form, K items at a time
        for (int i0 = 0; i0 * NT < cn; i0 += K) {
            double prod[K];
            int m[K], nb[K];
            uint32_t j0[K], bs[K], c3[K];
#pragma unroll
            for (int k = 0; k < K; k++) {
                const int i = i0 + k, t = c0 + tid + i * NT;
                const bool valid = i * NT + tid < cn;
                const double al = valid ? buf[t] : -1.0;
                const bool pm = al >= 1.0 && al <= (double)GB_NMAX && al == floor(al);
                if (valid && al >= 0.0 && !pm) mt |= 1ull << i;
                if (valid && al < 0.0) buf[t] = 0.0;
                m[k] = pm ? (int)al : 0;
                nb[k] = (m[k] + 3) >> 2;
                prod[k] = 1.0;
                stream(valid ? t : c0, j0[k], bs[k], c3[k]);
            }
            for (int b = 0; b < GB_NMAX / 4; b++) {
                bool more = false;
#pragma unroll
                for (int k = 0; k < K; k++) more = more || b < nb[k];
                if (!__any(more)) break;
#pragma unroll
                for (int k = 0; k < K; k++) {
                    if (!__any(b < nb[k])) continue;
                    uint32_t p[4] = {j0[k] + (uint32_t)b, bs[k], chain, c3[k]};
                    philox4x32_10(p, key0, key1);
#pragma unroll
                    for (int q = 0; q < 4; q++) prod[k] *= 4 * b + q < m[k] ? u32o(p[q]) : 1.0;
                }
            }
#pragma unroll
            for (int k = 0; k < K; k++)
                if (m[k]) buf[c0 + tid + (i0 + k) * NT] = -flog(prod[k]);
        }
        // 2. Marsaglia-Tsang, K slots refilled from the thread's queue `mt`
        int ts[K], rd[K];
        double dk[K], ck[K], bo[K];
        uint32_t j0[K], bs[K], c3[K];
        auto take = [&](int k) {
            ts[k] = -1;
            if (mt == 0) return;
            const int i = __builtin_ctzll(mt);
            mt &= mt - 1;
            const int t = c0 + tid + i * NT;
            const double al = buf[t];
            const double a = al < 1.0 ? al + 1.0 : al;
            ts[k] = t;
            rd[k] = 0;
            dk[k] = a - 1.0 / 3.0;
            ck[k] = 1.0 / sqrt(9.0 * dk[k]);
            stream(t, j0[k], bs[k], c3[k]);
            bo[k] = 1.0;
            if (al < 1.0) {
                uint32_t p[4] = {j0[k] + 255u, bs[k], chain, c3[k]};
                philox4x32_10(p, key0, key1);
                bo[k] = pow(u53(p[0], p[1]), 1.0 / al);
            }
        };
#pragma unroll
        for (int k = 0; k < K; k++) take(k);
        for (;;) {
            bool live = false;
#pragma unroll
            for (int k = 0; k < K; k++) live = live || ts[k] >= 0;
            if (!__any(live)) break;
#pragma unroll
            for (int k = 0; k < K; k++) {
                if (!__any(ts[k] >= 0)) continue;
                uint32_t p[4] = {j0[k] + 16u + (uint32_t)rd[k], bs[k], chain, c3[k]};
                philox4x32_10(p, key0, key1);
                const double u1 = u53(p[0], p[1]), u2 = u32o(p[2]), w = u32o(p[3]);
                const double x = sqrt(-2.0 * flog(1.0 - u1)) * cospi(2.0 * u2);
                const double v = 1.0 + ck[k] * x;
                const double v3 = v * v * v, x2 = x * x;
                const bool ok = v > 0.0 && (w < 1.0 - 0.0331 * x2 * x2 ||
                                            flog(w) < 0.5 * x2 + dk[k] * (1.0 - v3 + flog(v3 > 0.0 ? v3 : 1.0)));
                rd[k]++;
                if (ts[k] >= 0 && (ok || rd[k] >= 64)) {
                    buf[ts[k]] = dk[k] * (ok ? v3 : 1.0) * bo[k];
                    take(k);
                }
            }
        }
    }
}

// MODE 0 / 2 resample: every source is redrawn from the current sample's posterior into `dst`
// (gibbs_sample_sources), with Philox uniforms (0) or the tape's (2); MODE 1 reads the sources
// `sv`.  All count the pass's sources into the count table `ct` and return the source-branch
// log-likelihood of the pass's sources, sum log t[k] (-inf when a selected normalised weight is 0,
// model.py:181-182).  Every thread of the workgroup calls it (it holds block barriers at its ends).
template <int C, int NW, int MODE>
__device__ __noinline__ TbPassOut tb_pass(TbPassArgs pa) {
    constexpr int NT = NW * WAVE;
    constexpr bool RS = MODE != 1, TP = MODE == 2;
    constexpr int ABL = SBZ_TB_ABL;  // timing ablations (diagnostic builds only, results invalid)
    const int tid = threadIdx.x, lane = tid % WAVE, wv = uni(tid / WAVE);
    const int N = pa.N, F = pa.F, S = pa.S, Z = pa.Z, Np = pa.Np, NF = N * F;
    const TbDims td = pa.td;
    const int E = td.E, CTP = td.CTP, WOFF = td.WOFF, FamC = td.FamC;
    const TbLayout L = tb_layout(td, Np, NW);
    unsigned char *base = (unsigned char *)pa.base;
    double *T = (double *)(base + (size_t)wv * L.wave);              // this wave's table [E + 1][3]
    double *cs = (double *)(base + (size_t)wv * L.wave + L.col);     // its column [NCOL]
    int *kc = (int *)(base + (size_t)wv * L.wave + L.kcnt);          // its count block [CTP]
    uint32_t *pinfo = (uint32_t *)(base + L.pinfo);                  // [Np]
    uint32_t *edl = (uint32_t *)(base + L.ed);                       // [E]
    const uint8_t *zos = (const uint8_t *)pa.zos;
    double *red = (double *)pa.red;
    int *redi = (int *)pa.redi;
    const int *perm = (const int *)pa.perm;
    const uint8_t *famc = (const uint8_t *)pa.famc, *obs_fm = (const uint8_t *)pa.obs_fm;
    const double *w = (const double *)pa.w, *pg = (const double *)pa.pg, *pz = (const double *)pa.pz,
                 *pf = (const double *)pa.pf;
    const uint8_t *sv = (const uint8_t *)pa.sv;
    uint8_t *dst = (uint8_t *)pa.dst;
    int *ct = (int *)pa.ct;
    const double *tape = (const double *)pa.tape;
    uint64_t *tbst = pa.stamps;
    const int FX = S * (1 + Z);  // counter offset of the family rows
    int err = 0;
    long long err_val = 0;
    auto wsync = [&]() {  // a wave's LDS writes are seen by its later reads (LDS keeps a wave's order)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    };
    uint64_t st_prev = SBZ_TB_STAMP ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int k) {
        if (SBZ_TB_STAMP) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const uint64_t t = __builtin_amdgcn_s_memtime();
            tbst[k] += t - st_prev;
            st_prev = t;
        }
    };

    // per-position class words: table row base | the zone counters' row << 16 | the family
    // counters' row << 24 (the count table's p_zones [zc] / p_families [fc - 1] rows; 255: none, the
    // site is in no zone / no family; CTP <= 192)
    for (int p = tid; p < Np; p += NT) {
        uint32_t pw = 0xffff0000u;
        if (p < N) {
            const int z0 = zos[perm[p]];
            const int zc = z0 < Z ? z0 : Z;
            const int fc = C == 3 ? (int)famc[p] : 0;
            const uint32_t b1 = zc < Z ? (uint32_t)(S + zc * S) : 255u;
            const uint32_t b2 = fc > 0 ? (uint32_t)(FX + (fc - 1) * S) : 255u;
            pw = (uint32_t)((zc * FamC + fc) * (S + 1)) | (b1 << 16) | (b2 << 24);
        }
        pinfo[p] = pw;
    }
    for (int e = tid; e < E; e += NT) {  // entry e: state | zone class << 8 | family class << 16
        const int x = e % (S + 1), r = e / (S + 1);
        const int zc = r / FamC, fc = r - zc * FamC;
        edl[e] = (uint32_t)x | ((uint32_t)zc << 8) | ((uint32_t)fc << 16);
    }
    for (int i = lane; i < CTP; i += WAVE) kc[i] = 0;
    if (lane < 3) T[(size_t)E * 3 + lane] = 1.0;  // the neutral entry: t = 1 (u * s below it: k = 0)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    Xoro xr{0, 0};
    const bool have = !tape || pa.pos0 + NF <= pa.len;
    if (MODE == 0) {
        uint32_t c[4] = {(uint32_t)tid, (uint32_t)pa.ctr, (uint32_t)pa.chain, (uint32_t)(pa.ctr >> 32) ^ 0xFD000000u};
        philox4x32_10(c, pa.key0, pa.key1);
        xr.s0 = ((uint64_t)c[1] << 32) | c[0];
        xr.s1 = ((uint64_t)c[3] << 32) | c[2];
        if ((xr.s0 | xr.s1) == 0) xr.s0 = 1;
    }
    // this lane's column values (three: j = lane, lane + 64, lane + 128 of the NL): base + feature *
    // stride, and the column slot (-1: none; a dummy load of w[0])
    const double *cb[3];
    int cstr[3], cslot[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const int j0 = lane + WAVE * i;
        cb[i] = w;
        cstr[i] = 0;
        cslot[i] = -1;
        if (j0 < C) {
            cb[i] = w + j0;
            cstr[i] = C;
            cslot[i] = 12 + j0;
        } else if (j0 < td.NL) {
            const int j = j0 - C;
            cstr[i] = S;
            cslot[i] = 15 + j;
            if (j < S) {
                cb[i] = pg + j;
            } else if (j < FX) {
                const int z = (j - S) / S;
                cb[i] = pz + (size_t)z * F * S + (j - S - z * S);
            } else {
                const int r = (j - FX) / S;
                cb[i] = pf + (size_t)r * F * S + (j - FX - r * S);
            }
        }
    }
    // out-of-range stores (features beyond F, positions beyond Np, counters beyond CTP) are dropped
    // by the buffer range check
    const __amdgpu_buffer_rsrc_t rdst = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, RS ? F * Np : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rct = __builtin_amdgcn_make_buffer_rsrc(ct, (short)0, F * CTP * 4, 0x00020000);
    TbLogAcc acc;
    int zf = 0;
    // a feature's loads, issued one feature ahead (a dummy feature beyond F reads the last one)
    struct Pre {
        double col[3];
        uint32_t ob[TB_NCH], sw[TB_NCH];
    };
    auto load = [&](int f, Pre &pr) {
        const int fl = min(f, F - 1);
#pragma unroll
        for (int i = 0; i < 3; i++) pr.col[i] = ldp(cb[i] + (size_t)fl * cstr[i]);
#pragma unroll
        for (int r = 0; r < TB_NCH; r++) {
            const int p0 = min(256 * r + 4 * lane, Np - 4);
            pr.ob[r] = *reinterpret_cast<const uint32_t *>(obs_fm + (size_t)fl * Np + p0);
            if (!RS)
                pr.sw[r] = __hip_atomic_load(reinterpret_cast<const uint32_t *>(sv + (size_t)fl * Np + p0), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    auto process = [&](int f, const Pre &pr) {
        // the column, then the normalised weights of the 4 classes (lanes 0..11) and their zero mask
#pragma unroll
        for (int i = 0; i < 3; i++)
            if (cslot[i] >= 0) cs[cslot[i]] = pr.col[i];
        wsync();
        bool wz = false;
        if (lane < 12) {
            const int h = lane / 3, k = lane - h * 3;
            const double w0 = cs[12] * 1.0, w1 = cs[13] * ((h & 1) ? 1.0 : 0.0);
            double sum = w0 + w1, w2 = 0.0;
            if (C == 3) {
                w2 = cs[14] * ((h & 2) ? 1.0 : 0.0);
                sum = sum + w2;
            }
            const double wn = k == 0 ? w0 / sum : (k == 1 ? w1 / sum : (C == 3 ? w2 / sum : 0.0));
            cs[lane] = wn;
            wz = k < C && wn == 0.0;
        }
        const uint32_t zmask = (uint32_t)__ballot(wz);
        wsync();
        stamp(0);
        // the table: t_k = l_k * w_norm_k (obs_terms' operations)
        if (!(ABL & 4)) {
#pragma unroll 2
            for (int e = lane; e < E; e += WAVE) {
                const uint32_t ed = edl[e];
                const int x = ed & 255, zc = (ed >> 8) & 255, fc = (int)(ed >> 16);
                const bool hz = zc < Z, hf = C == 3 && fc > 0, na = x >= S;
                const int xc = na ? 0 : x;
                const double *wn = cs + ((hz ? 1 : 0) | (hf ? 2 : 0)) * 3;
                const double *pp = cs + 15;
                const double l0 = na ? 1.0 : pp[xc];
                const double l1 = na ? 1.0 : (hz ? pp[S + zc * S + xc] : 0.0);
                const double l2 = C == 3 ? (na ? 1.0 : (hf ? pp[FX + (fc - 1) * S + xc] : 0.0)) : 0.0;
                T[e * 3] = l0 * wn[0];
                T[e * 3 + 1] = l1 * wn[1];
                T[e * 3 + 2] = C == 3 ? l2 * wn[2] : 0.0;
            }
        }
        wsync();
        stamp(1);
        // the cells: chunk r holds positions 256 r + 4 lane .. + 3
        uint32_t R[3] = {0, 0, 0};  // class counts by component, 8-bit fields by class h
#pragma unroll 1
        for (int r = 0; r < TB_NCH; r++) {
            const int p0 = 256 * r + 4 * lane;
            // the chunk's observation (source) word, selected without indexing the register array
            uint32_t obw = pr.ob[0], sww = pr.sw[0];
#pragma unroll
            for (int i = 1; i < TB_NCH; i++) {
                obw = r == i ? pr.ob[i] : obw;
                if (!RS) sww = r == i ? pr.sw[i] : sww;
            }
            const uint4 pin = *reinterpret_cast<const uint4 *>(pinfo + min(p0, Np - 4));
            const uint32_t pis[4] = {pin.x, pin.y, pin.z, pin.w};
            uint32_t outw = 0;
            uint64_t rr[2] = {0, 0};  // MODE 0: the four cells' uniforms
            if (MODE == 0) {
                rr[0] = xr.next();
                rr[1] = xr.next();
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                // (selects, no branches: every lane runs the same instructions)
                const bool val = p0 + j < N;
                const int xb = (obw >> (8 * j)) & 255;
                const int x = pa.xs8 ? xb >> 3 : xb;
                const int e = val ? (int)(pis[j] & 0xffffu) + x : E;
                const double t0 = T[e * 3], t1 = T[e * 3 + 1], t2 = C == 3 ? T[e * 3 + 2] : 0.0;
                int k;
                if constexpr (RS) {
                    double sum = t0 + t1;
                    if (C == 3) sum = sum + t2;
                    if constexpr (TP) {
                        // the reference's normalize + sample_categorical, bit for bit
                        const double u = (have && val) ? tape[pa.pos0 + (int64_t)perm[p0 + j] * F + f] : 0.0;
                        const double q0 = t0 / sum, q1 = t1 / sum, q2 = C == 3 ? t2 / sum : 0.0;
                        const double c1 = q0 + q1, c2 = c1 + q2;
                        const int k12 = u < c1 ? 1 : ((C == 3 && u < c2) ? 2 : 0);
                        k = u < q0 ? 0 : k12;
                    } else {
                        const uint32_t w32 = (j & 1) ? (uint32_t)rr[j >> 1] : (uint32_t)(rr[j >> 1] >> 32);
                        const double us = ((ABL & 8) ? 0.5 : u32u(w32)) * sum;
                        const int k12 = us < t0 + t1 ? 1 : ((C == 3 && us < sum) ? 2 : 0);
                        k = us < t0 ? 0 : k12;
                    }
                    outw |= (uint32_t)k << (8 * j);
                } else {
                    k = (sww >> (8 * j)) & 255;
                    if (k >= C && val && !err) {
                        err = 14;
                        err_val = k;
                    }
                    k = k < C ? k : 0;
                }
                const double t = __longlong_as_double(
                    k == 0 ? __double_as_longlong(t0) : (k == 1 ? __double_as_longlong(t1) : __double_as_longlong(t2)));
                if (!(ABL & 16)) {
                    acc.m *= __builtin_amdgcn_frexp_mant(t);
                    acc.e += __builtin_amdgcn_frexp_exp(t);
                }
                const uint32_t b1 = (pis[j] >> 16) & 255u, b2 = pis[j] >> 24;
                const bool hz = b1 != 255u, hf = b2 != 255u;
                if (!(ABL & 1)) {
                    // the component row's counter: p_global [x], p_zones [zc][x], p_families [fc - 1][x]
                    const uint32_t row = k == 0 ? 0u : (k == 1 ? b1 : b2);
                    if (val && x < S && row != 255u) atomicAdd(&kc[row + x], 1);
                }
                const uint32_t inc = val ? 1u << ((hz ? 8 : 0) + (hf ? 16 : 0)) : 0u;
                R[0] += k == 0 ? inc : 0u;
                R[1] += k == 1 ? inc : 0u;
                R[2] += k == 2 ? inc : 0u;
            }
            renorm(acc.m, acc.e);
            if (RS)
                __builtin_amdgcn_raw_buffer_store_b32(outw, rdst, (f < F && p0 < Np) ? f * Np + p0 : 0x7ffffff0, 0, 16);
        }
        stamp(2);
        // the class counts [h][k] (wave sums of the 8-bit fields), then the block out to the count
        // table and cleared
        int myc = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            if (k >= C) break;
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const int n = wave_sum_i((int)((R[k] >> (8 * h)) & 255u));
                myc = lane == h * 3 + k ? n : myc;
                if (((zmask >> (h * 3 + k)) & 1) && n > 0) zf = 1;
            }
        }
        if (lane < 12) kc[WOFF + lane] = myc;
        wsync();
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const int idx = lane + WAVE * i;
            int v = 0;
            if (idx < CTP) {
                v = kc[idx];
                kc[idx] = 0;
            }
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, rct, (f < F && idx < CTP) ? (f * CTP + idx) * 4 : 0x7ffffff0,
                                                  0, 16);
        }
        wsync();
        stamp(3);
    };
    Pre A, B;
    load(wv, A);
    load(wv + NW, B);
    for (int f = wv; f < F; f += 2 * NW) {
        process(f, A);
        load(f + 2 * NW, A);
        if (f + NW < F) process(f + NW, B);
        load(f + 3 * NW, B);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sources and counts have landed
    // block reductions, wave partials added in wave order; a trailing barrier, so the caller's next
    // reduction may reuse the slots
    double v = wave_sum(acc.value());
    const int zw = __ballot(zf != 0) ? 1 : 0;
    if (lane == 0) {
        red[wv] = v;
        redi[wv] = zw;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    double tot = red[0];
    int zt = redi[0];
#pragma unroll
    for (int i = 1; i < NW; i++) {
        tot += red[i];
        zt |= redi[i];
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    TbPassOut o;
    o.ll = uni(zt ? -INFINITY : tot);
    o.err = err;
    o.err_val = err_val;
    o.bad = TP && !have ? 1 : 0;
    return o;
}

// One workgroup of NW waves runs one chain.  Every decision is uniform across the workgroup:
// all waves draw the same values from identical RNG states and take the same branches; the
// NW * 64 threads share the N * F passes (block reductions through LDS, summed in wave order)
// and the per-feature Gibbs draws.  Shared LDS state (zone assignment, counters) is written by
// thread 0 and published by a barrier.
// GS: the current sources are the chain's own array in HBM (updated in place) and the candidate
// sources a per-chain scratch row, for N * F too large for LDS, both POSITION-MAJOR ([F][Np], the
// context's family-sorted site order; launch_mh_source transposes a caller's site-major array):
// the N * F passes then walk the cells feature by feature, consecutive threads on consecutive
// positions, so every source and observation access is coalesced.  Only this chain's threads
// touch them; they exchange cells through agent-scope (sc1, L1-bypassing) byte accesses and a
// vmcnt(0) wait at every barrier.  Without GS the sources live in LDS as [N][F]; a.src_pm says
// which layout the chain's array in HBM has (copied in and out at the launch's ends).
// TB (with GS): the N * F passes are the feature-table passes above and the Gibbs parameter
// operators take their counts from the chain's count table; the current and candidate sources
// (and count tables) swap roles on an accepted move instead of being copied.
template <int C, bool GS, int NW, bool TB = false>
__global__ __launch_bounds__(NW * WAVE) void mh_src_kernel(MhArgs a) {
    static_assert(GS || !TB, "the table passes walk sources kept in HBM");
    constexpr int NT = NW * WAVE;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int lane = tid % WAVE;
    const int wv = uni(tid / WAVE);
    const int b = blockIdx.x;
    const int N = a.N, F = a.F, S = a.S, Z = a.Z, Fam = (C == 3) ? a.Fam : 0;
    const int NF = N * F;
    const sbz_chains &ch = a.ch;

    // LDS carve-up (reduction slots, then ints, then u16, then bytes)
    double *red = reinterpret_cast<double *>(lds);                    // [2][MH_SRC_MAX_WAVES]
    int *redi = reinterpret_cast<int *>(red + 2 * MH_SRC_MAX_WAVES);   // [2][MH_SRC_MAX_WAVES]
    const int ncnt = F * (S > C ? S : C);
    int *cnt = redi + 2 * MH_SRC_MAX_WAVES;                           // [F][max(S, C)] counts
    int *zsize = cnt + ncnt;                                          // [Z]
    int *stat = zsize + ((Z + 1) & ~1);                               // [MH_STAT_INTS]
    uint16_t *nb = reinterpret_cast<uint16_t *>(stat + MH_STAT_INTS);  // [N] neighbour stamps
    uint8_t *src = reinterpret_cast<uint8_t *>(nb + ((N + 1) & ~1));   // [N][F] current sources
    uint8_t *srcb = src + (GS ? 0 : ((NF + 15) & ~15));              // [N][F] candidate sources
    uint8_t *zos = srcb + (GS ? 0 : ((NF + 15) & ~15));              // [N] zone of site
    uint8_t *sub = zos + ((N + 15) & ~15);                           // [F] feature subset
    // geo prior scratch (geo_zone_prior), 16-B aligned after the subset
    // (offsets from sizes, not pointer differences against the LDS base)
    const size_t sub_end = (size_t)2 * MH_SRC_MAX_WAVES * (8 + 4) + (size_t)ncnt * 4 + (size_t)((Z + 1) & ~1) * 4 +
                           (size_t)MH_STAT_INTS * 4 + (size_t)((N + 1) & ~1) * 2 +
                           (GS ? 0 : (size_t)2 * ((NF + 15) & ~15)) + (size_t)((N + 15) & ~15) + (size_t)((F + 15) & ~15);
    const size_t geo_off = (sub_end + 15) & ~(size_t)15;
    double *geo_key = reinterpret_cast<double *>(lds + geo_off);
    uint16_t *geo_mem = reinterpret_cast<uint16_t *>(geo_key + N);
    int *geo_cnt = reinterpret_cast<int *>(geo_mem + ((N + 7) & ~7));
    double *geo_rd = reinterpret_cast<double *>(geo_cnt + 4);
    int *geo_ri = reinterpret_cast<int *>(geo_rd + 16);
    // redraw_rows scratch, 16-B aligned after the geo scratch
    const size_t par_off = (geo_off + (a.geo_cost ? geo_scratch_bytes(N) : 0) + 15) & ~(size_t)15;
    // TB: the operator CDF first, then one region holding either the redraw scratch (Gibbs
    // parameter operators) or the table-pass buffers (tb_layout)
    const size_t uni_off = TB ? ((par_off + (size_t)SBZ_N_OPS * 8 + 15) & ~(size_t)15) : par_off;
    double *gbuf = reinterpret_cast<double *>(lds + uni_off);  // [F][max(S, 2)] draws
    int *fpre = reinterpret_cast<int *>(gbuf + (size_t)F * max(S, 2));  // [F] tape offset of feature f
    int *frank = fpre + F;                                      // [F] counter rank of feature f
    int *misc_i = frank + F;                                    // [2] totals of those scans
    // a.stage: the N*F passes read the chain's parameters and normalised weights from LDS copies
    // (staged when a pass starts after the parameters changed) instead of L2
    // the operator CDF (once per launch), 8-B aligned after misc_i
    const size_t cdf_off = TB ? par_off : (par_off + (size_t)F * max(S, 2) * 8 + (size_t)F * 8 + 8 + 7) & ~(size_t)7;
    double *cdf = reinterpret_cast<double *>(lds + cdf_off);  // [SBZ_N_OPS]
    // (read through a local-address-space pointer: ds_read, not a flat load)
    const __attribute__((address_space(3))) double *cdf3 =
        (const __attribute__((address_space(3))) double *)((__attribute__((address_space(3))) unsigned char *)lds + cdf_off);
    const size_t stg_off = (cdf_off + (size_t)SBZ_N_OPS * 8 + 15) & ~(size_t)15;
    double *lnw = reinterpret_cast<double *>(lds + stg_off);  // [F][4][3] by h = hz | hf << 1
    double *lpg = lnw + (size_t)F * 12;                        // [F][S]
    double *lpz = lpg + (size_t)F * S;                         // [Z][F][S]
    double *lpf = lpz + (size_t)Z * F * S;                     // [Fam][F][S]
    uint8_t *lobs = reinterpret_cast<uint8_t *>(lpf + (size_t)Fam * F * S);  // [N][F] x by site
    uint8_t *lfam = lobs + NF;                                                 // [N] family class
    const bool stg = a.stage != 0;
    bool stg_ok = false;
    // a.cstage: the constant tables, after the staged parameters (16-B aligned)
    const bool cst = a.cstage != 0;
    // (TB: after the region of the redraw scratch / pass buffers, as mh_src_lds_bytes counts it)
    const size_t cst_off =
        TB ? (uni_off + max(tb_layout(tb_dims(S, Z, Fam, C), a.Np, NW).end, redraw_bytes(F, S)) + 15) & ~(size_t)15
           : (stg_off + ((size_t)F * 12 + (size_t)(1 + Z + Fam) * F * S) * 8 + (size_t)NF + N + 15) & ~(size_t)15;
    const int FS = F * S;
    // (the global tables are read with ldp, as before staging: a plain LDS load and an atomic
    // global one are never merged into one load through a generic pointer)
    double *c_alg = reinterpret_cast<double *>(lds + cst_off);   // [F][S] if alpha_g
    double *c_alf = c_alg + (a.alpha_g ? FS : 0);                  // [Fam][F][S] if alpha_f
    double *c_gcg = c_alf + (a.alpha_f ? Fam * FS : 0);            // [F][S] if gc_g
    double *c_gcf = c_gcg + (a.gc_g ? FS : 0);                     // [Fam][F][S] if gc_f
    uint8_t *c_app = reinterpret_cast<uint8_t *>(c_gcf + (a.gc_f ? Fam * FS : 0));  // [F][S]
    uint8_t *c_acnt = c_app + FS;                                                   // [F]
    auto app_cnt = [&](int f) -> int { return cst ? (int)lds_rd(c_acnt + f) : a.app_cnt[f]; };
    auto app_list = [&](int f, int j) -> int { return cst ? (int)lds_rd(c_app + f * S + j) : a.app_list[(size_t)f * S + j]; };
    // Gibbs prior count of component comp's row `row` at i = f * S + x (1 where none is set)
    auto gcv = [&](int comp, int row, int i) -> double {
        if (comp == 0 && a.gc_g) return cst ? lds_rd(c_gcg + i) : ldp(a.gc_g + i);
        if (comp == 2 && a.gc_f) return cst ? lds_rd(c_gcf + (size_t)row * FS + i) : ldp(a.gc_f + (size_t)row * FS + i);
        return 1.0;
    };
    // 'counts' prior alpha (p_global, p_families) at i, where set
    auto has_al = [&](int comp) { return (comp == 0 && a.alpha_g) || (comp == 2 && a.alpha_f); };
    auto alv = [&](int comp, int row, int i) -> double {
        if (comp == 0) return cst ? lds_rd(c_alg + i) : ldp(a.alpha_g + i);
        return cst ? lds_rd(c_alf + (size_t)row * FS + i) : ldp(a.alpha_f + (size_t)row * FS + i);
    };

    uint8_t *gzos = ch.zone_of_site + (size_t)b * N;
    const int Np = a.Np;
    const size_t NFP = (size_t)F * Np;  // position-major cells per chain
    uint8_t *gsrc = ch.source + (size_t)b * (a.src_pm ? NFP : (size_t)NF);
    if (GS) {
        src = gsrc;
        srcb = a.src_scratch + (size_t)b * NFP;
    }
    // source cell access
    auto rsrc = [&](const uint8_t *p, int c) -> int {
        if constexpr (GS) return __hip_atomic_load(p + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else return p[c];
    };
    auto wsrc = [&](uint8_t *p, int c, int v) {
        if constexpr (GS) __hip_atomic_store(p + c, (uint8_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else p[c] = (uint8_t)v;
    };
    // workgroup barrier after this thread's LDS (and, GS / parameter stores, global) accesses
    // completed; a compiler memory barrier on both sides
    auto sync = [&]() {
        if constexpr (GS) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    auto gsync = [&]() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // block reductions (deterministic: wave partials summed in wave order); uniform results
    int rslot = 0;
    auto bsum = [&](double v) -> double {
        v = wave_sum(v);
        double *r = red + rslot * MH_SRC_MAX_WAVES;
        rslot ^= 1;
        if (lane == 0) r[wv] = v;
        sync();
        double t = r[0];
#pragma unroll
        for (int i = 1; i < NW; i++) t += r[i];
        return uni(t);
    };
    int islot = 0;
    auto bor = [&](int v) -> int {
        const int wvv = __ballot(v != 0) ? 1 : 0;
        int *r = redi + islot * MH_SRC_MAX_WAVES;
        islot ^= 1;
        if (lane == 0) r[wv] = wvv;
        sync();
        int t = 0;
#pragma unroll
        for (int i = 0; i < NW; i++) t |= r[i];
        return uni(t);
    };
    double *w = ch.w + (size_t)b * F * C;
    double *pg = ch.p_global + (size_t)b * F * S;
    double *pz = Z > 0 ? ch.p_zones + (size_t)b * Z * F * S : pg;
    double *pf = (C == 3 && Fam > 0) ? ch.p_fam + (size_t)b * Fam * F * S : pg;
    const int max_size = ch.max_size[b];
    const double p_grow = ch.p_grow_connected[b];

    for (int z = tid; z < Z; z += NT) zsize[z] = 0;
    if (a.stage) {  // the observations and family classes never change: staged once
        for (int c = tid; c < NF; c += NT) lobs[c] = a.obs_sm[c];
        for (int s = tid; s < N; s += NT) lfam[s] = C == 3 ? a.fam_site[s] : 0;
    }
    if (tid < SBZ_N_OPS - 1) cdf[tid] = a.op_cdf[tid];
    if (cst) {  // so do the constant tables
        for (int i = tid; i < FS; i += NT) {
            c_app[i] = (uint8_t)a.app_list[i];
            if (a.alpha_g) c_alg[i] = a.alpha_g[i];
            if (a.gc_g) c_gcg[i] = a.gc_g[i];
        }
        for (int i = tid; i < Fam * FS; i += NT) {
            if (a.alpha_f) c_alf[i] = a.alpha_f[i];
            if (a.gc_f) c_gcf[i] = a.gc_f[i];
        }
        for (int f = tid; f < F; f += NT) c_acnt[f] = (uint8_t)a.app_cnt[f];
    }
    if (tid < MH_STAT_INTS) stat[tid] = 0;
    for (int s = tid; s < N; s += NT) nb[s] = 0;
    if (!GS) {
        if (a.src_pm) {  // [F][Np] by position -> [N][F] by site
            for (int i = tid; i < (int)NFP; i += NT) {
                const int f = i / Np, p = i - f * Np;
                if (p < N) src[a.perm[p] * F + f] = gsrc[i];
            }
        } else {
            for (int c = tid; c < NF; c += NT) src[c] = gsrc[c];
        }
    }
    sync();
    int occ = 0;
    for (int s = tid; s < N; s += NT) {
        const int z = gzos[s];
        zos[s] = (uint8_t)z;
        if (z < Z) {
            atomicAdd(&zsize[z], 1);
            occ++;
        }
    }
    int occupied = (int)bsum((double)occ);
    sync();
    // 'cost_based' geo prior: only the last zone counts (model.py:1110-1139); its current value
    auto geo_prior = [&]() -> double {
        return geo_zone_prior<NW>(a.geo_cost, a.geo_scale, N, zos, Z - 1, -1, -1, -1, geo_key, geo_mem,
                                  geo_cnt, geo_rd, geo_ri);
    };
    double geo_cur = (a.geo_cost && Z > 0) ? geo_prior() : 0.0;

    Rng rng;
    rng.tape = ch.tape ? ch.tape + (size_t)b * ch.tape_stride : nullptr;
    rng.pos = ch.tape ? uni64(ch.tape_pos[b]) : 0;
    rng.len = ch.tape ? uni64(ch.tape_len[b]) : 0;
    rng.key0 = (uint32_t)ch.seed;
    rng.key1 = (uint32_t)(ch.seed >> 32);
    rng.chain = ch.chain_id0 + (uint64_t)b;
    rng.ctr = ch.counter ? (uint64_t)uni64((int64_t)ch.counter[b]) : 0;
    rng.bad = 0;

    double ll = ch.ll[b];
    double prior = ch.prior ? ch.prior[b] : 0.0;
    int alias = ch.alias_pending ? uni(ch.alias_pending[b]) : 0;
    int err = 0;
    long long err_val = 0;
    uint16_t stamp = 0;

    // ---- zone-move helpers (as the SAMPLE_SOURCE = false kernel, sbz_mh.hip).  The scans over
    // the sites run in every wave (identical results); the stamps are written by all threads.
    auto mark = [&](int z) {
        stamp++;
        if (stamp == 0) {
            for (int s = tid; s < N; s += NT) nb[s] = 0;
            sync();
            stamp = 1;
        }
        for (int s = tid; s < N; s += NT)
            if (zos[s] == z)
                for (int e = a.adj_ptr[s]; e < a.adj_ptr[s + 1]; e++)
                    nb[MH_IDX(a.adj_idx[MH_IDX(e, a.nnz, 1)], N, 2)] = stamp;
        sync();
    };
    auto is_nb = [&](int s) { return nb[s] == stamp && zos[s] == NONE; };
    enum { SEL_NB = 0, SEL_FREE = 1, SEL_ZONE = 2 };
    auto sel = [&](int mode, int z, int s) -> bool {
        const int zs = zos[s];
        return mode == SEL_NB ? (nb[s] == stamp && zs == NONE) : (mode == SEL_FREE ? zs == NONE : zs == z);
    };
    auto count_sel = [&](int mode, int z) -> int {
        int c = 0;
        for (int s0 = 0; s0 < N; s0 += WAVE) {
            const int s = s0 + lane;
            const bool f = s < N ? sel(mode, z, min(s, N - 1)) : false;
            c += __popcll(__ballot(f));
        }
        return uni(c);
    };
    auto kth_sel = [&](int mode, int z, int k) -> int {
        int found = -1;
        for (int s0 = 0; s0 < N; s0 += WAVE) {
            const int s = s0 + lane;
            const bool f = s < N ? sel(mode, z, min(s, N - 1)) : false;
            const uint64_t m = __ballot(f);
            const int n = __popcll(m);
            if (found < 0 && k < n) {
                const uint64_t hit = __ballot(f && lane_prefix(m) == k);
                found = hit ? s0 + (int)__builtin_ctzll(hit) : -1;
                k = -1;
            } else if (found < 0) {
                k -= n;
            }
        }
        return uni(found);
    };

    // normalize_weights (model.py:436-452) of feature f's weights for the 4 classes h = hz | hf << 1
    auto stage_nw = [&](int f, double w0r, double w1r, double w2r) {
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const double w0 = w0r * 1.0, w1 = w1r * ((h & 1) ? 1.0 : 0.0);
            double sum = w0 + w1, w2 = 0.0;
            if (C == 3) {
                w2 = w2r * ((h & 2) ? 1.0 : 0.0);
                sum = sum + w2;
            }
            lnw[(f * 4 + h) * 3] = w0 / sum;
            lnw[(f * 4 + h) * 3 + 1] = w1 / sum;
            lnw[(f * 4 + h) * 3 + 2] = C == 3 ? w2 / sum : 0.0;
        }
    };
    auto ensure_staged = [&]() {
        if (!stg || stg_ok) return;
        const int fs = F * S;
        for (int i = tid; i < fs; i += NT) lpg[i] = ldp(pg + i);
        for (int i = tid; i < Z * fs; i += NT) lpz[i] = ldp(pz + i);
        if (C == 3)
            for (int i = tid; i < Fam * fs; i += NT) lpf[i] = ldp(pf + i);
        for (int f = tid; f < F; f += NT)
            stage_nw(f, ldp(w + (size_t)f * C), ldp(w + (size_t)f * C + 1), C == 3 ? ldp(w + (size_t)f * C + 2) : 0.0);
        sync();
        stg_ok = true;
    };
    // obs_terms from the staged copies (the same values, the same operations); x = the observed
    // state of (s, f) (S = NA)
    auto terms_z = [&](int s, int f, int x, int zc, double (&l)[3], double (&wn)[3]) {
        if (!stg) {
            const int fc = C == 3 ? a.fam_site[s] : 0;
            obs_terms<C>(a, w, pg, pz, pf, f, x, zc, fc, l, wn);
            return;
        }
        const int fc = lfam[s];
        const bool na = x >= S;
        const int xc = na ? 0 : x;
        const bool hz = zc < Z, hf = (C == 3) && fc > 0;
        const double *q = lnw + ((size_t)f * 4 + (hz ? 1 : 0) + (hf ? 2 : 0)) * 3;
        wn[0] = q[0];
        wn[1] = q[1];
        wn[2] = q[2];
        l[0] = na ? 1.0 : lpg[f * S + xc];
        l[1] = na ? 1.0 : (hz ? lpz[(zc * F + f) * S + xc] : 0.0);
        l[2] = (C == 3) ? (na ? 1.0 : (hf ? lpf[((fc - 1) * F + f) * S + xc] : 0.0)) : 0.0;
    };
    auto terms = [&](int s, int f, int x, double (&l)[3], double (&wn)[3]) { terms_z(s, f, x, zos[s], l, wn); };
    // ---- passes over the N*F observations; (s, f) stepped with the cell index instead of a
    // division per cell.  body(s, f, x, g, c): x the observed state, g the cell's index in the
    // source arrays, c = s * F + f its index in C order (the reference's order of the tape's
    // per-observation uniforms).  Without GS the cells go in C order (g = c, LDS [N][F]); with GS
    // position-major (g = f * Np + p, s = perm[p]), so consecutive threads read consecutive bytes.
    const int cdS = NT / F, cdF = NT - cdS * F;
    const int pdF = NT / Np, pdP = NT - pdF * Np;
    const int xdiv = a.xs8 ? 8 : 1;
    auto for_cells = [&](auto &&body) {
        if constexpr (!GS) {
            CellWalk cw{tid / F, tid - (tid / F) * F, cdS, cdF, F};
#pragma unroll SBZ_SRC_UNR
            for (int c = tid; c < NF; c += NT, cw.next()) {
                const int x = stg ? lds_rd(lobs + c) : a.obs_sm[c];
                body(cw.s, cw.f, x, c, c);
            }
        } else {
            PosWalk pw{tid - (tid / Np) * Np, tid / Np, pdP, pdF, Np};
#pragma unroll SBZ_SRC_UNR
            for (int i = tid; i < (int)NFP; i += NT, pw.next()) {
                const int p = pw.p, f = pw.f;
                if (p >= N) continue;
                const int s = a.perm[p];
                const int c = s * F + f;
                const int x = stg ? lds_rd(lobs + c) : a.obs_fm[i] / xdiv;
                body(s, f, x, i, c);
            }
        }
    };
    // Sums of logs as one log per thread: each factor's mantissa multiplies a product and its
    // exponent adds to an integer (exact for any factor, denormals included), the product is
    // renormalised every 8 cells, and log(m) + e ln 2 is taken once (~1e-16 relative).
    struct LogAcc {
        double m = 1.0;
        int e = 0, k = 0;
        __device__ __forceinline__ void add(double v) {
            e += __builtin_amdgcn_frexp_exp(v);
            m *= __builtin_amdgcn_frexp_mant(v);
            if (++k == 8) {
                k = 0;
                e += __builtin_amdgcn_frexp_exp(m);
                m = __builtin_amdgcn_frexp_mant(m);
            }
        }
        __device__ __forceinline__ double value() const { return flog(m) + (double)e * LN2; }
    };
    // sum over observations of log posterior[src] for the current sample (zone_sampling.py:718-722)
    auto pass_logq = [&]() -> double {
        ensure_staged();
        LogAcc acc;
        for_cells([&](int s, int f, int x, int g, int) {
            double l[3], wn[3], p[3];
            terms(s, f, x, l, wn);
            posterior_draw<C>(l, wn, 2.0, p);
            acc.add(p[rsrc(src, g)]);
        });
        return bsum(acc.value());
    };
    // log-likelihood of the current sample with sources `sv` (combine_lh source branch,
    // model.py:177-184): sum log(w_src * lh_src), -inf if a selected weight is 0
    auto pass_ll = [&](const uint8_t *sv) -> double {
        ensure_staged();
        LogAcc acc;
        int zero_w = 0;
        if (SBZ_SRC_LL1 && stg) {
            // staged: only the selected component's weight and likelihood, two LDS reads per
            // cell whose addresses come straight from the cell's bytes (the same products as
            // terms(): a component the site lacks has weight 0, so its likelihood is irrelevant)
            for_cells([&](int s, int f, int x, int g, int) {
                const int k = rsrc(sv, g);
                const int zc = zos[s], fc = C == 3 ? lfam[s] : 0;
                const bool na = x >= S;
                const int xc = na ? 0 : x;
                const int h = (zc < Z ? 1 : 0) | ((C == 3 && fc > 0) ? 2 : 0);
                const double wk = lnw[(f * 4 + h) * 3 + k];
                const int zr = zc < Z ? zc : 0, fr = fc > 0 ? fc - 1 : 0;
                // lpg, lpz, lpf are consecutive: [F][S], [Z][F][S], [Fam][F][S]
                const int pi = k == 0 ? f * S + xc
                                      : (k == 1 ? (F + zr * F + f) * S + xc : (F + Z * F + fr * F + f) * S + xc);
                const double lk = na ? 1.0 : lpg[pi];
                zero_w |= wk == 0.0;
                acc.add(wk * lk);
            });
        } else {
            for_cells([&](int s, int f, int x, int g, int) {
                double l[3], wn[3];
                terms(s, f, x, l, wn);
                const int k = rsrc(sv, g);
                zero_w |= wn[k] == 0.0;
                acc.add(wn[k] * l[k]);
            });
        }
        const double v = bsum(acc.value());
        return bor(zero_w) ? -INFINITY : v;
    };
    // redraw every source from the current sample's posterior into srcb; returns log q (sum log
    // posterior[new source]) and the new log-likelihood
    auto pass_resample = [&](double &log_q_s, double &ll_new) {
        ensure_staged();
        LaneRng lr;
        lr.initw(rng, tid);
        LogAcc acc_q, acc_l;
        int zero_w = 0;
        const int64_t pos0 = rng.pos;
        const bool have = !rng.tape || pos0 + NF <= rng.len;
        for_cells([&](int s, int f, int x, int g, int c) {
            double l[3], wn[3], p[3];
            terms(s, f, x, l, wn);
            const double u = rng.tape ? (have ? rng.tape[pos0 + c] : 0.0) : lr.u();
            const int k = posterior_draw<C>(l, wn, u, p);
            wsrc(srcb, g, k);
            acc_q.add(p[k]);
            zero_w |= wn[k] == 0.0;
            acc_l.add(wn[k] * l[k]);
        });
        if (rng.tape) {
            if (!have) rng.bad = 1;
            rng.pos = uni64(pos0 + NF);
        } else {
            rng.ctr++;
        }
        log_q_s = bsum(acc_q.value());
        const double v = bsum(acc_l.value());
        ll_new = bor(zero_w) ? -INFINITY : v;
    };
    auto commit_sources = [&]() {
        for (int c = tid; c < (GS ? (int)NFP : NF); c += NT) wsrc(src, c, rsrc(srcb, c));
        sync();
    };

    // ---- TB: the feature-table passes (tb_pass) and the chain's count tables (current / candidate)
    const TbDims td = tb_dims(S, Z, Fam, C);
    int *ct_cur = TB ? a.ctab + (size_t)b * F * td.CTP : nullptr;
    int *ct_alt = TB ? a.ctab + a.ct_half + (size_t)b * F * td.CTP : nullptr;
    // One pass over every observation (tb_pass), the generator advanced as the pass drew
    uint64_t tbst[16] = {};
    auto tpass = [&](auto mode_c, const uint8_t *sv, uint8_t *dst, int *ct) -> double {
        constexpr int MODE = decltype(mode_c)::value;
        TbPassArgs pa;
        pa.N = N;
        pa.F = F;
        pa.S = S;
        pa.Z = Z;
        pa.Np = Np;
        pa.xs8 = a.xs8;
        pa.td = td;
        pa.perm = (gbl_ptr<const int>)a.perm;
        pa.famc = (gbl_ptr<const uint8_t>)a.famc;
        pa.obs_fm = (gbl_ptr<const uint8_t>)a.obs_fm;
        pa.zos = (lds_ptr<uint8_t>)zos;
        pa.base = (lds_ptr<unsigned char>)(lds + uni_off);
        pa.red = (lds_ptr<double>)red;
        pa.redi = (lds_ptr<int>)redi;
        pa.w = (gbl_ptr<const double>)w;
        pa.pg = (gbl_ptr<const double>)pg;
        pa.pz = (gbl_ptr<const double>)pz;
        pa.pf = (gbl_ptr<const double>)pf;
        pa.sv = (gbl_ptr<const uint8_t>)sv;
        pa.dst = (gbl_ptr<uint8_t>)dst;
        pa.ct = (gbl_ptr<int>)ct;
        pa.tape = (gbl_ptr<const double>)rng.tape;
        pa.pos0 = rng.pos;
        pa.len = rng.len;
        pa.key0 = rng.key0;
        pa.key1 = rng.key1;
        pa.chain = rng.chain;
        pa.ctr = rng.ctr;
        pa.stamps = SBZ_TB_STAMP ? tbst : nullptr;
        if (SBZ_TB_STAMP) tbst[4]++;  // passes
        const TbPassOut o = tb_pass<C, NW, MODE>(pa);
        if (o.err && !err) {
            err = o.err;
            err_val = o.err_val;
        }
        if (MODE == 2) {
            if (o.bad) rng.bad = 1;
            rng.pos = uni64(rng.pos + NF);
        } else if (MODE == 0) {
            rng.ctr++;
        }
        return uni(o.ll);
    };
    // a resample pass with the draws' source (tape or Philox)
    auto tresample = [&](int *ct) -> double {
        return rng.tape ? tpass(std::integral_constant<int, 2>(), src, srcb, ct)
                        : tpass(std::integral_constant<int, 0>(), src, srcb, ct);
    };
    // per-feature counts of sources / states into cnt
    auto clear_cnt = [&]() {
        for (int i = tid; i < ncnt; i += NT) cnt[i] = 0;
        sync();
    };
    // F uniforms -> sub[f] = u < fraction (np.random.random(n_features) < 0.4, :335, :383)
    auto draw_subset = [&]() {
        LaneRng lr;
        lr.initw(rng, tid);
        const int64_t pos0 = rng.pos;
        const bool have = !rng.tape || pos0 + F <= rng.len;
        for (int f = tid; f < F; f += NT) {
            const double u = rng.tape ? (have ? rng.tape[pos0 + f] : 1.0) : lr.u();
            sub[f] = u < 0.4 ? 1 : 0;
        }
        if (rng.tape) {
            if (!have) rng.bad = 1;
            rng.pos = uni64(pos0 + F);
        } else {
            rng.ctr++;
        }
        sync();
    };
    // Every feature f with sub[f]: p_row(f)[idx] = np.random.dirichlet(alpha) over f's applicable
    // states, alpha_x = base(x) + cnt[f][x]; the values come from the tape (in feature order, idx
    // order) or from per-lane gammas.  Wave w draws the features f = w (mod NW); a running scan in
    // feature order gives each feature its tape offset / Philox counter, so the draws do not
    // depend on NW.  Returns the change of the 'counts' prior (xlogy(alpha_prior - 1, p) terms)
    // if al != null.
    // (the generator's fields come in as values and go out through pos / ctr / bad: the lambda
    // does not touch `rng`, which keeps it in registers)
    // want_dl (TB): also the source log-likelihood's change, sum over the redrawn entries of
    // cnt * (log new - log old) (the cells whose source is this row's component and state); dzf set
    // where that sum is not exact (an old or new value 0 / not finite under a non-zero count)
    auto redraw_rows = [&](double *base, double *lbase, int comp, int row,
                           const double *tape, int64_t len, uint32_t key0, uint32_t key1,
                           uint64_t chain, int64_t &pos, uint64_t &ctr, int &bad, bool want_dl, double &dll,
                           int &dzf) -> double {
        // every (feature, state) draw at once: thread t <-> (f, j) = (t / S, t % S).  Feature f's
        // draws are its tape values pos + fpre[f] + j, or the gammas of lane stream j at counter
        // ctr + frank[f] (LaneRng, as one wave per feature drew them), fpre / frank the exclusive
        // scans over the subset features (wave 0, 64 features at a time).  Philox needs only frank:
        // every wave counts the subset blocks by ballots and writes the ranks of its own blocks.
        if (!tape) {
            int cr = 0;
            for (int f0 = 0; f0 < F; f0 += WAVE) {
                const int f = f0 + lane;
                const uint64_t m = __ballot(f < F && sub[f]);
                if ((f0 / WAVE) % NW == wv && f < F) frank[f] = cr + lane_prefix(m);
                cr += __popcll(m);
            }
            if (tid == 0) {
                misc_i[0] = 0;
                misc_i[1] = cr;
            }
        } else if (wv == 0) {
            int cn = 0, cr = 0;
            for (int f0 = 0; f0 < F; f0 += WAVE) {
                const int f = f0 + lane;
                const int in = f < F && sub[f];
                int v = in ? app_cnt(f) : 0;
#pragma unroll
                for (int o = 1; o < WAVE; o <<= 1) {
                    const int t = __shfl_up(v, o, WAVE);
                    if (lane >= o) v += t;
                }
                const uint64_t m = __ballot(in);
                if (f < F) {
                    fpre[f] = cn + v - (in ? app_cnt(f) : 0);
                    frank[f] = cr + lane_prefix(m);
                }
                cn += uni(__shfl(v, WAVE - 1, WAVE));
                cr += __popcll(m);
            }
            if (lane == 0) {
                misc_i[0] = cn;
                misc_i[1] = cr;
            }
        }
        sync();
        uint64_t rst = SBZ_TB_STAMP ? __builtin_amdgcn_s_memtime() : 0;
        auto rstamp = [&](int k) {  // SBZ_TB_STAMP: scan / alphas / gammas / rows
            if (SBZ_TB_STAMP) {
                const uint64_t t = __builtin_amdgcn_s_memtime();
                tbst[k] += t - rst;
                rst = t;
            }
        };
        rstamp(8);
        const int tot_n = uni(misc_i[0]), tot_r = uni(misc_i[1]);
        const int64_t pos0 = pos;
        const uint64_t ctr0 = ctr;
        const bool have = !tape || pos0 + tot_n <= len;
        if (tape) {
            for (int t = tid; t < FS; t += NT) {
                const int f = t / S, j = t - f * S;
                const bool act = sub[f] && j < app_cnt(f);
                gbuf[t] = act && have ? tape[pos0 + fpre[f] + j] : 0.0;
            }
        } else {
            // Philox: item (f, j)'s alpha, then the gammas (gamma_fill, the same thread's items)
            {
                const int dF = NT / S, dJ = NT - dF * S;
                int f = tid / S, j = tid - f * S;
                for (int t = tid; t < FS; t += NT) {
                    const bool act = sub[f] && j < app_cnt(f);
                    const int x = app_list(f, j);
                    gbuf[t] = act ? gcv(comp, row, f * S + x) + (double)cnt[f * S + x] : -1.0;
                    f += dF;
                    j += dJ;
                    if (j >= S) {
                        j -= S;
                        f++;
                    }
                }
            }
            rstamp(9);
            gamma_fill<SBZ_RB_REDRAW, NT>((lds_ptr<double>)gbuf, FS, S, (lds_ptr<const int>)frank, key0, key1,
                                          (uint32_t)chain, ctr0, 0);
        }
        sync();
        rstamp(10);
        double dp = 0.0, dl = 0.0;
        int zfl = 0;
        const bool al = has_al(comp);
        // Philox: each feature's total of its draws, once (over fpre / frank, no longer needed)
        double *ftot = reinterpret_cast<double *>(fpre);
        if (!tape) {
            for (int f = tid; f < F; f += NT) {
                const int n = app_cnt(f);
                double tot = 0.0;
                for (int i = 0; i < n; i++) tot += gbuf[f * S + i];
                ftot[f] = tot;
            }
            sync();
        }
        // four items per thread at a time: their loads (the old values from L2) first; item
        // t = t0 + u NT is (f, j) = (t / S, t % S), walked by (NT / S, NT % S) steps
        const int dF = NT / S, dJ = NT - dF * S;
        for (int t0 = tid; t0 < FS; t0 += 4 * NT) {
            int ns[4], xs[4], fs[4], js[4];
            double olds[4];
            {
                int f = t0 / S, j = t0 - f * S;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    fs[u] = min(f, F - 1);
                    js[u] = f < F ? j : 0;
                    f += dF;
                    j += dJ;
                    if (j >= S) {
                        j -= S;
                        f++;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int f = fs[u], j = js[u];
                ns[u] = app_cnt(f);
                xs[u] = app_list(f, j);  // (entries past the count are 0)
                // the current value: the staged copy once staged (an exact copy), else the global row
                olds[u] = stg_ok ? lds_rd(lbase + (size_t)f * S + xs[u]) : ldp(base + (size_t)f * S + xs[u]);
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int t = t0 + u * NT;
                if (t >= FS) break;
                const int f = fs[u], j = js[u], n = ns[u], x = xs[u];
                if (!(sub[f] && j < n)) continue;
                double g = gbuf[t];
                if (!tape) g = g / ftot[f];
                const double old = olds[u];
                stp(base + (size_t)f * S + x, g);
                if (stg) lbase[(size_t)f * S + x] = g;  // the staged copy follows
                if (al) {
                    const double am1 = alv(comp, row, f * S + x) - 1.0;
                    dp += xlogy(am1, g) - xlogy(am1, old);
                }
                if (want_dl) {
                    const int c = cnt[f * S + x];
                    if (c > 0) {
                        // (one log of the ratio)
                        if (g > 0.0 && old > 0.0 && g < INFINITY && old < INFINITY) dl += (double)c * flog(g / old);
                        else zfl = 1;
                    }
                }
            }
        }
        if (want_dl) {
            dll = bsum(dl);
            dzf = bor(zfl);
        }
        rstamp(11);
        bad = have ? 0 : 1;
        pos = uni64(pos0 + (tape ? tot_n : 0));
        ctr = (uint64_t)uni64((int64_t)(ctr0 + (tape ? 0 : (uint64_t)tot_r)));
        // once the parameters are staged every later read of them is the LDS copy (passes, `old`
        // above), so the global stores need not have landed before the next barrier; the alias copy
        // and the end of the kernel wait for them
        if (!(stg && stg_ok)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return bsum(dp);
    };

    // ---- gibbsish_sample_zones scratch (a.gib): per available site its two log marginals, the
    // available list, its in / out flags, and the position of every site (GS: cells by position)
    double *g_lw = reinterpret_cast<double *>(lds + a.gib_off);  // [N]
    double *g_lwo = g_lw + N;                                     // [N]
    uint16_t *g_lst = reinterpret_cast<uint16_t *>(g_lwo + N);    // [N]
    uint16_t *g_pos = g_lst + N;                                  // [N] (GS only)
    uint8_t *g_fl = reinterpret_cast<uint8_t *>(g_pos + N);       // [N] bit 0 new, bit 1 old
    if (a.gib && GS) {
        for (int p = tid; p < N; p += NT) g_pos[a.perm[p]] = (uint16_t)p;  // positions < N hold sites
        sync();
    }
    // the source-array index of observation (s, f)
    auto cell_of = [&](int s, int f) -> int { return GS ? f * Np + (int)g_pos[s] : s * F + f; };
    // the observed state of (s, f) (S = NA)
    auto obs_of = [&](int s, int f) -> int { return stg ? lds_rd(lobs + s * F + f) : a.obs_sm[(size_t)s * F + f]; };
    // TB zone moves: the mixture log-likelihood of site s's F cells with zone class zc minus with
    // zone class zo (sum log sum_k l_k w_k, the same operations as the posterior's normaliser).
    // With every source resampled, ll_new - ll - (log q_s - log q_back_s) of the reference's
    // ratio is exactly this sum over the moved sites: the sources' terms cancel.
    auto site_mix_delta = [&](int s, int zc, int zo) -> double {
        LogAcc an, ao;
        for (int f = tid; f < F; f += NT) {
            const int x = obs_of(s, f);
            double l[3], wn[3];
            terms_z(s, f, x, zc, l, wn);
            double v = l[0] * wn[0] + l[1] * wn[1];
            if (C == 3) v = v + l[2] * wn[2];
            an.add(v);
            terms_z(s, f, x, zo, l, wn);
            v = l[0] * wn[0] + l[1] * wn[1];
            if (C == 3) v = v + l[2] * wn[2];
            ao.add(v);
        }
        return bsum(an.value() - ao.value());
    };
    // the n sites of the list, compacted in ascending order by `keep` (wave 0 writes; every wave
    // gets the count).  Reads of a chunk precede its writes, so the compaction may be in place.
    auto compact = [&](int n, auto &&site_at, auto &&keep) -> int {
        int kept = 0;
        for (int k0 = 0; k0 < n; k0 += WAVE) {
            const int k = k0 + lane;
            const int st = k < n ? site_at(k) : 0;
            const bool in = k < n && keep(k, st);
            const uint64_t m = __ballot(in);
            if (wv == 0 && in) g_lst[kept + lane_prefix(m)] = (uint16_t)st;
            kept += __popcll(m);
        }
        sync();
        return uni(kept);
    };

    // TB: the chain's count table from its current sources (one pass per launch)
    if constexpr (TB) (void)tpass(std::integral_constant<int, 1>(), src, nullptr, ct_cur);

    bool broken = false;
    for (int step = 0; step < a.n_steps; step++) {
        if (rng.bad || broken) break;
        const uint64_t sst = SBZ_TB_STAMP ? __builtin_amdgcn_s_memtime() : 0;  // step start (stamp builds)
        // rng.op with the CDF in LDS: numpy choice(p), the number of cdf entries <= u
        int op;
        if (rng.tape) {
            op = uni((int)rng.tape_item());
        } else {
            const double u = rng.uniform53();
            int i = 0;
#pragma unroll
            for (int k = 0; k < SBZ_N_OPS - 1; k++) i += (k < a.nops - 1 && !(u < cdf3[k])) ? 1 : 0;
            op = uni(i);
        }
        const bool zone_op = op <= SWAP;
        if (!(zone_op || op == GIBBSISH || (op >= G_SOURCES && op <= G_P_FAMILIES)) ||
            ((zone_op || op == GIBBSISH) && Z == 0) ||
            (op == G_P_ZONES && Z == 0) || (op == G_P_FAMILIES && (C == 2 || Fam == 0))) {
            broken = true;
            break;
        }
        double log_q = -INFINITY, log_q_back = 0.0;  // Gibbs operators: Q_GIBBS, Q_BACK_GIBBS
        double dprior = 0.0, ll_new = ll;
        int sa = -1, zoa = NONE, zna = NONE, sb = -1;
        bool new_sources = false;
        double geo_new = geo_cur;
        // gibbsish_sample_zones: zone gz, gn sites in g_lst, proposed size; gtent: zos holds the
        // proposal (undone on rejection)
        bool gtent = false;
        int gz = 0, gn = 0, gsize = 0, gdocc = 0;
        // TB zone move: the proposal's q, q_back and the moved sites' mixture delta
        bool tb_zone = false, tb_defer = false;
        double tb_q = 0.0, tb_qb = 0.0, tb_ds = 0.0;

        if (zone_op) {
            // ---- zone move with source resampling
            double log_q_back_s = 0.0;
            if constexpr (!TB) log_q_back_s = pass_logq();
            log_q = 0.0;
            log_q_back = -INFINITY;
            const int n_free = N - occupied;
            const int z = rng.below(Z);
            if (z < 0 || z >= Z) {
                broken = true;
                break;
            }
            const int size = uni(zsize[z]);
            double q = 0.0, q_back = 0.0;
            if (op == GROW || op == SWAP) {
                if (op == SWAP || size < max_size) {
                    mark(z);
                    const bool connected = rng.real() < p_grow;
                    const int n_nb = count_sel(SEL_NB, 0);
                    const int cnt_c = connected ? n_nb : n_free;
                    if (cnt_c > 0) {
                        const int site = kth_sel(connected ? SEL_NB : SEL_FREE, 0, rng.below(cnt_c));
                        int site_rm = -2;
                        if (op == SWAP) site_rm = kth_sel(SEL_ZONE, z, rng.below(size));
                        if (site < 0 || site_rm == -1) {
                            broken = true;
                            break;
                        }
                        q = (1.0 - p_grow) * (1.0 / (double)n_free);
                        if (is_nb(site)) q += p_grow * (1.0 / (double)n_nb);
                        if (op == GROW) {
                            q_back = 1.0 / (double)(size + 1);
                            dprior = uni(size_prior_delta(a.size_prior, N, size, size + 1));
                        } else {
                            q_back = (1.0 - p_grow) * (1.0 / (double)n_free);
                            if (is_nb(site_rm)) q_back += p_grow * (1.0 / (double)n_nb);
                            sb = site_rm;
                        }
                        sa = site;
                        zoa = NONE;
                        zna = z;
                    }
                }
            } else if (size > a.min_size) {  // SHRINK
                const int site = kth_sel(SEL_ZONE, z, rng.below(size));
                if (site < 0) {
                    broken = true;
                    break;
                }
                sync();
                if (tid == 0) zos[site] = NONE;
                sync();
                mark(z);
                const int n_back = count_sel(SEL_NB, 0);
                q_back = (1.0 - p_grow) * (1.0 / (double)(n_free + 1));
                if (is_nb(site)) q_back += p_grow * (1.0 / (double)n_back);
                if (a.warmup) q_back = 1.0 / (double)(size + 1);  // zone_sampling.py:1561
                sync();
                if (tid == 0) zos[site] = (uint8_t)z;
                sync();
                q = 1.0 / (double)size;
                dprior = uni(size_prior_delta(a.size_prior, N, size, size - 1));
                sa = site;
                zoa = z;
                zna = NONE;
            }
            if (sa >= 0) {
                // the new zones (tentatively, undone on rejection), then every source redrawn
                sync();
                if (tid == 0) {
                    zos[sa] = (uint8_t)zna;
                    if (sb >= 0) zos[sb] = NONE;
                }
                sync();
                if (a.geo_cost && (zna == Z - 1 || zoa == Z - 1)) {  // the last zone changed
                    geo_new = geo_prior();
                    dprior = uni(dprior + (geo_new - geo_cur));
                }
                if constexpr (TB) {
                    // tape: the reference's order (every source redrawn, then the acceptance
                    // uniform); Philox: the ratio does not depend on the new sources, so they are
                    // drawn only once the move is accepted
                    if (rng.tape) ll_new = tresample(ct_alt);
                    else tb_defer = true;
                    double ds = site_mix_delta(sa, zna, zoa);
                    if (sb >= 0) ds = ds + site_mix_delta(sb, NONE, zna);
                    tb_zone = true;
                    tb_q = q;
                    tb_qb = q_back;
                    tb_ds = uni(ds);
                } else {
                    double log_q_s;
                    pass_resample(log_q_s, ll_new);
                    log_q = a.warmup ? -INFINITY : uni(log(q) + log_q_s);
                    log_q_back = uni(log(q_back) + log_q_back_s);
                }
                new_sources = true;
            }
        } else if (op == GIBBSISH) {
            // ---- gibbsish_sample_zones (zone_sampling.py:619-702), as the SAMPLE_SOURCE = false
            // kernel (sbz_mh.hip) plus the sources of the available sites: log q_back gains their
            // current posterior terms, their sources are redrawn from the new sample's posterior
            // (gibbs_sample_sources(site_subset=available)) and log q gains those terms
            log_q = 0.0;
            log_q_back = -INFINITY;
            const int z = rng.below(Z);
            if (z < 0 || z >= Z) {
                broken = true;
                break;
            }
            gz = z;
            auto take = [&](int n) -> int64_t {  // n tape items / one Philox slot (uniform)
                const int64_t p0 = rng.pos;
                if (rng.tape) {
                    if (p0 + n > rng.len) rng.bad = 1;
                    rng.pos = uni64(min(p0 + n, rng.len));
                }
                return p0;
            };
            auto site_u = [&](int64_t p0, uint64_t slot, int k) {
                return rng.tape ? rng.tape[p0 + k] : site_uniform(rng.key0, rng.key1, rng.chain, slot, (uint32_t)k);
            };
            const int size = uni(zsize[z]);
            int n = compact(N, [&](int k) { return k; }, [&](int, int st) { return zos[st] == NONE || zos[st] == z; });
            if (n > 100) {  // available[available] &= np.random.random(n) < (100 / n)
                const double thr = 100.0 / (double)n;
                const int64_t p0 = take(n);
                const uint64_t slot = rng.ctr;
                if (!rng.tape) rng.ctr++;
                if (rng.bad) break;
                n = compact(n, [&](int k) { return (int)g_lst[k]; }, [&](int k, int) { return site_u(p0, slot, k) < thr; });
            }
            gn = n;
            if (n > 0) {
                const int nc = n * F;  // the available sites' observations, C order (site, feature)
                // log q_back_s: the current sources' posterior terms (zone_sampling.py:638-643)
                double log_q_back_s;
                {
                    ensure_staged();
                    LogAcc acc;
                    for (int c = tid; c < nc; c += NT) {
                        const int k = c / F, f = c - k * F, st = g_lst[k];
                        double l[3], wn[3], p[3];
                        terms(st, f, obs_of(st, f), l, wn);
                        posterior_draw<C>(l, wn, 2.0, p);
                        acc.add(p[rsrc(src, cell_of(st, f))]);
                    }
                    log_q_back_s = bsum(acc.value());
                }
                // each site's log marginal likelihood with zone z and without (:644-665): one wave
                // per site, the cells of the mixture (sum_c lh * w)
                for (int k = wv; k < n; k += NW) {
                    const int st = g_lst[k];
                    LogAcc aw, ao;
                    for (int f = lane; f < F; f += WAVE) {
                        const int x = obs_of(st, f);
                        double l[3], wn[3];
                        terms_z(st, f, x, z, l, wn);
                        double v = l[0] * wn[0] + l[1] * wn[1];
                        if (C == 3) v = v + l[2] * wn[2];
                        aw.add(v);
                        terms_z(st, f, x, NONE, l, wn);
                        v = l[0] * wn[0] + l[1] * wn[1];
                        if (C == 3) v = v + l[2] * wn[2];
                        ao.add(v);
                    }
                    const double lw = wave_sum(aw.value()), lwo = wave_sum(ao.value());
                    if (lane == 0) {
                        g_lw[k] = lw;
                        g_lwo[k] = lwo;
                    }
                }
                sync();
                const int64_t p1 = take(n);  // new_zone = np.random.random(n) < posterior_zone
                const uint64_t slot = rng.ctr;
                if (!rng.tape) rng.ctr++;
                if (rng.bad) break;
                double lq = 0.0, lqb = 0.0, n_new = 0.0, n_old = 0.0, n_zero = 0.0;
                for (int k = tid; k < n; k += NT) {
                    const double mw = exp(g_lw[k]), mo = exp(g_lwo[k]);
                    const double post = mw / (mw + mo);
                    const bool nz = site_u(p1, slot, k) < post;
                    const bool oz = zos[g_lst[k]] == (uint8_t)z;
                    const double fn = nz ? 1.0 : 0.0, fo = oz ? 1.0 : 0.0;
                    const double q = post * fn + (1.0 - post) * (1.0 - fn);
                    const double qb = post * fo + (1.0 - post) * (1.0 - fo);
                    lq += log(q);
                    lqb += log(qb);
                    n_zero += qb == 0.0 ? 1.0 : 0.0;
                    n_new += fn;
                    n_old += fo;
                    g_fl[k] = (uint8_t)((nz ? 1 : 0) | (oz ? 2 : 0));
                }
                const double LQ = bsum(lq), LQB = bsum(lqb);
                const int nn = (int)bsum(n_new), no = (int)bsum(n_old), nzb = (int)bsum(n_zero);
                gsize = size - no + nn;
                gdocc = nn - no;
                if (a.min_size <= gsize && gsize <= max_size && nzb == 0) {
                    if (a.size_prior == 1) {  // -log C(N, size) per zone: one site at a time
                        double dp = 0.0;
                        for (int sz = size; sz != gsize; sz += gsize > sz ? 1 : -1)
                            dp += size_prior_delta(1, N, sz, sz + (gsize > sz ? 1 : -1));
                        dprior = uni(dp);
                    } else {
                        dprior = uni(size_prior_delta(a.size_prior, N, size, gsize));
                    }
                    // the proposed zone (tentatively), every source into the candidate array
                    for (int k = tid; k < n; k += NT) zos[g_lst[k]] = (g_fl[k] & 1) ? (uint8_t)z : (uint8_t)NONE;
                    for (int c = tid; c < (GS ? (int)NFP : NF); c += NT) wsrc(srcb, c, rsrc(src, c));
                    sync();
                    gtent = true;
                    if (a.geo_cost && z == Z - 1) {
                        geo_new = geo_prior();
                        dprior = uni(dprior + (geo_new - geo_cur));
                    }
                    // gibbs_sample_sources(sample_new, as_gibbs=False, site_subset=available):
                    // one uniform per available observation in C order
                    double log_q_s;
                    {
                        LaneRng lr;
                        lr.initw(rng, tid);
                        LogAcc acc;
                        const int64_t p2 = rng.pos;
                        const bool have = !rng.tape || p2 + nc <= rng.len;
                        for (int c = tid; c < nc; c += NT) {
                            const int k = c / F, f = c - k * F, st = g_lst[k];
                            double l[3], wn[3], p[3];
                            terms(st, f, obs_of(st, f), l, wn);
                            const double u = rng.tape ? (have ? rng.tape[p2 + c] : 0.0) : lr.u();
                            const int kk = posterior_draw<C>(l, wn, u, p);
                            wsrc(srcb, cell_of(st, f), kk);
                            acc.add(p[kk]);
                        }
                        if (rng.tape) {
                            if (!have) rng.bad = 1;
                            rng.pos = uni64(p2 + nc);
                        } else {
                            rng.ctr++;
                        }
                        log_q_s = bsum(acc.value());
                    }
                    sync();
                    if constexpr (TB) ll_new = tpass(std::integral_constant<int, 1>(), srcb, nullptr, ct_alt);
                    else ll_new = pass_ll(srcb);
                    new_sources = true;
                    // ZoneMCMCWarmup.gibbs_sample_sources returns Q_GIBBS = -inf (:1293-1296)
                    log_q = a.warmup ? -INFINITY : uni(LQ + log_q_s);
                    log_q_back = uni(LQB + log_q_back_s);
                }
            }
        } else if (op == G_SOURCES) {
            if constexpr (TB) {
                ll_new = tresample(ct_alt);
            } else {
                double log_q_s;
                pass_resample(log_q_s, ll_new);
            }
            new_sources = true;
        } else if (op == G_WEIGHTS) {
            // (SBZ_TB_STAMP builds: cycles of the counts + gammas [14], of the whole operator [15])
            const uint64_t wst = SBZ_TB_STAMP ? __builtin_amdgcn_s_memtime() : 0;
            // source counts per feature over the sites of a zone (or of a family)
            const int fixed = C == 3 ? rng.below(2) : 0;  // random.choice(['inheritance', 'contact'])
            if (fixed < 0 || fixed > 1) {
                broken = true;
                break;
            }
            if constexpr (TB) {
                // from the count table's class counters [h][k]: zoned sites are h = 1, 3, sites
                // with a family h = 2, 3
                for (int f = tid; f < F; f += NT) {
                    const int *wc = ct_cur + (size_t)f * td.CTP + td.WOFF;
                    const int h1 = (C == 2 || fixed == 0) ? 1 : 2;
                    int a3[3], b3[3];
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        a3[k] = ldi(wc + h1 * 3 + k);
                        b3[k] = ldi(wc + 9 + k);
                    }
#pragma unroll
                    for (int k = 0; k < C; k++) cnt[f * C + k] = a3[k] + b3[k];
                }
            } else {
                clear_cnt();
                for_cells([&](int s, int f, int, int g, int) {
                    const bool in = (C == 2 || fixed == 0) ? zos[s] < Z : (stg ? lds_rd(lfam + s) : a.fam_site[s]) > 0;
                    if (in) atomicAdd(&cnt[f * C + rsrc(src, g)], 1);
                });
            }
            sync();
            const int64_t pos0 = rng.pos;
            const int64_t need = 2LL * F;  // C == 2: F pairs; C == 3: F beta draws + F uniforms
            const bool have = !rng.tape || pos0 + need <= rng.len;
            if (!rng.tape) {
                // Philox: the 2F gammas in parallel, thread t -> feature t / 2, gamma t % 2 (C == 2:
                // g0 / g1 of Dirichlet(1 + counts); C == 3: ga / gb of the Beta ratio), into gbuf
                // (gamma_fill: item t's alpha, then the gammas; stream of counter ctr, tag 0xFFF)
                for (int t = tid; t < 2 * F; t += NT) {
                    const int f = t >> 1, k = t & 1;
                    const int cc = C == 2 ? cnt[f * C + k]
                                          : (k == 0 ? cnt[f * C + (fixed == 0 ? 1 : 2)] : cnt[f * C]);
                    gbuf[t] = 1.0 + cc;
                }
                gamma_fill<SBZ_RB_WEIGHTS, NT>((lds_ptr<double>)gbuf, 2 * F, 1, (lds_ptr<const int>)nullptr,
                                               rng.key0, rng.key1, (uint32_t)rng.chain, rng.ctr, 1);
                sync();
                if (SBZ_TB_STAMP) tbst[14] += __builtin_amdgcn_s_memtime() - wst;
            }
            double wdl = 0.0;  // TB: the log-likelihood change from the class counters
            int wzf = 0;
            for (int f = tid; f < F; f += NT) {
                double *wf = w + (size_t)f * C;
                double o[3] = {ldp(wf), ldp(wf + 1), C == 3 ? ldp(wf + 2) : 0.0}, n[3] = {0.0, 0.0, 0.0};
                // TB: the feature's 12 class counters, loaded with the old weights
                int wcv[12];
                if constexpr (TB) {
                    const int *wc = ct_cur + (size_t)f * td.CTP + td.WOFF;
#pragma unroll
                    for (int i = 0; i < 12; i++) wcv[i] = ldi(wc + i);
                }
                if (C == 2) {
                    double d0, d1;
                    if (rng.tape) {
                        d0 = have ? rng.tape[pos0 + 2 * f] : 0.5;
                        d1 = have ? rng.tape[pos0 + 2 * f + 1] : 0.5;
                    } else {
                        const double g0 = gbuf[2 * f], g1 = gbuf[2 * f + 1];
                        d0 = g0 / (g0 + g1);
                        d1 = g1 / (g0 + g1);
                    }
                    stp(wf, d0);
                    stp(wf + 1, d1);
                    if (stg) stage_nw(f, d0, d1, 0.0);
                    n[0] = d0;
                    n[1] = d1;
                } else {
                    double r;
                    if (rng.tape) {
                        r = have ? rng.tape[pos0 + f] : 0.5;
                    } else {
                        const double ga = gbuf[2 * f], gb = gbuf[2 * f + 1];
                        r = ga / (ga + gb);
                    }
                    double w0 = o[0], w1 = o[1], w2 = o[2];
                    if (fixed == 0) w1 = r * w0 / (1.0 - r);
                    else w2 = r * w0 / (1.0 - r);
                    const double sum = (w0 + w1) + w2;
                    stp(wf, w0 / sum);
                    stp(wf + 1, w1 / sum);
                    stp(wf + 2, w2 / sum);
                    if (stg) stage_nw(f, w0 / sum, w1 / sum, w2 / sum);
                    n[0] = w0 / sum;
                    n[1] = w1 / sum;
                    n[2] = w2 / sum;
                }
                if constexpr (TB) {
                    // sum over classes h and components k of count * (log w_norm new - log w_norm old)
                    // log(wn / wo) = log(n_k / o_k) + log(so_h / sn_h): 3 + 4 logs per feature
                    double lk[3];
                    bool okk[3];
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        okk[k] = k < C && o[k] > 0.0 && n[k] > 0.0 && o[k] < INFINITY && n[k] < INFINITY;
                        lk[k] = okk[k] ? flog(n[k] / o[k]) : 0.0;
                    }
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        const double on1 = o[1] * ((h & 1) ? 1.0 : 0.0), nn1 = n[1] * ((h & 1) ? 1.0 : 0.0);
                        const double on2 = C == 3 ? o[2] * ((h & 2) ? 1.0 : 0.0) : 0.0;
                        const double nn2 = C == 3 ? n[2] * ((h & 2) ? 1.0 : 0.0) : 0.0;
                        double so = o[0] * 1.0 + on1, sn = n[0] * 1.0 + nn1;
                        if (C == 3) {
                            so = so + on2;
                            sn = sn + nn2;
                        }
                        const bool oks = so > 0.0 && sn > 0.0 && so < INFINITY && sn < INFINITY;
                        const double lh = oks ? flog(so / sn) : 0.0;
#pragma unroll
                        for (int k = 0; k < C; k++) {
                            const int c = wcv[h * 3 + k];
                            if (c <= 0) continue;
                            const bool present = k == 0 || (k == 1 ? (h & 1) != 0 : (h & 2) != 0);
                            if (present && okk[k] && oks) wdl += (double)c * (lk[k] + lh);
                            else wzf = 1;
                        }
                    }
                }
            }
            if (rng.tape) {
                if (!have) rng.bad = 1;
                rng.pos = uni64(pos0 + need);
            } else {
                rng.ctr++;
            }
            gsync();  // the new weights are visible to every thread (and their staged forms)
            if constexpr (TB) {
                const double d = bsum(wdl);
                ll_new = (bor(wzf) || !(ll > -INFINITY && ll < INFINITY))
                             ? tpass(std::integral_constant<int, 1>(), src, nullptr, ct_alt)
                             : uni(ll + d);
                if (SBZ_TB_STAMP) tbst[15] += __builtin_amdgcn_s_memtime() - wst;
            } else {
                ll_new = pass_ll(src);
            }
        } else {
            // ---- gibbs_sample_p_global / p_zones / p_families
            // (SBZ_TB_STAMP builds: cycles of the subset + counts, redraw_rows and the ll update)
            uint64_t gst = SBZ_TB_STAMP ? __builtin_amdgcn_s_memtime() : 0;
            if (SBZ_TB_STAMP) tbst[13] += gst - sst;
            auto gstamp = [&](int k) {
                if (SBZ_TB_STAMP) {
                    const uint64_t t = __builtin_amdgcn_s_memtime();
                    tbst[k] += t - gst;
                    gst = t;
                }
            };
            int row = 0;
            if (op == G_P_ZONES) row = rng.below(Z);        // np.random.randint(0, n_zones)
            if (op == G_P_FAMILIES) row = rng.below(Fam);   // np.random.randint(0, n_families)
            if (row < 0 || (op == G_P_ZONES && row >= Z) || (op == G_P_FAMILIES && row >= Fam)) {
                broken = true;
                break;
            }
            if (op == G_P_ZONES) {
                for (int f = tid; f < F; f += NT) sub[f] = 1;
                sync();
            } else {
                draw_subset();
            }
            const int comp = op == G_P_GLOBAL ? 0 : (op == G_P_ZONES ? 1 : 2);
            if constexpr (TB) {
                // the count table's row of this component: p_global [S], p_zones [row][S],
                // p_families [row][S] per feature (subset features only)
                // (four items per thread in flight: the loads first, unconditional, then the stores)
                const int off = comp == 0 ? 0 : (comp == 1 ? S + row * S : S * (1 + Z) + row * S);
                for (int i0 = tid; i0 < FS; i0 += 4 * NT) {
                    int v[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int i = min(i0 + u * NT, FS - 1), f = i / S, x = i - f * S;
                        v[u] = ldi(ct_cur + (size_t)f * td.CTP + off + x);
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int i = i0 + u * NT;
                        if (i < FS) cnt[i] = sub[i / S] ? v[u] : 0;
                    }
                }
            } else {
                clear_cnt();
                for_cells([&](int s, int f, int x, int g, int) {
                    bool in = sub[f] && rsrc(src, g) == comp && x < S;
                    if (comp == 1) in = in && zos[s] == row;
                    if (comp == 2) in = in && (stg ? lds_rd(lfam + s) : a.fam_site[s]) == row + 1;
                    if (in) atomicAdd(&cnt[f * S + x], 1);
                });
            }
            sync();
            double *base = comp == 0 ? pg : (comp == 1 ? pz + (size_t)row * F * S : pf + (size_t)row * F * S);
            int64_t rpos = rng.pos;
            uint64_t rctr = rng.ctr;
            int rbad = 0;
            // (an LDS address, used only when the parameters are staged)
            double *lbase = comp == 0 ? lpg : (comp == 1 ? lpz + (size_t)row * F * S : lpf + (size_t)row * F * S);
            double dll = 0.0;
            int dzf = 0;
            gstamp(5);
            dprior = redraw_rows(base, lbase, comp, row, rng.tape, rng.len, rng.key0, rng.key1, rng.chain,
                                 rpos, rctr, rbad, true, dll, dzf);
            gstamp(6);
            rng.pos = rpos;
            rng.ctr = rctr;
            if (rbad) rng.bad = 1;
            // the new rows are visible to every thread (the staged copies; the global rows too
            // before the parameters are staged)
            if (stg && stg_ok) sync();
            else gsync();
            if constexpr (TB) {
                ll_new = (dzf || !(ll > -INFINITY && ll < INFINITY))
                             ? tpass(std::integral_constant<int, 1>(), src, nullptr, ct_alt)
                             : uni(ll + dll);
                gstamp(7);
            } else {
                // the change from the row's source counts (cnt, as the table kernel's count table)
                ll_new = (dzf || !(ll > -INFINITY && ll < INFINITY)) ? pass_ll(src) : uni(ll + dll);
            }
        }

        // ---- metropolis_hastings_ratio (mcmc_generative.py:307-318)
        bool accept;
        if (tb_zone) {
            // TB zone move: log q_back = -inf when q_back is 0 or a current source has posterior 0
            // (then ll = -inf); log q = -inf (accepted) in the warm-up, when q is 0, or when a new
            // source landed on a zero-posterior component (ll_new = -inf beside a finite mixture
            // delta; an all-zero moved cell is a 0/0 posterior, NaN in the reference: rejected
            // after the uniform); otherwise the ratio with the sources' terms cancelled
            // (a Philox draw picks only components with a positive term, so there a new source
            // never lands on a zero-posterior one)
            if (tb_qb == 0.0 || !(ll > -INFINITY)) accept = false;
            else if (a.warmup || tb_q == 0.0 ||
                     (!tb_defer && ll_new == -INFINITY && tb_ds > -INFINITY && tb_ds < INFINITY))
                accept = true;
            else accept = flog(rng.real()) < (log(tb_qb) - log(tb_q)) + tb_ds + dprior;
            if (accept && tb_defer) ll_new = tresample(ct_alt);
        } else if (log_q_back == -INFINITY) accept = false;
        else if (log_q == -INFINITY) accept = true;
        else accept = flog(rng.real()) < ((ll_new - ll) * 1.0) - (log_q - log_q_back) + dprior;
        if (tid == 0) stat[op]++;
        if (accept) {
            if (tid == 0) stat[SBZ_N_OPS + op]++;
            ll = ll_new;
            prior = prior + dprior;
            geo_cur = geo_new;
            if (new_sources) {
                if constexpr (TB) {  // the candidate sources and their counts become current
                    uint8_t *t = src;
                    src = srcb;
                    srcb = t;
                    int *c = ct_cur;
                    ct_cur = ct_alt;
                    ct_alt = c;
                } else {
                    commit_sources();
                }
            }
            if (sa >= 0) {
                if (tid == 0) {
                    if (zoa < Z) zsize[zoa]--;
                    if (zna < Z) zsize[zna]++;
                    if (sb >= 0) zsize[zna]--;
                }
                occupied += (zna < Z ? 1 : -1) + (sb >= 0 ? -1 : 0);
                sync();
            }
            if (gtent) {
                if (tid == 0) zsize[gz] = gsize;
                occupied += gdocc;
                sync();
            }
        } else if (gtent) {  // undo the proposed zone
            for (int k = tid; k < gn; k += NT) zos[g_lst[k]] = (g_fl[k] & 2) ? (uint8_t)gz : (uint8_t)NONE;
            sync();
        } else if (sa >= 0) {
            sync();
            if (tid == 0) {  // undo the tentative zone change
                zos[sa] = (uint8_t)zoa;
                if (sb >= 0) zos[sb] = (uint8_t)zna;
            }
            sync();
        }
        if (alias && accept && op != G_SOURCES && op != G_P_GLOBAL && op != G_P_ZONES &&
            op != G_P_FAMILIES) {
            gsync();  // every thread's parameter stores have landed
            // this accept replaces the reference's Sample object: the arrays of the logged
            // sample stop changing here (sbz.h, alias_pending)
            const size_t fs = (size_t)F * S;
            for (size_t k = tid; k < fs; k += NT) ch.alias_p_global[b * fs + k] = ldp(pg + k);
            for (size_t k = tid; k < (size_t)Z * fs; k += NT)
                ch.alias_p_zones[b * Z * fs + k] = ldp(pz + k);
            if (C == 3)
                for (size_t k = tid; k < (size_t)Fam * fs; k += NT)
                    ch.alias_p_fam[b * Fam * fs + k] = ldp(pf + k);
            alias = 0;
        }
        if (ch.trace_op && tid == 0) {
            const size_t t = (size_t)b * a.n_steps + step;
            ch.trace_op[t] = (int8_t)op;
            ch.trace_accept[t] = accept ? 1 : 0;
            ch.trace_ll[t] = ll;
        }

        if (ch.trace_zos) {
            uint8_t *tz = ch.trace_zos + ((size_t)b * a.n_steps + step) * N;
            for (int s = tid; s < N; s += NT) tz[s] = zos[s];
        }
        if (bor(err)) break;  // an out-of-range index (reported below)
        if (SBZ_TB_STAMP && op >= G_P_GLOBAL && op <= G_P_FAMILIES) tbst[12] += __builtin_amdgcn_s_memtime() - sst;
    }

    sync();
    for (int s = tid; s < N; s += NT) gzos[s] = zos[s];
    if (TB && src != gsrc) {  // the current sources are the scratch row: back into the chain's array
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(src);
        uint32_t *d32 = reinterpret_cast<uint32_t *>(gsrc);
        for (int i = tid; i < (int)(NFP / 4); i += NT)
            __hip_atomic_store(d32 + i, __hip_atomic_load(s32 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!GS) {
        if (a.src_pm) {  // back to [F][Np] by position (padding positions untouched)
            for (int i = tid; i < (int)NFP; i += NT) {
                const int f = i / Np, p = i - f * Np;
                if (p < N) gsrc[i] = src[a.perm[p] * F + f];
            }
        } else {
            for (int c = tid; c < NF; c += NT) gsrc[c] = src[c];
        }
    }
    if (SBZ_TB_STAMP && ch.trace_ll && a.n_steps >= 32 && (tid == 0 || tid == NT - 64)) {
        for (int k = 0; k < 16; k++) ch.trace_ll[(size_t)b * a.n_steps + (tid ? 16 : 0) + k] = (double)tbst[k];
    }
    if (tid == 0) {
        ch.ll[b] = ll;
        if (ch.prior) ch.prior[b] = prior;
        if (ch.alias_pending) ch.alias_pending[b] = alias;
        if (ch.tape_pos) ch.tape_pos[b] = rng.pos;
        if (ch.counter) ch.counter[b] = rng.ctr;
        if (ch.status) ch.status[b] = broken ? 2 : (rng.bad ? 1 : 0);
    }
    if (tid < SBZ_N_OPS) {  // per-operator counters, one thread each
        if (ch.accepted) ch.accepted[(size_t)b * SBZ_N_OPS + tid] += stat[SBZ_N_OPS + tid];
        if (ch.proposed) ch.proposed[(size_t)b * SBZ_N_OPS + tid] += stat[tid];
    }
    // an out-of-range index: the first faulting thread's code (status 16 + code)
    sync();
    if (tid == 0) redi[0] = 0;
    sync();
    if (err) atomicCAS(&redi[0], 0, err);
    sync();
    if (tid == 0 && redi[0] && ch.status) ch.status[b] = 16 + redi[0];
}

}  // namespace

int launch_mh_source(sbz_ctx *ctx, int B, const MhArgs &a0) {
    MhArgs a = a0;
    constexpr size_t LDS_MAX = 160 * 1024;
    const sbz_dims &d = ctx->d;
    const bool geo = a.geo_cost != nullptr;
    // gibbsish_sample_zones scratch (a non-zero weight): part of every placement decision below,
    // so a shape at the edge falls back to HBM sources / no staging instead of failing
    const size_t gib = a.gib ? 16 + (size_t)d.n_sites * 21 : 0;
    // waves per chain: 8 (SBZ_OPT_SRC_WAVES overrides: 1, 4 or 8).  8 waves = 2 per SIMD, so up to
    // 256 VGPRs: no spills.  Measured against 4 on the real-data shapes (tools/src_optime.py):
    // Balkan 12.4 -> 11.2 us per step, South America 18.0 -> 14.2.
    int nw = 8;
    if (ctx->src_waves == 1 || ctx->src_waves == 4 || ctx->src_waves == 8) nw = ctx->src_waves;
    const bool gs = ctx->src_hbm || mh_src_lds_bytes(d, ctx->C, false, geo, false) + gib > LDS_MAX;  // do not fit: HBM
    // sources in HBM: the feature-table passes and count tables where they apply (4 or 8 waves,
    // one source dword per thread and feature, the tables within LDS; SBZ_OPT_SRC_PASS_TABLES 0: off)
    const TbDims td = tb_dims(d.n_states, d.n_zones, d.n_families, ctx->C);
    const bool tb = gs && ctx->src_pass_tables && nw >= 4 && tb_fits(td, ctx->Np) &&
                    mh_src_lds_bytes(d, ctx->C, true, geo, false, true, ctx->Np, nw) + gib <= LDS_MAX;
    // parameters staged in LDS when they fit too (SBZ_OPT_SRC_STAGE 0: off; not with the table passes)
    a.stage = !tb && ctx->src_stage && mh_src_lds_bytes(d, ctx->C, gs, geo, true) + gib <= LDS_MAX ? 1 : 0;
    size_t lds = mh_src_lds_bytes(d, ctx->C, gs, geo, a.stage != 0, tb, ctx->Np, nw);
    // the constant tables too, when they fit beside the staged parameters or the table-pass region
    const size_t cst = mh_src_const_bytes(d, ctx->C, a.alpha_g != nullptr, a.alpha_f != nullptr,
                                          a.gc_g != nullptr, a.gc_f != nullptr);
    a.cstage = (a.stage || tb) && d.n_states <= 255 && lds + cst + gib <= LDS_MAX ? 1 : 0;
    if (a.cstage) lds += cst;
    if (a.gib) {  // gibbsish_sample_zones scratch at the end (16-B aligned)
        lds = (lds + 15) & ~(size_t)15;
        a.gib_off = (uint32_t)lds;
        lds += (size_t)d.n_sites * 21;
    }
    if (lds > LDS_MAX)
        return fail(ctx, SBZ_EINVAL, "SAMPLE_SOURCE sampler needs " + std::to_string(lds) +
                                         " B of LDS per chain even with the sources in HBM (> 160 KiB)");
    const size_t nfp = (size_t)d.n_features * ctx->Np;
    // the chain's sources: position-major as given, or (site-major) copied in / out by the kernel
    // (LDS) or transposed around the launch (HBM, whose passes walk them position-major)
    a.src_pm = a.ch.source_layout == SBZ_SOURCE_BY_POSITION ? 1 : 0;
    uint8_t *src_sm = nullptr;  // the caller's site-major array, transposed around an HBM launch
    if (gs) {
        int rc = ensure(ctx, ctx->src_cand, (size_t)B * nfp);
        if (rc) return rc;
        a.src_scratch = static_cast<uint8_t *>(ctx->src_cand.ptr);
        if (!a.src_pm) {
            rc = ensure(ctx, ctx->src_t, (size_t)B * nfp);
            if (rc) return rc;
            src_sm = a.ch.source;
            a.ch.source = static_cast<uint8_t *>(ctx->src_t.ptr);
            rc = launch_source_transpose(ctx, B, src_sm, a.ch.source, true);
            if (rc) return rc;
            a.src_pm = 1;
        }
    }
    if (tb) {  // count tables: current and candidate, [2][B][F][CTP] ints
        a.ct_half = (size_t)B * d.n_features * td.CTP;
        int rc = ensure(ctx, ctx->src_ctab, 2 * a.ct_half * sizeof(int));
        if (rc) return rc;
        a.ctab = static_cast<int *>(ctx->src_ctab.ptr);
    }
    static bool configured = false;
    if (!configured) {
        const void *fns[] = {
            reinterpret_cast<const void *>(&mh_src_kernel<2, false, 1>), reinterpret_cast<const void *>(&mh_src_kernel<3, false, 1>),
            reinterpret_cast<const void *>(&mh_src_kernel<2, true, 1>), reinterpret_cast<const void *>(&mh_src_kernel<3, true, 1>),
            reinterpret_cast<const void *>(&mh_src_kernel<2, false, 4>), reinterpret_cast<const void *>(&mh_src_kernel<3, false, 4>),
            reinterpret_cast<const void *>(&mh_src_kernel<2, true, 4>), reinterpret_cast<const void *>(&mh_src_kernel<3, true, 4>),
            reinterpret_cast<const void *>(&mh_src_kernel<2, false, 8>), reinterpret_cast<const void *>(&mh_src_kernel<3, false, 8>),
            reinterpret_cast<const void *>(&mh_src_kernel<2, true, 8>), reinterpret_cast<const void *>(&mh_src_kernel<3, true, 8>),
            reinterpret_cast<const void *>(&mh_src_kernel<2, true, 4, true>), reinterpret_cast<const void *>(&mh_src_kernel<3, true, 4, true>),
            reinterpret_cast<const void *>(&mh_src_kernel<2, true, 8, true>), reinterpret_cast<const void *>(&mh_src_kernel<3, true, 8, true>)};
        for (const void *fn : fns) {
            hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
            if (e != hipSuccess) return hip_fail(ctx, e, "hipFuncSetAttribute(sampler LDS)");
        }
        configured = true;
    }
    auto go = [&](auto cc, auto gsc, auto nwc, auto tbc) {
        constexpr int CC = decltype(cc)::value, NWC = decltype(nwc)::value;
        constexpr bool GSC = decltype(gsc)::value, TBC = decltype(tbc)::value;
        mh_src_kernel<CC, GSC, NWC, TBC><<<B, NWC * WAVE, lds, ctx->stream>>>(a);
    };
    auto by_nw = [&](auto cc, auto gsc) {
        if constexpr (decltype(gsc)::value) {
            if (tb) {
                if (nw == 4) go(cc, gsc, std::integral_constant<int, 4>(), std::true_type());
                else go(cc, gsc, std::integral_constant<int, 8>(), std::true_type());
                return;
            }
        }
        if (nw == 1) go(cc, gsc, std::integral_constant<int, 1>(), std::false_type());
        else if (nw == 4) go(cc, gsc, std::integral_constant<int, 4>(), std::false_type());
        else go(cc, gsc, std::integral_constant<int, 8>(), std::false_type());
    };
    auto by_gs = [&](auto cc) {
        if (gs) by_nw(cc, std::true_type());
        else by_nw(cc, std::false_type());
    };
    if (ctx->C == 3) by_gs(std::integral_constant<int, 3>());
    else by_gs(std::integral_constant<int, 2>());
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "source-mode sampler launch");
    ctx->last_kernels = std::string("mh_src_kernel") + (gs ? (tb ? "<hbm, tables>" : "<hbm>") : "<lds>");
    if (src_sm) return launch_source_transpose(ctx, B, a.ch.source, src_sm, false);
    return SBZ_OK;
}

}  // namespace sbz
