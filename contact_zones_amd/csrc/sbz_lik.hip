// sbz_lik.hip — batched full log-likelihood kernels for CDNA4 (gfx950).
//
// Computes, for each of B chains, the reference Likelihood.__call__(sample, caching=False)
// (sbayes/model.py:145-171):
//   mixture : sum_{s,f} log( (w0*l0 + w1*l1) + w2*l2 )          combine_lh  model.py:174-176
//   source  : sum_{s,f} log( w_src * l_src ), -inf on w_src == 0  combine_lh  model.py:177-184
// with l_c the one-hot gathers of p_global / p_zones / p_families (model.py:297-433), NA -> 1
// (model.py:247) and w_c = w[f,c]*has[s,c] / ((w0*h0 + w1*h1) + w2*h2) (model.py:436-452).
//
// Design — memory-bound gather-reduce, no MFMA, one wave per task:
//   * A task is (chain b, a contiguous range of features).  Tasks are single-wave workgroups,
//     so a CU holds up to 32 independent tasks and no block-wide barrier is ever waited on.
//   * Every cell value depends only on (site class, f, x), class = (zone or none) x (family or
//     none).  For each feature the wave builds a table T[class][x] (x = S is the NA column) in
//     its own few KB of LDS, in the reference's operation order (products, then the component
//     sum left to right; -ffp-contract=off), so every entry is bit-identical to the reference's
//     per-cell value.  The products n_c * l_c are formed once per (x, class part) and combined
//     with two adds per entry.
//   * The lane owns SPL sites (4*lane + 256*k + j); their class row offsets live in registers.
//     Observations are stored feature-major (obs_fm[f][site]) as byte offsets x*8, so a cell
//     is one v_add_u32 (row + byte), one ds_read_b64 and one v_mul_f64.
//   * Instead of one fp64 log per cell, the lane multiplies its cells into a mantissa/exponent
//     accumulator (v_frexp every 8 factors) and takes ONE log at the end:
//     sum log(c_i) = log(prod c_i) to ~1e-16 relative.  A table entry outside [2^-120, 2^120]
//     (or negative / NaN) switches the wave to renormalising after every factor for that
//     feature, so the product never under/overflows for any normal double.
//   * The next feature's parameters are loaded into registers before the current feature's
//     gathers, so the HBM stream overlaps the LDS/VALU work of up to 32 waves per CU.
//   * One fp64 partial per task; a tiny second kernel sums a chain's partials in task order
//     (deterministic, bit-reproducible).
#include <algorithm>
#include <cmath>
#include <vector>

#include "sbz_internal.h"

namespace sbz {

namespace {

constexpr double LN2 = 0.69314718055994530941723212145818;
constexpr int WAVE = 64;
constexpr int ZR = 2;  // zone classes per lane held in registers
constexpr int NW_BYTES = 16 * 8;  // nw[4][4] doubles ahead of the table

__device__ __forceinline__ bool safe_factor(double v) {
    return v == 0.0 || (v >= 0x1p-120 && v <= 0x1p120);
}

__device__ __forceinline__ void renorm(double &m, int &e) {
    const int ex = __builtin_amdgcn_frexp_exp(m);
    m = __builtin_amdgcn_frexp_mant(m);
    e += ex;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v |= __shfl_xor(v, off, 64);
    return v;
}

// Make this wave's LDS writes visible to its other lanes.  The workgroup is one wave, so no
// s_barrier is needed, and unlike __syncthreads() this does not drain the vector-memory
// counter: the next feature's prefetched loads stay in flight.
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// normalize_weights (model.py:451-452) for the 4 (has_zone, has_family) classes, lanes 0..3.
template <int C>
__device__ __forceinline__ void store_nw(double *nw, int lane, double w0r, double w1r, double w2r) {
    if (lane < 4) {
        const double hz = (lane & 1) ? 1.0 : 0.0, hf = (lane & 2) ? 1.0 : 0.0;
        const double w0 = w0r * 1.0, w1 = w1r * hz;
        double s = w0 + w1, w2 = 0.0;
        if (C == 3) {
            w2 = w2r * hf;
            s = s + w2;
        }
        nw[lane * 4 + 0] = w0 / s;
        nw[lane * 4 + 1] = w1 / s;
        nw[lane * 4 + 2] = (C == 3) ? w2 / s : 0.0;
    }
}

// ---------------------------------------------------------------------------------------
// Mixture kernel (table path).  Requires S + 1 <= 64, Z + 1 <= ZR * (64 / (S + 1)),
// Fam <= FR, (Z+1)(Fam+1) + 1 <= 256 and a per-feature slot of <= 4*64 doubles (checked on
// the host; otherwise lik_mixture_generic_kernel runs).
//
// A task is (chain b, features [fa, fb)).  LDS (bytes from the dynamic base):
//   [0, 128)   nw[4][4]: normalised weights of the 4 (has_zone, has_family) classes
//   slot       one feature's parameters, `per` doubles: p_global[f][0..S) | p_zones[z][f][0..S)
//              for z < Z | p_fam[fam][f][0..S) for fam < Fam | w[f][0..C)
//   table      T[ncls + 1][S1] doubles, class = zc*FamC + fc; the last row is neutral (1.0)
//   junk       64 doubles (table-build writes of lanes without an entry)
// Parameter pipeline: the loads of feature f+2 are issued (branch-free, 4 per lane) at the
// start of feature f into one of two register sets and written into the slot at the end of
// feature f+1, once its table has been built; HBM latency is covered by two features of work.
// Lane (lx = lane % S1, lg = lane / S1) builds the entries of state x = lx for the zone
// classes zc = lg + i*G, i < ZR (G = 64 / S1), every family class.
// ---------------------------------------------------------------------------------------
constexpr int PL = 4;  // slot doubles per lane (per <= 4 * 64)
#ifndef SBZ_ABLATE
#define SBZ_ABLATE 0  // diagnostic builds only: 1 = skip gathers, 2 = skip table build (wrong results)
#endif
#ifndef SBZ_MIX_WAVES
#define SBZ_MIX_WAVES 3  // launch bound: minimum waves per SIMD of the mixture table kernel
#endif

// A parameter or normalised weight is "tame" if it is 0 or in [2^-60, 2^60]: every table entry
// is then a sum of <= 3 products of tame values, i.e. 0 or in [2^-120, 3*2^120], and 8 such
// factors times a mantissa in [0.5, 1) stay in the normal range.  Otherwise (tiny / huge /
// negative / NaN inputs) the wave renormalises after every factor for that feature.
__device__ __forceinline__ bool tame(double v) { return v == 0.0 || (v >= 0x1p-60 && v <= 0x1p60); }

template <int C, int SPL, int FR, bool XS8>
__global__ __launch_bounds__(WAVE, SBZ_MIX_WAVES) void lik_mixture_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int NO = SPL / 4;  // observation words (4 sites each) per lane per feature
    double *nw = reinterpret_cast<double *>(lds);
    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    const int S = a.S, S1 = a.S + 1, FamC = a.FamC, Z = a.Z;
    const int Fam = (C == 3) ? a.Fam : 0;
    const int ncls = (Z + 1) * FamC;
    const int G = WAVE / S1;
    const int lx = lane % S1, lg = lane / S1;
    const bool na = lx == S;
    const int lxc = min(lx, S - 1);  // the NA column and idle lanes read state 0
    const int nps = (1 + Z + Fam) * S;  // parameter doubles of a slot (then C weights)
    const int per = nps + C;
    const uint32_t zfs = (uint32_t)(a.F * S);
    const double *pgb = a.pg + (size_t)b * zfs;
    const double *zbase = Z > 0 ? a.pz + (size_t)b * Z * zfs : pgb;
    const double *fbase = Fam > 0 ? a.pf + (size_t)b * Fam * zfs : pgb;
    const double *wb = a.w + (size_t)b * a.F * C;
    double *slot = nw + 16;
    double *tab = slot + ((per + 1) & ~1);
    double *junk = tab + (ncls + 1) * S1 + lane;
    const int row_bytes = S1 * 8;
    const int tab_off = (int)((tab - nw) * 8);

    // Per-lane source rows of the slot elements i = lane + 64k: element i of feature f is
    // sbase[k][f * sstride[k]] (p_global / p_zones / p_fam rows: stride S; weights: stride C).
    const double *sbase[PL];
    uint32_t sstride[PL];
#pragma unroll
    for (int k = 0; k < PL; k++) {
        const uint32_t ic = (uint32_t)min(lane + WAVE * k, per - 1);
        const uint32_t seg = (uint32_t)(((uint64_t)ic * a.s_magic) >> 32);  // ic / S
        const uint32_t r = ic - seg * (uint32_t)S;
        if (seg == 0) {
            sbase[k] = pgb + r;
            sstride[k] = (uint32_t)S;
        } else if (seg <= (uint32_t)Z) {
            sbase[k] = zbase + (size_t)(seg - 1) * zfs + r;
            sstride[k] = (uint32_t)S;
        } else if (seg < (uint32_t)(1 + Z + Fam)) {
            sbase[k] = fbase + (size_t)(seg - 1 - Z) * zfs + r;
            sstride[k] = (uint32_t)S;
        } else {
            sbase[k] = wb + (ic - (uint32_t)nps);
            sstride[k] = (uint32_t)C;
        }
    }
    auto load_slot = [&](int f, double (&r)[PL]) {
#pragma unroll
        for (int k = 0; k < PL; k++) r[k] = sbase[k][(uint32_t)f * sstride[k]];
    };
    // store the slot (branch-free: out-of-range elements go to the lane's junk word); returns
    // whether every stored value is tame
    auto store_slot = [&](const double (&r)[PL]) -> int {
        int ok = 1;
#pragma unroll
        for (int k = 0; k < PL; k++) {
            const bool in = lane + WAVE * k < per;
            *(in ? slot + lane + WAVE * k : junk) = r[k];
            ok &= (!in) | tame(r[k]);
        }
        return ok;
    };
    auto load_obs = [&](int f, int c0, uint32_t (&o)[NO]) {
        const uint32_t *op = reinterpret_cast<const uint32_t *>(a.obs_fm + (size_t)f * a.Np + c0);
#pragma unroll
        for (int k = 0; k < NO; k++) o[k] = op[lane + 64 * k];
    };

    for (int x = lane; x < S1; x += WAVE) tab[ncls * S1 + x] = 1.0;

    double m[4] = {1.0, 1.0, 1.0, 1.0};  // four independent product chains
    int e = 0;
    uint32_t base2[SPL / 2];  // per-site class row offsets (bytes, < 64 KiB), two per register
    uint32_t oa[NO], ob[NO];
    double ra[PL], rb[PL];
    int slot_ok = 1;  // the slot's values are tame

    // One feature.  `cur`: f's observations; `nxt` <- f+1's.  `fill` <- f+2's parameters;
    // `wr` holds f+1's parameters (issued during f-1), written to the slot at the end.
    // Every global load is unconditional (feature index clamped to fb-1): a load under a branch
    // makes the compiler's vmcnt bookkeeping conservative at the join, and the gathers of f would
    // then wait for f+1's observations.  `live` = false only for the padding feature of an odd
    // range, whose gathers are skipped (the skipped block issues no global loads).
    auto feature = [&](int f, int c0, bool live, uint32_t (&cur)[NO], uint32_t (&nxt)[NO],
                       double (&fill)[PL], double (&wr)[PL]) {
        wave_lds_sync();  // the slot holds feature f
        // 1. normalised weights, one division per lane: lane = h*3 + c (h = hz | hf<<1)
        //    normalize_weights model.py:451-452: w*has / ((w0*h0 + w1*h1) + w2*h2)
        int nok = 1;
        if (lane < 12) {
            const int h = lane / 3, c = lane - 3 * (lane / 3);
            const double hz = (h & 1) ? 1.0 : 0.0, hf = (h & 2) ? 1.0 : 0.0;
            const double w0 = slot[nps] * 1.0, w1 = slot[nps + 1] * hz;
            double sum = w0 + w1, w2 = 0.0;
            if (C == 3) {
                w2 = slot[nps + 2] * hf;
                sum = sum + w2;
            }
            const double wc = c == 0 ? w0 : (c == 1 ? w1 : w2);
            const double n = (C == 2 && c == 2) ? 0.0 : wc / sum;
            nw[h * 4 + c] = n;
            nok = tame(n);
        }
        const bool wide = __ballot(!(nok & slot_ok)) != 0;  // one v_cmp into an SGPR pair
        wave_lds_sync();
        // 2. table: the reference cell (n0*l0 + n1*l1) + n2*l2 for every class.  Branch-free:
        //    lanes without an entry write to their junk slot.
        const double l0 = na ? 1.0 : slot[lxc];
        const double lna = na ? 1.0 : 0.0;  // lh of a component the site lacks
#pragma unroll
        for (int i = 0; i < ZR; i++) {
#if SBZ_ABLATE & 2
            break;  // diagnostic build: skip the table build
#endif
            const int zc = lg + i * G;
            const bool valid = (lane < G * S1) && (zc <= Z);
            const int hz = zc > 0 ? 1 : 0;
            const double lzv = slot[min(zc, Z) * S + lxc];
            const double l1 = na ? 1.0 : (zc > 0 ? lzv : 0.0);
            const double *n0 = nw + hz * 4, *n1 = nw + (hz | 2) * 4;  // no family / family
            double *row = valid ? tab + (zc * FamC) * S1 + lx : junk;
            const int rs = valid ? S1 : 0;
            double v = n0[0] * l0 + n0[1] * l1;
            if (C == 3) v = v + n0[2] * lna;
            row[0] = v;
            if (C == 3) {
                const double a1 = n1[0] * l0 + n1[1] * l1;
#pragma unroll
                for (int fm = 0; fm < FR; fm++) {
                    if (fm < Fam) {
                        const double lf = slot[(1 + Z + fm) * S + lxc];
                        row[(fm + 1) * rs] = a1 + n1[2] * (na ? 1.0 : lf);
                    }
                }
            }
        }
        wave_lds_sync();
        __builtin_amdgcn_sched_barrier(0);
        // 3. issue the loads of f+2's parameters and f+1's observations
        load_slot(min(f + 2, fb - 1), fill);
        load_obs(min(f + 1, fb - 1), c0, nxt);
        // 4. gathers of feature f: cell (k, j) -> chain (k & 3)
        if (SBZ_ABLATE & 1 || !live) {
            // padding feature (or diagnostic build): no gathers
        } else if (!wide) {
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t bw = base2[2 * k + (j >> 1)];
                    const uint32_t bs = (j & 1) ? (bw >> 16) : (bw & 0xffffu);
                    const uint32_t xb = (cur[k] >> (8 * j)) & 0xffu;
                    const uint32_t addr = bs + (XS8 ? xb : (xb << 3));
                    m[k & 3] *= *reinterpret_cast<const double *>(lds + addr);
                    if (j == 3 && (k & 1)) __builtin_amdgcn_sched_barrier(0);  // <= 8 reads in flight
                }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (q < NO) renorm(m[q], e);
        } else {
            // untamed inputs: renormalise after every factor (exact for any normal double)
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t bw = base2[2 * k + (j >> 1)];
                    const uint32_t bs = (j & 1) ? (bw >> 16) : (bw & 0xffffu);
                    const uint32_t xb = (cur[k] >> (8 * j)) & 0xffu;
                    const uint32_t addr = bs + (XS8 ? xb : (xb << 3));
                    m[0] *= *reinterpret_cast<const double *>(lds + addr);
                    renorm(m[0], e);
                }
        }
        // 5. the table of f is built, so the slot can take f+1's parameters
        slot_ok = store_slot(wr);
    };

    for (int c0 = 0; c0 < a.Np; c0 += SPL * WAVE) {
        // classes of this chunk's sites, the first two features' parameters, f0's observations
        {
            const uint32_t *clw = reinterpret_cast<const uint32_t *>(a.cls + (size_t)b * a.Np + c0);
            uint32_t cw[NO];
#pragma unroll
            for (int k = 0; k < NO; k++) cw[k] = clw[lane + 64 * k];
            load_slot(fa, ra);
            load_slot(min(fa + 1, fb - 1), rb);
            load_obs(fa, c0, oa);
#pragma unroll
            for (int i = 0; i < SPL; i++) {
                const int cls = (cw[i / 4] >> (8 * (i % 4))) & 0xff;  // padded sites: neutral row
                const uint32_t off = (uint32_t)(tab_off + cls * row_bytes);
                if (i & 1) base2[i >> 1] |= off << 16;
                else base2[i >> 1] = off;
            }
            wave_lds_sync();  // previous chunk's gathers are done with the slot
            slot_ok = store_slot(ra);
        }
        for (int f = fa; f < fb; f += 2) {
            feature(f, c0, true, oa, ob, ra, rb);
            feature(f + 1, c0, f + 1 < fb, ob, oa, rb, ra);
        }
    }
    double v = (log(m[0]) + log(m[1])) + (log(m[2]) + log(m[3]));
    v = v + (double)e * LN2;
    const double tot = wave_sum(v);
    if (lane == 0) a.partial[(size_t)b * a.W + blockIdx.x] = tot;
}

// ---------------------------------------------------------------------------------------
// Mixture kernel, generic path (any S, Z, Fam within the ABI limits): one lane per site,
// cells computed directly from the parameters in the reference's operation order, one log
// per cell.  Used only when the table path's register layout does not apply.
// ---------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(WAVE) void lik_mixture_generic_kernel(LikArgs a) {
    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    const int S = a.S, Z = a.Z;
    const int Fam = (C == 3) ? a.Fam : 0;
    const size_t zfs = (size_t)a.F * S;
    const double *pgb = a.pg + (size_t)b * zfs;
    const double *pzb = a.pz + (size_t)b * Z * zfs;
    const double *pfb = (C == 3) ? a.pf + (size_t)b * Fam * zfs : nullptr;
    const double *wb = a.w + (size_t)b * a.F * C;
    const uint8_t *zb = a.zone + (size_t)b * a.N;
    const int div = a.xs8 ? 8 : 1;
    double lsum = 0.0;
    for (int s = lane; s < a.N; s += WAVE) {
        const int z = zb[s];
        const bool hz = z < Z;
        const int fc = (C == 3) ? a.famc[s] : 0;
        const bool hf = fc > 0;
        for (int f = fa; f < fb; f++) {
            const int x = a.obs_fm[(size_t)f * a.Np + s] / div;
            const bool na = x == S;
            const double w0 = wb[(size_t)f * C] * 1.0;
            const double w1 = wb[(size_t)f * C + 1] * (hz ? 1.0 : 0.0);
            double sum = w0 + w1, w2 = 0.0;
            if (C == 3) {
                w2 = wb[(size_t)f * C + 2] * (hf ? 1.0 : 0.0);
                sum = sum + w2;
            }
            const double l0 = na ? 1.0 : pgb[(size_t)f * S + x];
            const double l1 = na ? 1.0 : (hz ? pzb[(size_t)z * zfs + (size_t)f * S + x] : 0.0);
            double v = (w0 / sum) * l0 + (w1 / sum) * l1;
            if (C == 3) {
                const double l2 = na ? 1.0 : (hf ? pfb[(size_t)(fc - 1) * zfs + (size_t)f * S + x] : 0.0);
                v = v + (w2 / sum) * l2;
            }
            lsum += log(v);
        }
    }
    const double tot = wave_sum(lsum);
    if (lane == 0) a.partial[(size_t)b * a.W + blockIdx.x] = tot;
}

// ---------------------------------------------------------------------------------------
// Source kernel: cell = w_norm[src] * l_src.  Rows (each S1 doubles):
//   T0[h]            h = hz | hf<<1     w_norm[h][0] * l0                      rows 0..3
//   T1[z][hf]        has_zone           w_norm[1|hf<<1][1] * l1                rows 4..4+2Z-1
//   T2[fam][hz]      has_family         w_norm[hz|2][2] * l2                   rows 4+2Z..
//   Z0               selected component the site lacks: weight 0 -> cell 0 -> -inf
//   N1               neutral row (padded sites)
// Each lane packs its site's three row indices (r0 | r1<<8 | r2<<16); the cell's source
// byte selects one.
// ---------------------------------------------------------------------------------------
template <int C, int SPL>
__global__ __launch_bounds__(WAVE) void lik_source_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double *nw = reinterpret_cast<double *>(lds);
    double *tab = reinterpret_cast<double *>(lds + NW_BYTES);

    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    if (fa >= fb) {
        if (lane == 0) a.partial[(size_t)b * a.W + blockIdx.x] = 0.0;
        return;
    }
    const int S = a.S, S1 = a.S + 1, Z = a.Z;
    const int Fam = (C == 3) ? a.Fam : 0;
    const int off1 = 4, off2 = 4 + 2 * Z, rz = 4 + 2 * Z + 2 * Fam, rn = rz + 1;
    const size_t zfs = (size_t)a.F * S;
    const double *pgb = a.pg + (size_t)b * zfs;
    const double *pzb = a.pz + (size_t)b * Z * zfs;
    const double *pfb = (C == 3) ? a.pf + (size_t)b * Fam * zfs : nullptr;
    const double *wb = a.w + (size_t)b * a.F * C;
    const uint8_t *zb = a.zone + (size_t)b * a.N;
    const int row_bytes = S1 * 8;
    const int shift = a.xs8 ? 0 : 3;

    for (int x = lane; x < S1; x += WAVE) {
        tab[rz * S1 + x] = 0.0;
        tab[rn * S1 + x] = 1.0;
    }

    double m = 1.0;
    int e = 0;
    for (int c0 = 0; c0 < a.Np; c0 += SPL * WAVE) {
        uint32_t rows[SPL];
#pragma unroll
        for (int k = 0; k < SPL / 4; k++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int s = c0 + 4 * lane + 256 * k + j;
                uint32_t r = (uint32_t)rn | ((uint32_t)rn << 8) | ((uint32_t)rn << 16);
                if (s < a.N) {
                    const int z = zb[s];
                    const bool hz = z < Z;
                    const int fc = (C == 3) ? a.famc[s] : 0;
                    const bool hf = fc > 0;
                    const int r0 = (hz ? 1 : 0) | (hf ? 2 : 0);
                    const int r1 = hz ? off1 + 2 * z + (hf ? 1 : 0) : rz;
                    const int r2 = hf ? off2 + 2 * (fc - 1) + (hz ? 1 : 0) : rz;
                    r = (uint32_t)r0 | ((uint32_t)r1 << 8) | ((uint32_t)r2 << 16);
                }
                rows[4 * k + j] = r;
            }
        for (int f = fa; f < fb; f++) {
            {
                const double *wr = wb + (size_t)f * C;
                store_nw<C>(nw, lane, wr[0], wr[1], (C == 3) ? wr[2] : 0.0);
            }
            wave_lds_sync();
            int bad = 0;
            for (int x = lane; x < S1; x += WAVE) {
                const bool na = x == S;
                const size_t off = (size_t)f * S + (na ? 0 : x);
                const double l0 = na ? 1.0 : pgb[off];
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    const double v = nw[h * 4 + 0] * l0;
                    bad |= !safe_factor(v);
                    tab[h * S1 + x] = v;
                }
                for (int z = 0; z < Z; z++) {
                    const double l1 = na ? 1.0 : pzb[z * zfs + off];
                    const double v0 = nw[1 * 4 + 1] * l1, v1 = nw[3 * 4 + 1] * l1;
                    bad |= !safe_factor(v0) | !safe_factor(v1);
                    tab[(off1 + 2 * z) * S1 + x] = v0;
                    tab[(off1 + 2 * z + 1) * S1 + x] = v1;
                }
                for (int i = 0; i < Fam; i++) {
                    const double l2 = na ? 1.0 : pfb[i * zfs + off];
                    const double v0 = nw[2 * 4 + 2] * l2, v1 = nw[3 * 4 + 2] * l2;
                    bad |= !safe_factor(v0) | !safe_factor(v1);
                    tab[(off2 + 2 * i) * S1 + x] = v0;
                    tab[(off2 + 2 * i + 1) * S1 + x] = v1;
                }
            }
            const bool wide = __ballot(bad) != 0;
            wave_lds_sync();
            const uint32_t *ob =
                reinterpret_cast<const uint32_t *>(a.obs_fm + (size_t)f * a.Np + c0);
            const uint32_t *sb = reinterpret_cast<const uint32_t *>(
                a.src_fm + ((size_t)b * a.F + f) * a.Np + c0);
            uint32_t o[SPL / 4], sc[SPL / 4];
#pragma unroll
            for (int k = 0; k < SPL / 4; k++) {
                o[k] = ob[lane + 64 * k];
                sc[k] = sb[lane + 64 * k];
            }
#pragma unroll
            for (int k = 0; k < SPL / 4; k++) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t c = (sc[k] >> (8 * j)) & 0xff;
                    const uint32_t r = (rows[4 * k + j] >> (8 * min(c, 2u))) & 0xff;
                    const uint32_t rr = (c < (uint32_t)C) ? r : (uint32_t)rz;
                    const int addr = NW_BYTES + (int)rr * row_bytes +
                                     (int)(((o[k] >> (8 * j)) & 0xff) << shift);
                    m *= *reinterpret_cast<const double *>(lds + addr);
                    if (wide) renorm(m, e);
                }
                if (k & 1) renorm(m, e);
            }
            renorm(m, e);
            wave_lds_sync();
        }
    }
    const double v = log(m) + (double)e * LN2;
    const double tot = wave_sum(v);
    if (lane == 0) a.partial[(size_t)b * a.W + blockIdx.x] = tot;
}

// Per-chain site class bytes for the mixture table kernel: cls = zc*FamC + fc
// (zc = 0 no zone | z+1, fc = 0 no family | fam+1), padded sites -> ncls (the neutral row).
__global__ void site_class_kernel(int B, int N, int Np, int Z, int FamC, const uint8_t *zone,
                                  const uint8_t *famc, uint8_t *cls) {
    const int ncls = (Z + 1) * FamC;
    const size_t total = (size_t)B * Np;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int s = (int)(i % Np);
        const size_t b = i / Np;
        int c = ncls;
        if (s < N) {
            const int z = zone[b * N + s];
            c = ((z < Z) ? z + 1 : 0) * FamC + famc[s];
        }
        cls[i] = (uint8_t)c;
    }
}

// Sum the W task partials of each chain in task order (deterministic).
__global__ void lik_reduce_kernel(int B, int W, const double *partial, double *out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double s = 0.0;
    for (int t = 0; t < W; t++) s += partial[(size_t)b * W + t];
    out[b] = s;
}

// Row-major source [B][N][F] -> feature-major [B][F][Np] (padded sites -> component 0).
__global__ void repack_source_kernel(int B, int N, int F, int Np, const uint8_t *src, uint8_t *dst) {
    const size_t total = (size_t)B * F * Np;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int s = (int)(i % Np);
        const size_t r = i / Np;
        const int f = (int)(r % F);
        const int b = (int)(r / F);
        dst[i] = s < N ? src[((size_t)b * N + s) * F + f] : 0;
    }
}

template <int C, int FR, bool XS8>
void launch_mix_x(int spl, dim3 grid, size_t lds, hipStream_t st, const LikArgs &a) {
    switch (spl) {
        case 4: lik_mixture_kernel<C, 4, FR, XS8><<<grid, WAVE, lds, st>>>(a); break;
        case 8: lik_mixture_kernel<C, 8, FR, XS8><<<grid, WAVE, lds, st>>>(a); break;
        case 16: lik_mixture_kernel<C, 16, FR, XS8><<<grid, WAVE, lds, st>>>(a); break;
        default: lik_mixture_kernel<C, 32, FR, XS8><<<grid, WAVE, lds, st>>>(a); break;
    }
}

template <int C, int FR>
void launch_mix(int spl, dim3 grid, size_t lds, hipStream_t st, const LikArgs &a) {
    if (a.xs8) launch_mix_x<C, FR, true>(spl, grid, lds, st, a);
    else launch_mix_x<C, FR, false>(spl, grid, lds, st, a);
}

template <int C>
void launch_source(int spl, dim3 grid, size_t lds, hipStream_t st, const LikArgs &a) {
    switch (spl) {
        case 4: lik_source_kernel<C, 4><<<grid, WAVE, lds, st>>>(a); break;
        case 8: lik_source_kernel<C, 8><<<grid, WAVE, lds, st>>>(a); break;
        case 16: lik_source_kernel<C, 16><<<grid, WAVE, lds, st>>>(a); break;
        default: lik_source_kernel<C, 32><<<grid, WAVE, lds, st>>>(a); break;
    }
}

template <int C, int FR, bool XS8>
void configure_mix_x(std::vector<const void *> &v) {
    v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 4, FR, XS8>));
    v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 8, FR, XS8>));
    v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 16, FR, XS8>));
    v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 32, FR, XS8>));
}

template <int C>
void configure_mix(std::vector<const void *> &v) {
    configure_mix_x<C, 4, true>(v);
    configure_mix_x<C, 4, false>(v);
    if (C == 3) {
        configure_mix_x<C, 8, true>(v);
        configure_mix_x<C, 8, false>(v);
    }
}

template <int C>
void configure_source(std::vector<const void *> &v) {
    v.push_back(reinterpret_cast<const void *>(&lik_source_kernel<C, 4>));
    v.push_back(reinterpret_cast<const void *>(&lik_source_kernel<C, 8>));
    v.push_back(reinterpret_cast<const void *>(&lik_source_kernel<C, 16>));
    v.push_back(reinterpret_cast<const void *>(&lik_source_kernel<C, 32>));
}

// How the mixture branch runs for these dims: table path with FR family registers, or the
// generic per-cell path (fr == 0).
struct MixPlan {
    int fr = 0;
};

MixPlan plan_mixture(const sbz_dims &d, int C) {
    MixPlan p;
    const int S1 = d.n_states + 1;
    const int Fam = C == 3 ? d.n_families : 0;
    if (S1 > WAVE) return p;
    const int G = WAVE / S1;
    if (d.n_zones + 1 > ZR * G) return p;
    if ((d.n_zones + 1) * (Fam + 1) + 1 > 256) return p;  // class ids are bytes
    if ((1 + d.n_zones + Fam) * d.n_states + C > PL * WAVE) return p;
    if (C == 2 || Fam <= 4) p.fr = 4;
    else if (Fam <= 8) p.fr = 8;
    return p;
}

size_t mix_lds_bytes(const sbz_dims &d, int C) {
    const size_t S1 = (size_t)d.n_states + 1;
    const size_t Fam = C == 3 ? (size_t)d.n_families : 0;
    const size_t ncls = (size_t)(d.n_zones + 1) * (Fam + 1);
    const size_t per = (1 + d.n_zones + Fam) * d.n_states + C;
    return NW_BYTES + ((per + 1) & ~(size_t)1) * 8 + ((ncls + 1) * S1 + WAVE) * 8;
}

}  // namespace

int sites_per_lane(int n_sites) {
    if (n_sites <= 4 * WAVE) return 4;
    if (n_sites <= 8 * WAVE) return 8;
    if (n_sites <= 16 * WAVE) return 16;
    return 32;
}

size_t lik_lds_bytes(const sbz_dims &d, bool source_mode) {
    const bool inh = (d.flags & SBZ_INHERITANCE) != 0;
    const int C = inh ? 3 : 2;
    const size_t S1 = (size_t)d.n_states + 1;
    if (!source_mode) return plan_mixture(d, C).fr ? mix_lds_bytes(d, C) : 0;
    const size_t rows = 4 + 2 * (size_t)d.n_zones + (inh ? 2 * (size_t)d.n_families : 0) + 2;
    return NW_BYTES + rows * S1 * sizeof(double);
}

int lik_configure(sbz_ctx *ctx) {
    std::vector<const void *> fns;
    configure_mix<2>(fns);
    configure_mix<3>(fns);
    configure_source<2>(fns);
    configure_source<3>(fns);
    for (const void *fn : fns) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
    }
    return SBZ_OK;
}

int launch_loglik(sbz_ctx *ctx, int B, const uint8_t *zone, const double *w, const double *pg,
                  const double *pz, const double *pf, const uint8_t *source, double *out_ll) {
    const sbz_dims &d = ctx->d;
    const bool src_mode = source != nullptr;
    if (ctx->C == 3 && d.n_families > 0 && pf == nullptr)
        return fail(ctx, SBZ_EINVAL, "p_fam is required with inheritance");
    if (B <= 0) return SBZ_OK;
    const int F = d.n_features;

    LikArgs a{};
    a.N = d.n_sites;
    a.F = F;
    a.S = d.n_states;
    a.Z = d.n_zones;
    a.Fam = d.n_families;
    a.C = ctx->C;
    a.FamC = ctx->FamC;
    a.Np = ctx->Np;
    a.xs8 = ctx->xs8;
    a.B = B;
    a.obs_fm = ctx->d_obs_fm;
    a.famc = ctx->d_famc;
    a.zone = zone;
    a.w = w;
    a.pg = pg;
    a.pz = pz;
    a.pf = pf;

    MixPlan plan;
    size_t lds = 0;
    int rc;
    if (!src_mode) {
        plan = plan_mixture(d, ctx->C);
        if (plan.fr) {
            rc = ensure(ctx, ctx->cls, (size_t)B * ctx->Np);
            if (rc) return rc;
            const size_t n = (size_t)B * ctx->Np;
            site_class_kernel<<<(int)std::min<size_t>((n + 255) / 256, 4096), 256, 0, ctx->stream>>>(
                B, d.n_sites, ctx->Np, d.n_zones, ctx->FamC, zone, ctx->d_famc,
                static_cast<uint8_t *>(ctx->cls.ptr));
            a.cls = static_cast<const uint8_t *>(ctx->cls.ptr);
            lds = mix_lds_bytes(d, ctx->C);
            a.s_magic = ((1ull << 32) + d.n_states - 1) / d.n_states;  // ceil(2^32 / S)
            // long tasks (the parameter pipeline amortises the set-up): ~2 rounds of
            // 24 waves on 256 CUs
            const int W = std::max(1, std::min((F + 1) / 2, (256 * 48 + B - 1) / B));
            a.fpw = (F + W - 1) / W;
        }
    } else {
        lds = lik_lds_bytes(d, true);
        if (lds > 64 * 1024)
            return fail(ctx, SBZ_EINVAL, "source-mode table needs " + std::to_string(lds) +
                                             " B of LDS per wave (> 64 KiB)");
    }
    if (src_mode || !plan.fr) {
        // one wave per (chain, feature range): enough tasks to fill 256 CUs x 32 waves
        int W = std::max(1, std::min(F, (256 * 32 + B - 1) / B));
        a.fpw = (F + W - 1) / W;
    }
    a.W = (F + a.fpw - 1) / a.fpw;

    rc = ensure(ctx, ctx->partial, (size_t)B * a.W * sizeof(double));
    if (rc) return rc;
    a.partial = static_cast<double *>(ctx->partial.ptr);

    if (src_mode) {
        const size_t bytes = (size_t)B * F * ctx->Np;
        rc = ensure(ctx, ctx->src_t, bytes);
        if (rc) return rc;
        const int blocks = (int)std::min<size_t>((bytes + 255) / 256, 8192);
        repack_source_kernel<<<blocks, 256, 0, ctx->stream>>>(B, d.n_sites, F, ctx->Np, source,
                                                             static_cast<uint8_t *>(ctx->src_t.ptr));
        a.src_fm = static_cast<const uint8_t *>(ctx->src_t.ptr);
    }

    dim3 grid(a.W, B);
    hipStream_t st = ctx->stream;
    if (src_mode) {
        if (ctx->C == 3) launch_source<3>(ctx->spl, grid, lds, st, a);
        else launch_source<2>(ctx->spl, grid, lds, st, a);
    } else if (!plan.fr) {
        if (ctx->C == 3) lik_mixture_generic_kernel<3><<<grid, WAVE, 0, st>>>(a);
        else lik_mixture_generic_kernel<2><<<grid, WAVE, 0, st>>>(a);
    } else {
        if (ctx->C == 3) {
            if (plan.fr == 4) launch_mix<3, 4>(ctx->spl, grid, lds, st, a);
            else launch_mix<3, 8>(ctx->spl, grid, lds, st, a);
        } else {
            launch_mix<2, 4>(ctx->spl, grid, lds, st, a);
        }
    }
    lik_reduce_kernel<<<(B + 63) / 64, 64, 0, st>>>(B, a.W, a.partial, out_ll);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "likelihood launch");
    return SBZ_OK;
}

}  // namespace sbz
