// sbz_mh_common.h — device helpers shared by the sampler kernels (sbz_mh.hip: SAMPLE_SOURCE =
// false; sbz_mh_src.hip: SAMPLE_SOURCE = true): wave-uniform scalars, range-checked indices,
// L1-bypassing parameter loads/stores, Philox4x32-10 and the draw source (Rng), the Dirichlet
// proposal, the reference cell, and the kernel arguments.
#pragma once
#include <cmath>
#include <cstdint>

#include "sbz_internal.h"

namespace sbz {

namespace {

constexpr int WAVE = 64;
constexpr int NONE = 255;
constexpr double LN2 = 0.69314718055994530941723212145818;
enum Op { SHRINK = 0, GROW = 1, SWAP = 2, WEIGHTS = 3, P_GLOBAL = 4, P_ZONES = 5, P_FAMILIES = 6,
          GIBBSISH = 7, G_SOURCES = 8, G_WEIGHTS = 9, G_P_GLOBAL = 10, G_P_ZONES = 11, G_P_FAMILIES = 12 };

__device__ __forceinline__ void wsync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Wave reductions and scans on DPP lane moves (VALU, a few cycles each) instead of LDS-crossbar
// shuffles: butterflies inside each 16-lane row (quad_perm, half-mirror, mirror), then the row
// totals combined by row_bcast15 / row_bcast31, which leave the total in lane 63 (read back as a
// wave-uniform value).  Fixed order, so the double sum is deterministic.  All 64 lanes active.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {  // lanes without a source read 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp64(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = dpp32<CTRL, ROWS>((uint32_t)b), hi = dpp32<CTRL, ROWS>((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
enum : int { DPP_QP_1032 = 0xb1, DPP_QP_2301 = 0x4e, DPP_ROW_MIRROR = 0x140,
             DPP_ROW_HALF_MIRROR = 0x141, DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143,
             DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118 };

__device__ __forceinline__ double wave_sum(double v) {
    v = v + dpp64<DPP_QP_1032>(v);
    v = v + dpp64<DPP_QP_2301>(v);
    v = v + dpp64<DPP_ROW_HALF_MIRROR>(v);
    v = v + dpp64<DPP_ROW_MIRROR>(v);        // every lane of a row: the row total
    v = v + dpp64<DPP_BCAST15, 0xa>(v);      // rows 1, 3: + rows 0, 2
    v = v + dpp64<DPP_BCAST31, 0xc>(v);      // rows 2, 3: + rows 0 + 1
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, 63);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), 63);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ int wave_sum_i(int v) {
    v += (int)dpp32<DPP_QP_1032>((uint32_t)v);
    v += (int)dpp32<DPP_QP_2301>((uint32_t)v);
    v += (int)dpp32<DPP_ROW_HALF_MIRROR>((uint32_t)v);
    v += (int)dpp32<DPP_ROW_MIRROR>((uint32_t)v);
    v += (int)dpp32<DPP_BCAST15, 0xa>((uint32_t)v);
    v += (int)dpp32<DPP_BCAST31, 0xc>((uint32_t)v);
    return (int)__builtin_amdgcn_readlane((uint32_t)v, 63);
}

// inclusive prefix sum over the wave's lanes (lane order); the wave total is in lane 63
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += (int)dpp32<DPP_ROW_SHR1>((uint32_t)v);
    v += (int)dpp32<DPP_ROW_SHR2>((uint32_t)v);
    v += (int)dpp32<DPP_ROW_SHR4>((uint32_t)v);
    v += (int)dpp32<DPP_ROW_SHR8>((uint32_t)v);
    v += (int)dpp32<DPP_BCAST15, 0xa>((uint32_t)v);
    v += (int)dpp32<DPP_BCAST31, 0xc>((uint32_t)v);
    return v;
}

__device__ __forceinline__ int lane_prefix(uint64_t mask) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Range-checked index: an index outside [0, lim) is recorded (the first one, as `code`, with its
// value) and replaced by 0, so no access ever leaves its allocation; the chain then stops with
// status 16 + code (a replay mismatch or corrupt input, never silently).
#define MH_IDX(i, lim, code) sbz_mh_idx((long long)(i), (long long)(lim), (code), err, err_val)
__device__ __forceinline__ size_t sbz_mh_idx(long long i, long long lim, int code, int &err,
                                             long long &err_val) {
    if (i >= 0 && i < lim) return (size_t)i;
    if (!err) {
        err = code;
        err_val = i;
    }
    return 0;
}

// The chain's parameters are rewritten inside the kernel (lane 0, on acceptance) and re-read by
// every lane in later steps.  A plain load can hit a line the CU's vector L1 cached before the
// store, so parameter loads bypass L1 (sc1) and parameter stores are sc1 stores followed by
// vmcnt(0) (MI355X_MICROARCH.md, the sc1 rows of the hand-off table).
__device__ __forceinline__ double ldp(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stp(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ldi(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A read of LDS through a local-address-space pointer (ds_read).  A generic-pointer read of an
// LDS array beside a read of a global array under a uniform select (`staged ? lds[i] :
// global[i]`) lets the optimiser merge the two into one flat load of a selected pointer: slower
// than ds_read, and it has the shared aperture base allocated to VCC, whose copy ROCm 7.2's
// gfx950 back end lowers to an illegal "V_CMP_NE_U32_e32 0, $src_shared_base".  Reading the LDS
// side through this keeps the two loads apart.
template <class T>
__device__ __forceinline__ T lds_rd(const T *p) {
    return *(const __attribute__((address_space(3))) T *)p;
}

__device__ __forceinline__ void renorm(double &m, int &e) {
    e += __builtin_amdgcn_frexp_exp(m);
    m = __builtin_amdgcn_frexp_mant(m);
}

// log(x) in ~30 dependent f64 operations: x = m 2^e with m in [sqrt(1/2), sqrt(2)), log m =
// 2 atanh(s), s = (m - 1) / (m + 1) (v_rcp_f64, two Newton steps and the residual of m + 1's
// rounding), the atanh series to s^21 by Estrin, e ln 2 in two parts; 0 -> -inf, +inf -> +inf,
// x < 0 or NaN -> NaN.  Accuracy: <= 1.43 ulp (mean 0.31 ulp against a long-double log over 1e7
// arguments, denormals included) was measured on the Horner form of the series that came first;
// the Estrin form evaluates the same polynomial in another order (its rounding differs by a few
// ulp of the series tail, far below an ulp of the result), and every likelihood / acceptance
// value it feeds is held to 1e-9 by the parity tests.  The Estrin form once tripped a gfx950
// code-generation error ("V_CMP_NE_U32_e32 0, $src_shared_base") that came from LDS reads merged
// into flat loads, not from the series; lds_rd() keeps those apart (commit bf8a8f8).  The
// library's log is correctly rounded through double-double steps: ~670 cycles of latency on
// gfx950 against ~550 (tools/gamma_lat.hip, profiles/r04_gamma_lat.txt; a dependent f64
// operation costs ~18 cycles).  Used where a log sits on a step's critical path and the value is
// a likelihood / acceptance term (the tape replays' decisions and the 1e-9 parity bar are
// unaffected); SBZ_FLOG=0 builds (A/B only) use the library log everywhere.
#ifndef SBZ_FLOG
#define SBZ_FLOG 1
#endif
__device__ __forceinline__ double flog(double x) {
#if SBZ_FLOG
    double m = __builtin_amdgcn_frexp_mant(x);
    int e = __builtin_amdgcn_frexp_exp(x);
    const bool lo = m < 0.70710678118654752440;
    m = lo ? m * 2.0 : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0, d = m + 1.0;  // f exact
    const double dl = m - (d - 1.0);        // m + 1 = d + dl exactly
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    const double s0 = f * r;
    const double sv = fma(r, fma(-s0, d, f) - s0 * dl, s0);
    // the series' tail sum_k 2 / (2k + 3) z^k, k = 0..9, by Estrin (4 dependent levels after z)
    const double z = sv * sv;
    const double z2 = z * z, z4 = z2 * z2, z8 = z4 * z4;
    const double a0 = fma(2.0 / 5.0, z, 2.0 / 3.0), a1 = fma(2.0 / 9.0, z, 2.0 / 7.0);
    const double a2 = fma(2.0 / 13.0, z, 2.0 / 11.0), a3 = fma(2.0 / 17.0, z, 2.0 / 15.0);
    const double a4 = fma(2.0 / 21.0, z, 2.0 / 19.0);
    const double p = fma(a4, z8, fma(fma(a3, z2, a2), z4, fma(a1, z2, a0)));
    const double lm = fma(sv * z, p, 2.0 * sv);
    const double de = (double)e;
    double v = fma(de, 6.93147180369123816490e-01, fma(de, 1.90821492927058770002e-10, lm));
    v = x == 0.0 ? -INFINITY : v;
    v = x == INFINITY ? INFINITY : v;
    return (x < 0.0 || x != x) ? __builtin_nan("") : v;
#else
    return log(x);
#endif
}

// log(m 2^k) for a renormalised product m (frexp mantissa, or 0 / not finite) and its exponent k:
// flog's series with k added to the exponent part (two-part ln 2), so a product of exact 1.0
// factors gives exactly 0
__device__ __forceinline__ double flog_e(double x, int k) {
    double m = __builtin_amdgcn_frexp_mant(x);
    int e = __builtin_amdgcn_frexp_exp(x);
    const bool lo = m < 0.70710678118654752440;
    m = lo ? m * 2.0 : m;
    e = (lo ? e - 1 : e) + k;
    const double f = m - 1.0, d = m + 1.0;
    const double dl = m - (d - 1.0);
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    const double s0 = f * r;
    const double sv = fma(r, fma(-s0, d, f) - s0 * dl, s0);
    const double z = sv * sv;
    const double z2 = z * z, z4 = z2 * z2, z8 = z4 * z4;
    const double a0 = fma(2.0 / 5.0, z, 2.0 / 3.0), a1 = fma(2.0 / 9.0, z, 2.0 / 7.0);
    const double a2 = fma(2.0 / 13.0, z, 2.0 / 11.0), a3 = fma(2.0 / 17.0, z, 2.0 / 15.0);
    const double a4 = fma(2.0 / 21.0, z, 2.0 / 19.0);
    const double p = fma(a4, z8, fma(fma(a3, z2, a2), z4, fma(a1, z2, a0)));
    const double lm = fma(sv * z, p, 2.0 * sv);
    const double de = (double)e;
    double v = fma(de, 6.93147180369123816490e-01, fma(de, 1.90821492927058770002e-10, lm));
    v = x == 0.0 ? -INFINITY : v;
    v = x == INFINITY ? INFINITY : v;
    return (x < 0.0 || x != x) ? __builtin_nan("") : v;
}

// a / b for normal positive a, b away from the range limits (v_rcp_f64, two Newton steps and
// one residual correction: <= 1 ulp): ~7 dependent operations against the IEEE sequence's
// div_scale / div_fmas / div_fixup (~310 cycles, profiles/r04_gamma_lat.txt).
__device__ __forceinline__ double fdiv_pos(double a, double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    r = fma(fma(-b, r, 1.0), r, r);
    const double q = a * r;
    return fma(r, fma(-b, q, a), q);
}

// ---------------------------------------------------------------------------------------
// Random draws (wave-uniform).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void philox_round(uint32_t (&c)[4], const uint32_t (&k)[2]) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k[0];
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k[1];
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
}

__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
    uint32_t k[2] = {k0, k1};
#pragma unroll
    for (int i = 0; i < 10; i++) {
        philox_round(c, k);
        k[0] += 0x9E3779B9u;
        k[1] += 0xBB67AE85u;
    }
}

// Wave-uniform scalars: every decision of the step loop is forced through readfirstlane, so the
// lanes can never disagree on the control flow (and the values live in SGPRs).
__device__ __forceinline__ int uni(int v) { return (int)__builtin_amdgcn_readfirstlane((uint32_t)v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double uni(double v) {
    return __longlong_as_double((long long)uni64((int64_t)__double_as_longlong(v)));
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
    return (double)((((uint64_t)hi << 32) | lo) >> 11) * 0x1p-53;
}

// The draw source: a replay tape (read straight from HBM, one item per draw, broadcast to the
// wave) or Philox4x32-10.  Philox uniforms are numbered by `ctr` (per chain, carried across
// launches): uniform i is half (i & 1) of block (i >> 1, chain) under key = seed.  The wave keeps
// a pool of 32 consecutive uniforms (uniforms 2l, 2l + 1 in lane l < 16, computed by 16 lanes at
// once) and broadcasts them with v_readlane, so a draw costs no Philox rounds on the step's
// critical path.  The numbering does not depend on the pool, so a run split into several
// launches draws the same uniforms.  The scalar members live in SGPRs; nothing of it lives in
// per-lane scratch.
struct Rng {
    const double *tape;  // this chain's tape, or null (Philox)
    int64_t pos, len;    // tape cursor / length
    uint32_t key0, key1;
    uint64_t chain, ctr; // Philox stream (global chain id) and uniform counter
    int bad;             // tape exhausted
    uint64_t pbase = 1ull << 63;  // index of the pool's first uniform (multiple of 32); none yet
    double pool0, pool1;          // per lane: uniforms pbase + 2 lane, pbase + 2 lane + 1

    __device__ __forceinline__ double tape_item() {
        if (pos >= len) {
            bad = 1;
            return 0.0;
        }
        const double v = tape[pos];
        pos = uni64(pos + 1);
        return uni(v);
    }
    __device__ __forceinline__ void fill(uint64_t base) {  // wave-uniform call
        const uint64_t blk = (base >> 1) + (uint64_t)(threadIdx.x & 15);
        uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)chain, (uint32_t)(chain >> 32)};
        philox4x32_10(c, key0, key1);
        pool0 = u53(c[0], c[1]);
        pool1 = u53(c[2], c[3]);
        pbase = base;
    }
    __device__ __forceinline__ double uniform53() {  // [0, 1) with 53 random bits
        if (ctr - pbase >= 32) fill(ctr & ~31ull);
        const int i = (int)(ctr - pbase);
        ctr++;
        return uni(readlane_d((i & 1) ? pool1 : pool0, i >> 1));
    }
    // a real in [0, 1): python random.random() / the acceptance and connected-step uniforms
    __device__ __forceinline__ double real() { return tape ? tape_item() : uniform53(); }
    // an index in [0, n): np.random.choice(range(n)) / random.choice(seq) -> seq[k]
    __device__ __forceinline__ int below(int n) {
        if (tape) return uni((int)tape_item());
        return uni(min((int)(uniform53() * (double)n), n - 1));
    }
    __device__ __forceinline__ int op(const double *cdf, int nops) {
        if (tape) return uni((int)tape_item());
        const double u = uniform53();  // numpy choice(p): first cdf entry > u
        int i = 0;                     // = the number of entries <= u (the cdf is non-decreasing)
#pragma unroll
        for (int k = 0; k < SBZ_N_OPS - 1; k++) i += (k < nops - 1 && !(u < cdf[k])) ? 1 : 0;
        return uni(i);
    }
    // random.sample(population, 2): two distinct values in draw order (pop == null: 0..n-1)
    __device__ __forceinline__ void pair(const int *pop, int n, int &a, int &b) {
        if (tape) {
            a = uni((int)tape_item());
            b = uni((int)tape_item());
            return;
        }
        const int i = below(n);
        int j = below(n - 1);
        if (j >= i) j++;
        a = uni(pop ? pop[i] : i);
        b = uni(pop ? pop[max(j, 0)] : j);  // n < 2: j = -1, a pair the caller's checks reject
    }
    // np.random.dirichlet(alpha) for 2 components; Philox mode: the two gammas run at once on
    // lanes 0 and 1, each on its own lane stream (LaneRng) based at the current counter
    __device__ __forceinline__ void dirichlet2(double a0, double a1, double &x0, double &x1);
};

// Uniform number i of a chain's Rng stream, computed by one lane on its own (the value
// Rng::uniform53 returns for counter i): half (i & 1) of Philox block (i >> 1, chain).
__device__ __forceinline__ double philox_uniform(uint32_t key0, uint32_t key1, uint64_t chain, uint64_t i) {
    const uint64_t blk = i >> 1;
    uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)chain, (uint32_t)(chain >> 32)};
    philox4x32_10(c, key0, key1);
    return (i & 1) ? u53(c[2], c[3]) : u53(c[0], c[1]);
}

// gibbsish_sample_zones, Philox mode: uniform i of the per-site stream keyed by counter slot
// `slot` of the step's window (the subset draw at slot 2, the in / out draw at slot 3): half
// (i & 1) of block (i >> 1, slot lo, chain, slot hi ^ 0xFE << 24), a stream no LaneRng lane
// (lane + 1 < 0xFE) shares.  Any thread computes any site's uniform on its own.
__device__ __forceinline__ double site_uniform(uint32_t key0, uint32_t key1, uint64_t chain, uint64_t slot,
                                               uint32_t i) {
    uint32_t c[4] = {i >> 1, (uint32_t)slot, (uint32_t)chain, (uint32_t)(slot >> 32) ^ 0xFE000000u};
    philox4x32_10(c, key0, key1);
    return (i & 1) ? u53(c[2], c[3]) : u53(c[0], c[1]);
}

// Per-lane Philox stream: block (j, base lo, chain, base hi ^ (lane + 1) << 24), key = seed.
// `base` is the wave's 64-bit counter when the phase started (the wave then advances it by one),
// j counts the lane's draws in the phase.  The counter's high word goes into c3 (bits 0..19; a
// counter stays far below 2^52), so a chain's lane streams never repeat when its counter passes
// 2^32; the host keeps global chain ids below 2^32 (c2).
struct LaneRng {
    uint32_t k0, k1, base, c2, c3, j;
    // one Philox block gives two uniforms (words 0-1 and 2-3): the second is kept for the next call
    double spare;
    int has_spare;  // set by init / initk
    __device__ __forceinline__ void init(const Rng &r, int lane) {
        k0 = r.key0;
        k1 = r.key1;
        base = (uint32_t)r.ctr;
        c2 = (uint32_t)r.chain;
        c3 = (uint32_t)(r.ctr >> 32) ^ ((uint32_t)(lane + 1) << 24);
        j = 0;
        has_spare = 0;
    }
    // as init, from the key / chain / counter values themselves
    __device__ __forceinline__ void initk(uint32_t key0, uint32_t key1, uint64_t chain, uint64_t ctr,
                                          int lane) {
        k0 = key0;
        k1 = key1;
        base = (uint32_t)ctr;
        c2 = (uint32_t)chain;
        c3 = (uint32_t)(ctr >> 32) ^ ((uint32_t)(lane + 1) << 24);
        j = 0;
        has_spare = 0;
    }
    // a stream per thread of a multi-wave workgroup (id < 2048)
    __device__ __forceinline__ void initw(const Rng &r, int id) {
        init(r, 0);
        c3 = (uint32_t)(r.ctr >> 32) ^ ((uint32_t)(id + 1) << 20);
    }
    __device__ __forceinline__ double u() {
        if (has_spare) {
            has_spare = 0;
            return spare;
        }
        uint32_t c[4] = {j++, base, c2, c3};
        philox4x32_10(c, k0, k1);
        spare = u53(c[2], c[3]);
        has_spare = 1;
        return u53(c[0], c[1]);
    }
    __device__ __forceinline__ double normal() {
        const double u1 = 1.0 - u();
        const double u2 = u();
        // cos(2 pi u2) as cospi(2 u2): no large-argument reduction (u2 in [0, 1))
        return sqrt(-2.0 * flog(u1)) * cospi(2.0 * u2);
    }
    // Marsaglia-Tsang (alpha >= 1; boosted by u^(1/alpha) below 1), at most 64 rounds (each
    // accepts with probability > 0.95; reaching 64 has probability < 1e-80).  A two-candidate
    // form (both normals of one Box-Muller pair per round, so a wave mostly runs one round) was
    // measured slower on the cfg5 sampler (5.03 vs 4.82 us per step) and equal on the source
    // sampler (profiles/r03_ab_gamma.txt).
    __device__ __forceinline__ double gamma(double alpha) {
        const double boost = alpha < 1.0 ? pow(u(), 1.0 / alpha) : 1.0;
        const double a = alpha < 1.0 ? alpha + 1.0 : alpha;
        const double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
        double r = d;
        for (int it = 0; it < 64; it++) {
            const double x = normal();
            double v = 1.0 + c * x;
            if (v <= 0.0) continue;
            v = v * v * v;
            const double w = u();
            bool ok = w < 1.0 - 0.0331 * (x * x) * (x * x);
            if (!ok) {
                const double lw = flog(w), lv = flog(v);
                ok = lw < 0.5 * x * x + d * (1.0 - v + lv);
            }
            if (ok) {
                r = d * v;
                break;
            }
        }
        return r * boost;
    }
};

// Gamma draws of the source sampler's Gibbs redraws (Philox mode, sbz_mh_src.hip gamma_fill):
// integer alpha = n <= GB_NMAX as -log(u_1 ... u_n), exactly Gamma(n, 1) (a sum of n exponentials,
// no rejection), with 32-bit uniforms (w + 1/2) 2^-32; others by Marsaglia-Tsang.
constexpr int GB_NMAX = 16;
__device__ __forceinline__ double u32o(uint32_t w) { return ((double)w + 0.5) * 0x1p-32; }

__device__ __forceinline__ void Rng::dirichlet2(double a0, double a1, double &x0, double &x1) {
    if (tape) {
        x0 = tape_item();
        x1 = tape_item();
        return;
    }
    const int lane = threadIdx.x & 63;
    LaneRng lr;
    lr.init(*this, lane);
    double g = 0.0;
    if (lane < 2) g = lr.gamma(lane ? a1 : a0);
    ctr++;
    const double g0 = readlane_d(g, 0), g1 = readlane_d(g, 1);
    const double s = g0 + g1;
    x0 = uni(g0 / s);
    x1 = uni(g1 / s);
}

// scipy.stats.dirichlet._logpdf for 2 components:
//   -(sum gammaln(a) - gammaln(sum a)) + sum xlogy(a - 1, x)
__device__ __forceinline__ double dirichlet_logpdf2(double x0, double x1, double a0, double a1) {
    const double lnB = (lgamma(a0) + lgamma(a1)) - lgamma(a0 + a1);
    const double t0 = (a0 - 1.0) == 0.0 ? 0.0 : (a0 - 1.0) * log(x0);
    const double t1 = (a1 - 1.0) == 0.0 ? 0.0 : (a1 - 1.0) * log(x1);
    return -lnB + (t0 + t1);
}

// dirichlet_proposal on a pair w (sums to 1): new pair, log q, log q_back.  q = exp(logpdf) and
// log q as the reference (zone_sampling.py:537-569, util.py dirichlet_pdf); the ten lgamma / log
// terms of the two densities run at once on lanes 0..9 (same functions, same arguments as
// dirichlet_logpdf2), then exp and log on lanes 0 / 1.
__device__ __forceinline__ void dirichlet_proposal2(Rng &rng, double w0, double w1, double prec, double &n0,
                                    double &n1, double &log_q, double &log_q_back) {
    const double a0 = 1.0 + prec * w0, a1 = 1.0 + prec * w1;
    rng.dirichlet2(a0, a1, n0, n1);
    const double b0 = 1.0 + prec * n0, b1 = 1.0 + prec * n1;
    const int lane = threadIdx.x & 63;
    const double args[10] = {a0, a1, a0 + a1, b0, b1, b0 + b1, n0, n1, w0, w1};
    double arg = 1.0;
#pragma unroll
    for (int i = 0; i < 10; i++) arg = lane == i ? args[i] : arg;
    double r;
    if (lane < 6) r = lgamma(arg);
    else r = log(arg);
    double v[10];
#pragma unroll
    for (int i = 0; i < 10; i++) v[i] = readlane_d(r, i);
    // -(sum gammaln(a) - gammaln(sum a)) + sum xlogy(a - 1, x)
    const double tq0 = (a0 - 1.0) == 0.0 ? 0.0 : (a0 - 1.0) * v[6];
    const double tq1 = (a1 - 1.0) == 0.0 ? 0.0 : (a1 - 1.0) * v[7];
    const double tb0 = (b0 - 1.0) == 0.0 ? 0.0 : (b0 - 1.0) * v[8];
    const double tb1 = (b1 - 1.0) == 0.0 ? 0.0 : (b1 - 1.0) * v[9];
    const double lq = -((v[0] + v[1]) - v[2]) + (tq0 + tq1);
    const double lb = -((v[3] + v[4]) - v[5]) + (tb0 + tb1);
    const double e = exp(lane == 0 ? lq : lb);
    const double l = log(lane == 0 ? readlane_d(e, 0) : readlane_d(e, 1));
    log_q = uni(readlane_d(l, 0));
    log_q_back = uni(readlane_d(l, 1));
}

// scipy.special.xlogy(a, x): 0 where a == 0, else a * log(x)
__device__ __forceinline__ double xlogy(double a, double x) { return a == 0.0 ? 0.0 : a * log(x); }

// Change of the zone-size prior (ZoneSizePrior, model.py:932-971) when one zone goes from size
// s to s1 = s +- 1: 'uniform' is -sum log C(N, size) (log_binom, util.py:1202-1217), and
// C(N, k+1) / C(N, k) = (N-k) / (k+1), so the change is one log of that ratio; 'quadratic' is
// -sum log(size^2).
__device__ __forceinline__ double size_prior_delta(int kind, int N, int s, int s1) {
    if (kind == 1) {
        return s1 > s ? -log((double)(N - s) / (double)(s + 1))   // grow
                      : -log((double)s / (double)(N - s + 1));    // shrink
    }
    if (kind == 2) return log((double)s * (double)s) - log((double)s1 * (double)s1);
    return 0.0;
}

// The reference cell for one (site, feature): normalize_weights (model.py:436-452) then
// (n0*l0 + n1*l1) + n2*l2 with NA -> every lh 1 and absent components -> lh 0.
template <int C>
__device__ __forceinline__ double cell(const double (&w)[3], bool hz, bool hf, bool na, double l0,
                                       double l1, double l2) {
    const double w0 = w[0] * 1.0, w1 = w[1] * (hz ? 1.0 : 0.0);
    double sum = w0 + w1, w2 = 0.0;
    if (C == 3) {
        w2 = w[2] * (hf ? 1.0 : 0.0);
        sum = sum + w2;
    }
    const double L0 = na ? 1.0 : l0;
    const double L1 = na ? 1.0 : (hz ? l1 : 0.0);
    double v = (w0 / sum) * L0 + (w1 / sum) * L1;
    if (C == 3) v = v + (w2 / sum) * (na ? 1.0 : (hf ? l2 : 0.0));
    return v;
}

// The reference cell from pre-normalised weights n (normalize_weights, model.py:436-452, computed
// exactly as cell() computes them): the same operations in the same order as cell().
template <int C>
__device__ __forceinline__ double cell_nw(const double (&n)[3], bool hz, bool hf, bool na, double l0,
                                          double l1, double l2) {
    const double L0 = na ? 1.0 : l0;
    const double L1 = na ? 1.0 : (hz ? l1 : 0.0);
    double v = n[0] * L0 + n[1] * L1;
    if (C == 3) v = v + n[2] * (na ? 1.0 : (hf ? l2 : 0.0));
    return v;
}

// A table factor that keeps an 8-factor product of mantissas in the normal range: 0 or within
// [2^-120, 2^120]; otherwise the gathers renormalise after every factor.
__device__ __forceinline__ bool safe_cell(double v) { return v == 0.0 || (v >= 0x1p-120 && v <= 0x1p120); }

__device__ __forceinline__ void *align16(void *p) {
    return reinterpret_cast<void *>((reinterpret_cast<uintptr_t>(p) + 15) & ~(uintptr_t)15);
}

struct Chain {
    // LDS
    uint8_t *zos;       // [N] zone of site
    uint16_t *nb;       // [N] neighbour stamps
    int *zsize;         // [Z]
    double *col;        // staged parameter column (old values)
    uint16_t stamp;
    int occupied;       // sites in any zone
};

}  // namespace

struct MhArgs {
    int N, F, S, Z, Fam, C, FamC, Np, xs8;
    int n_steps, nops, min_size, warmup;
    int la;     // mh_kernel, Philox draws: proposals planned ahead per batch (1 = none; <= LA = 24;
                // the host lowers it until the plan columns fit the 160 KiB of LDS)
    int ntab;   // mh_kernel: per-wave cell-table slots (1 .. waves): planned parameter moves on
                // different features computed at once, at most ntab (the host fits it to the LDS)
    int stage;  // mh_src_kernel: parameters and normalised weights staged in LDS for the N*F passes
    int cstage; // mh_src_kernel (with stage): the constant tables (applicable states, Gibbs prior
                //   counts, 'counts' prior) staged in LDS too
    int gib;    // gibbsish_sample_zones has a non-zero weight: LDS holds its per-site scratch
    uint32_t gib_off;  // mh_src_kernel: byte offset of that scratch in LDS
    double op_cdf[SBZ_N_OPS];
    double prec[4];
    const uint8_t *obs_fm;      // [F][Np] by position
    const uint8_t *famc;        // [Np] by position
    const int *perm;            // [Np] site of position
    const uint8_t *obs_sm;      // [N][F] x by site (S = NA)
    const uint8_t *fam_site;    // [N] family class by site
    const int *adj_ptr, *adj_idx;
    int nnz;
    const int *app_list;        // [F][S] applicable states of each feature (ascending)
    const int *app_cnt;         // [F]
    const double *alpha_g;      // [F][S] 'counts' prior on p_global, or null (sbz_set_priors)
    const double *alpha_f;      // [Fam][F][S] 'counts' prior on p_families, or null
    int size_prior;             // 0 none, 1 uniform, 2 quadratic
    const double *gc_g;         // [F][S] Gibbs prior counts of p_global (sbz_set_gibbs_counts) or null = 1
    const double *gc_f;         // [Fam][F][S] of p_families, or null = 1
    uint8_t *src_scratch;       // [B][F][Np] candidate sources when they live in HBM (source mode)
    int *ctab;                  // source mode, table passes: count tables [2][B][F][CTP] (current /
    size_t ct_half;             //   candidate halves, B * F * CTP ints apart; TbDims)
    int src_pm;                 // ch.source is [B][F][Np] by position (SBZ_SOURCE_BY_POSITION)
    const double *geo_cost;     // [N][N] 'cost_based' geo prior costs (sbz_set_geo_prior), or null
    double geo_scale;
    sbz_chains ch;
};

// GeoPrior 'cost_based' (geo_prior_distance, sbayes/model.py:1096-1139) of zone zt with the
// tentative change (+add, -rm1, -rm2; -1 = none): the mean exponential(scale) log density
// -(d / scale) - log(scale) over the positive-cost edges of the minimum spanning tree of the
// zone's cost submatrix (scipy's sparse tree leaves zero-cost edges out; inf = no edge, a forest
// then), -log(scale) when no edge is positive.  Prim's algorithm, block-cooperative: the members
// are gathered into mem[], key[] holds each unused member's cheapest link (-1 once in the tree),
// and one block argmin (ties: lowest index) per added vertex.  Every thread gets the same value.
// LDS scratch: key [N] doubles, mem [N] u16, cnt 1 int, redd / redi [NW].
__host__ __device__ constexpr size_t geo_scratch_bytes(int N) {
    return (size_t)N * 8 + (size_t)((N + 7) & ~7) * 2 + 16 + 16 * 8 + 16 * 4;
}

template <int NW>
__device__ double geo_zone_prior(const double *cost, double scale, int N, const uint8_t *zos, int zt,
                                 int add, int rm1, int rm2, double *key, uint16_t *mem, int *cnt,
                                 double *redd, int *redi) {
    constexpr int NT = NW * 64;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    auto bar = [&]() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    if (tid == 0) *cnt = 0;
    bar();
    for (int s = tid; s < N; s += NT) {
        const bool in = (zos[s] == zt && s != rm1 && s != rm2) || s == add;
        if (in) mem[atomicAdd(cnt, 1)] = (uint16_t)s;
    }
    bar();
    const int m = uni(*cnt);
    const double lsc = log(scale);
    if (m <= 1) {  // (the reference raises "Too few locations"; zones have >= MIN_M sites)
        bar();
        return -lsc;
    }
    for (int i = tid; i < m; i += NT) key[i] = i == 0 ? 0.0 : INFINITY;
    bar();
    double sum = 0.0;
    int npos = 0;
    for (int it = 0; it < m; it++) {
        double bk = INFINITY;
        int bi = 0x7fffffff;
        for (int i = tid; i < m; i += NT) {
            const double k = key[i];
            if (k >= 0.0 && (k < bk || (k == bk && i < bi))) {
                bk = k;
                bi = i;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const double ok = __shfl_xor(bk, off, 64);
            const int oi = __shfl_xor(bi, off, 64);
            if (ok < bk || (ok == bk && oi < bi)) {
                bk = ok;
                bi = oi;
            }
        }
        if (lane == 0) {
            redd[wv] = bk;
            redi[wv] = bi;
        }
        bar();
        bk = redd[0];
        bi = redi[0];
#pragma unroll
        for (int w = 1; w < NW; w++)
            if (redd[w] < bk || (redd[w] == bk && redi[w] < bi)) {
                bk = redd[w];
                bi = redi[w];
            }
        bi = uni(bi);
        if (bk > 0.0 && bk < INFINITY) {  // a positive tree edge (bk == inf: a new component)
            sum += -(bk / scale) - lsc;
            npos++;
        }
        const double *row = cost + (size_t)mem[bi] * N;
        for (int i = tid; i < m; i += NT) {
            if (i == bi) {
                key[i] = -1.0;
            } else {
                const double k = key[i];
                if (k >= 0.0) {
                    const double c = row[mem[i]];
                    if (c < k) key[i] = c;
                }
            }
        }
        bar();
    }
    double r;
    if (npos > 0) r = sum / (double)npos;
    else r = -lsc;
    return uni(r);
}

// Normalised operator probabilities -> cumulative table (numpy choice(p), mcmc_generative.py:294).
constexpr int MH_STAT_INTS = 2 * SBZ_N_OPS;  // LDS counters: proposed | accepted
constexpr int MH_SRC_MAX_WAVES = 16;         // waves per chain of the source-mode sampler (max)

// SAMPLE_SOURCE = true sampler (sbz_mh_src.hip): LDS bytes per chain (sources in LDS, or in
// HBM: hbm_sources) and the launch.
size_t mh_src_lds_bytes(const sbz_dims &d, int C, bool hbm_sources = false, bool geo = false, bool stage = false,
                        bool tb = false, int Np = 0, int nw = 8);
int launch_mh_source(sbz_ctx *ctx, int B, const MhArgs &a);

}  // namespace sbz
