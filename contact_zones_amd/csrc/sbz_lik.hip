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
//     sum left to right).  Since round 4 the entries are built with fused multiply-adds
//     (MixTable::prep): an entry may differ from the reference's per-cell value by an ulp, which
//     the 1e-9 tolerance (north_star) covers many times over.
//   * The lane owns SPL sites (4*lane + 256*k + j); their class row offsets live in registers.
//     Observations are stored feature-major (obs_fm[f][site]) as byte offsets x*8, so a cell
//     is one v_add_u32 (row + byte), one ds_read_b64 and one v_mul_f64.
//   * Instead of one fp64 log per cell, the lane multiplies its cells into 4 mantissa/exponent
//     product chains (v_frexp every 4 features) and takes ONE log per chain at the end:
//     sum log(c_i) = log(prod c_i) to ~1e-16 relative.  Products that leave the normal range
//     (zero, tiny or NaN cells) are detected at each renormalisation and the task re-runs with a
//     renormalisation after every factor, which is exact for any double.
//   * The next feature's parameters are loaded into registers before the current feature's
//     gathers (buffer loads, per-feature advance in the scalar offset), so the HBM stream
//     overlaps the LDS/VALU work of the other waves of the CU.
//   * One fp64 partial per task; the chain's last task adds the partials in task order
//     (deterministic, bit-reproducible; finish_chain).
// The kernels the experiments of rounds 1-2 tried and did not adopt (double-buffered,
// wave-specialised, zone-sparse counts / direct, per-cell source select) are described in
// DESIGN.md §3 and live in the git history, not in this library.
#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "sbz_internal.h"

namespace sbz {

namespace {

constexpr double LN2 = 0.69314718055994530941723212145818;
constexpr int WAVE = 64;
constexpr int ZR = 2;        // zone classes per lane held in registers
#ifndef SBZ_MIX_WAVES
#define SBZ_MIX_WAVES 3
#endif
constexpr int MIX_WAVES = SBZ_MIX_WAVES; // launch bound of the dense kernel: waves per SIMD
constexpr int RN = 4;        // product chains checked and renormalised once per RN features
constexpr int GIF = 16;      // table reads in flight per wave (scheduling barrier every GIF)
// Gathers: table reads issued per group before their products (0: one read per multiply, as in
// round 3).  A/B on one box (profiles/r04_gather_groups.txt, us per 256-chain launch): the dense
// kernel at C = 3 is equal within 0.5 % for 0 / 8 / 16 (and at 2 waves per SIMD with 32 reads in
// flight), at C = 2 (cfg5 without families) 59.3 -> 55.5 with 8; the source kernel 121.3 -> 120.0
// with 16.
#ifndef SBZ_LIK_STAGGER
#define SBZ_LIK_STAGGER 0
#endif
#ifndef SBZ_GTREE
#define SBZ_GTREE 8
#endif
#ifndef SBZ_SRC_GTREE
#define SBZ_SRC_GTREE 16
#endif
#ifndef SBZ_LIK_FMA
#define SBZ_LIK_FMA 1  // (A/B only) 0: the table entries in the reference's unfused operation order
#endif

__device__ __forceinline__ void renorm(double &m, int &e) {
    const int ex = __builtin_amdgcn_frexp_exp(m);
    m = __builtin_amdgcn_frexp_mant(m);
    e += ex;
}

// m * 2^e *= v exactly for any v (denormal v too): v is split into its mantissa and exponent
// first, then the product renormalised (the per-factor paths of untamed inputs)
__device__ __forceinline__ void mul_exact(double &m, int &e, double v) {
    e += __builtin_amdgcn_frexp_exp(v);
    m *= __builtin_amdgcn_frexp_mant(v);
    renorm(m, e);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Make this wave's LDS writes visible to its other lanes.  The workgroup is one wave, so no
// s_barrier is needed, and unlike __syncthreads() this does not drain the vector-memory
// counter: the next feature's prefetched loads stay in flight.
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Store a task's partial sum; the chain's last task to finish adds the W partials in task order
// (deterministic, independent of which task finishes last) into out[b] and re-arms the chain's
// ticket for the next launch.
//
// Memory ordering.  This is NOT the HIP/LLVM memory model's release/acquire pattern: it is the
// hand-off MI355X_MICROARCH.md ("Hand-offs measured with sc1 loads in place of the acquire",
// first row) lists as measured-valid on gfx950 / ROCm 7.2, and which that guide states is not an
// architectural guarantee.  Every condition of that row holds here: (1) every load of the
// handed-off bytes is a global sc1 load (relaxed agent-scope atomic load, L1 bypassed), (2) the
// producer stores every byte sc1 (relaxed agent-scope atomic store), (3) the storing lane (the
// only lane that stores) runs s_waitcnt vmcnt(0) before its agent-scope atomic add to the
// chain's one unsharded counter, (4) the consumer is the task whose add returned W-1, and its lanes
// load (one partial each, in parallel) only after that add has returned; buffers come from hipMalloc, one single-wave task per
// workgroup.  The release/acquire form (a release on every ticket add, an acquire on the winner)
// writes back the XCD's L2 once per task: ~1.7 us per fence, measured ~2x the kernel here.
// tests/test_gpu_likelihood.py::test_partials_handoff_stress re-checks the hand-off under uneven
// load across all XCDs; the host re-zeroes the tickets when a launch fails (launch_loglik).
//
// `zw` (source branch): the task saw a selected normalised weight of exactly 0.  The reference
// then returns -inf whatever the other cells hold (model.py:181-182, NaN cells included), so the
// flag travels beside the partials (zflag[b], same sc1 hand-off) and overrides the sum.
//
// Contract: the workgroup is exactly one wave (every caller launches blockDim.x == WAVE) and all
// 64 lanes call this in wave-uniform control flow: the partials are loaded and broadcast with
// __shfl (ds_bpermute), which reads garbage from lanes that did not arrive.
__device__ __forceinline__ void finish_chain(const LikArgs &a, int b, double tot, bool zw = false) {
    const bool leader = threadIdx.x % WAVE == 0;
    if (a.W == 1) {
        if (leader) a.out[b] = zw ? -INFINITY : tot;
        return;
    }
    double *pb = a.partial + (size_t)b * a.W;
    unsigned prev = 0;
    if (leader) {
        __hip_atomic_store(&pb[blockIdx.x], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (zw) __hip_atomic_store(&a.zflag[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        prev = __hip_atomic_fetch_add(&a.ticket[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    prev = __shfl(prev, 0, WAVE);
    if (prev != (unsigned)a.W - 1) return;
    asm volatile("" ::: "memory");
    // the W partials loaded by the wave's lanes at once (one round trip, not W), then added in
    // task order as before: s = ((0 + p0) + p1) + ..., bit-identical for any W
    const int lane = threadIdx.x % WAVE;
    double s = 0.0;
    for (int t0 = 0; t0 < a.W; t0 += WAVE) {
        const double v = t0 + lane < a.W
                             ? __hip_atomic_load(&pb[t0 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : 0.0;
        const int n = min(WAVE, a.W - t0);
        for (int i = 0; i < n; i++) s += __shfl(v, i, WAVE);
    }
    if (!leader) return;
    if (a.zflag != nullptr && __hip_atomic_load(&a.zflag[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        s = -INFINITY;
        __hip_atomic_store(&a.zflag[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    a.out[b] = s;
    __hip_atomic_store(&a.ticket[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A normalised weight is "tame" if it is 0 or in [2^-60, 2^60]; an untamed one switches its
// feature to per-factor renormalisation.
__device__ __forceinline__ bool tame(double v) { return v == 0.0 || (v >= 0x1p-60 && v <= 0x1p60); }
__device__ __forceinline__ uint32_t hiword(double v) {
    return (uint32_t)((unsigned long long)__double_as_longlong(v) >> 32);
}

// ---------------------------------------------------------------------------------------
// Mixture tables.  Requires S + 1 <= 64, Z + 1 <= ZR * (64 / (S + 1)), Fam <= FR and
// (Z+1)(Fam+1) + 1 <= 256 (checked on the host; otherwise lik_mixture_generic_kernel runs).
//
// A task is (chain b, features [fa, fb)).  Two LDS layouts:
//   packed  T[ncls + 1][S1] doubles, class = zc*FamC + fc (rows 0..FamC-1, zc = 0, are the
//           no-zone classes T0[fc][x]); the last row is neutral (1.0); then 64 junk slots
//           (writes of lanes without an entry) and the normalised weights.
//   banked  (S + 1 <= 16) 256-B LDS lines, one line per LDS bank sweep (64 banks x 4 B).  The
//           no-zone rows T0[fc] (read by ~80 % of the sites, mostly one family per 32-lane group
//           after the family sort) own slots [0, S1) of lines 0 .. FamC-1; every zone row
//           (zc, fc) has a line of its own and sits in slots [S1, 2 S1) or [32 - S1, 32) by zone
//           parity, so a zoned lane never lands on a bank the group's hot row uses, and zoned
//           lanes of different zones spread over both halves.  Line FamC slots [0, S1) hold the
//           neutral row (padding sites), lines FamC+1.. slots [0, S1) the junk slots.  Simulated
//           on the bench data: 3.3 LDS cycles per ds_read_b64 against 4.1 packed.
// Lane (lx = lane % S1, lg = lane / S1) builds the entries of state x = lx for the zone
// classes zc = lg + i*G, i < ZR (G = 64 / S1), every family class.  It loads exactly the
// parameters those entries need (p_global[f][x], p_zones[zc-1][f][x], p_fam[fm][f][x]) straight
// into registers one feature ahead, as buffer loads whose per-feature (and per-family) advance is
// the scalar offset.  The NA column's lanes, and the zone loads of the no-zone class, use an
// out-of-range offset: the load returns 0, and adding `naone` (1 on the NA column, else 0) gives
// the reference's lh of 1 for NA cells (model.py:247) and 0 for the zone lh outside every zone,
// with no selects (p + 0 == p for every p but -0).  Every global load is unconditional (indices
// clamped): a load under a branch makes the compiler's vmcnt bookkeeping conservative at the
// join, and a feature's gathers would then wait for the next feature's loads.
// ---------------------------------------------------------------------------------------
__host__ __device__ constexpr int bk_lines(int Z, int FamC, int S1) {
    return Z * FamC > FamC + 1 + (WAVE + S1 - 1) / S1 ? Z * FamC : FamC + 1 + (WAVE + S1 - 1) / S1;
}
// first double of row (zc, fc), zc = zone + 1 (0 = no zone)
// SBZ_BK_ROT=1 (A/B): zone z's rows start at slot S1 + z mod (33 - 2 S1) instead of the two
// parity offsets, so build()'s writes (lanes of one state x, different zones) and the gathers of
// zoned lanes of different zones land on different banks.
#ifndef SBZ_BK_ROT
#define SBZ_BK_ROT 0
#endif
__host__ __device__ __forceinline__ uint32_t bk_row(int zc, int fc, int FamC, int S1) {
#if SBZ_BK_ROT
    return zc == 0 ? (uint32_t)fc * 32u
                   : (uint32_t)(((zc - 1) * FamC + fc) * 32 + S1 + (zc - 1) % (33 - 2 * S1));
#else
    return zc == 0 ? (uint32_t)fc * 32u
                   : (uint32_t)(((zc - 1) * FamC + fc) * 32 + S1 + ((zc - 1) & 1) * (32 - 2 * S1));
#endif
}

// One feature's parameters as one lane needs them (the weights come from MixTable::prep).
template <int C, int FR>
struct MixParams {
    double g;       // p_global[f][lxc]
    double z[ZR];   // p_zones[zc_i - 1][f][lxc]
    double fm[FR];  // p_fam[fm][f][lxc]
};

// Per feature, h = hz | hf << 1: (c0, c1) of h at [2h, 2h + 1]; c2 of h at 8 + 2 * hz + hf, so
// c2 of (h, h + 2) is one 16-B pair.  Every read of build() is a ds_read_b128.
constexpr int NW_PER_F = 12;
constexpr int NWC = 32;  // features per normalised-weight batch (packed layout)

template <int C, int FR, bool BK>
struct MixTable {
    // features per normalised-weight batch: 16 in the banked layout, so that 12 tasks per CU
    // (3 waves per SIMD) fit the 160 KiB of LDS at the bench shape
    static constexpr int NWCT = BK ? 16 : NWC;
    int lane, S, S1, FamC, Z, Fam, ncls, G, lx, lg;
    uint32_t lxc;
    bool na;
    uint32_t zfs;
    unsigned char *lds;
    double *tab, *junk;
    double *nwt;       // [NWCT][NW_PER_F] normalised weights of features nwf0 .. nwf0 + NWCT
    int nwf0;          // first feature of the weights in nwt (wave-uniform)
    uint64_t nwbad;    // bits 2k, 2k+1: feature nwf0 + k has an untamed normalised weight
    int hz0;           // has-zone flag of the lane's slot-0 class (lg > 0)
    const double *wb;
    __amdgpu_buffer_rsrc_t rg, rz, rf;
    uint32_t vg_off, vz_off[ZR];
    double naone;

    __device__ __forceinline__ MixTable(const LikArgs &a, unsigned char *lds_, int b) : lds(lds_) {
        lane = threadIdx.x % WAVE;
        S = a.S;
        S1 = a.S + 1;
        FamC = a.FamC;
        Z = a.Z;
        Fam = (C == 3) ? a.Fam : 0;
        ncls = (Z + 1) * FamC;
        G = WAVE / S1;
        lx = lane % S1;
        lg = lane / S1;
        na = lx == S;
        lxc = (uint32_t)min(lx, S - 1);  // the NA column and idle lanes read state 0
        tab = reinterpret_cast<double *>(lds);
        if (BK) {
            junk = tab + (FamC + 1 + lane / S1) * 32 + lane % S1;
            nwt = tab + bk_lines(Z, FamC, S1) * 32;
        } else {
            double *dyn = tab + (ncls + 1) * S1;
            junk = dyn + lane;
            nwt = dyn + WAVE + (((ncls + 1) * S1) & 1);  // 16-B aligned (one pad slot budgeted)
        }
        nwf0 = -(1 << 30);
        nwbad = 0;
        hz0 = lg > 0 ? 1 : 0;
        zfs = (uint32_t)(a.F * S);
        const double *pgb = a.pg + (size_t)b * zfs;
        const double *zbase = Z > 0 ? a.pz + (size_t)b * Z * zfs : pgb;
        const double *fbase = Fam > 0 ? a.pf + (size_t)b * Fam * zfs : pgb;
        wb = a.w + (size_t)b * a.F * C;
        constexpr uint32_t OOB = 0x80000000u;  // beyond every buffer: the load returns 0
        vg_off = na ? OOB : lxc * 8u;
#pragma unroll
        for (int i = 0; i < ZR; i++) {
            const uint32_t pzo = (uint32_t)(max(min(lg + i * G, Z), 1) - 1) * zfs + lxc;
            vz_off[i] = (na || lg + i * G == 0) ? OOB : pzo * 8u;
        }
        naone = na ? 1.0 : 0.0;
        rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(pgb), (short)0, (int)(zfs * 8u), 0x00020000);
        rz = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(zbase), (short)0,
                                               (int)((uint32_t)max(Z, 1) * zfs * 8u), 0x00020000);
        rf = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(fbase), (short)0,
                                               (int)((uint32_t)max(Fam, 1) * zfs * 8u), 0x00020000);
        for (int x = lane; x < S1; x += WAVE) tab[(BK ? FamC * 32 : ncls * S1) + x] = 1.0;  // neutral row
    }

    __device__ __forceinline__ void load(int f, MixParams<C, FR> &r) const {
        const int so = (int)((uint32_t)f * (uint32_t)S * 8u);
        r.g = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rg, (int)vg_off, so, 0));
#pragma unroll
        for (int i = 0; i < ZR; i++)
            r.z[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rz, (int)vz_off[i], so, 0));
#pragma unroll
        for (int fm = 0; fm < FR; fm++)
            r.fm[fm] = __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(
                            rf, (int)vg_off, so + (int)((uint32_t)min(fm, max(Fam - 1, 0)) * zfs * 8u), 0));
    }

    // normalize_weights (model.py:451-452): w*has / ((w0*h0 + w1*h1) + w2*h2) for the 4 classes
    // h = hz | hf << 1 of features f0 .. f0 + NWCT (clamped to fb - 1), into nwt.  Lane 2k + hp
    // computes feature k's h = 2hp and 2hp + 1 (one division per weight, as the reference).
    // The weights of the next batch are loaded one batch ahead (prep_issue), so prep does not
    // wait a memory round trip; a batch other than the one in flight loads on the spot.
    double pw0 = 0.0, pw1 = 0.0, pw2 = 0.0;
    int pwf0 = -(1 << 30);
    __device__ __forceinline__ void prep_issue(int f0, int fb) {
        const uint32_t f = (uint32_t)min(f0 + (lane >> 1), fb - 1);
        pw0 = wb[f * C];
        pw1 = wb[f * C + 1];
        pw2 = C == 3 ? wb[f * C + 2] : 0.0;
        pwf0 = f0;
    }
    __device__ __forceinline__ void prep(int f0, int fb) {
        const int k = lane >> 1, hp = lane & 1;
        if (pwf0 != f0) prep_issue(f0, fb);
        const double w0r = pw0, w1r = pw1, w2r = pw2;
        prep_issue(f0 + NWCT, fb);
        int ok = 1;
        double n[2][3];
#pragma unroll
        for (int hz = 0; hz < 2; hz++) {
            const double hzf = hz ? 1.0 : 0.0, hff = hp ? 1.0 : 0.0;
            const double w0 = w0r * 1.0, w1 = w1r * hzf;
            double sum = w0 + w1, w2 = 0.0;
            if (C == 3) {
                w2 = w2r * hff;
                sum = sum + w2;
            }
            n[hz][0] = w0 / sum;
            n[hz][1] = w1 / sum;
            n[hz][2] = C == 3 ? w2 / sum : 0.0;
            ok &= (int)tame(n[hz][0]) & (int)tame(n[hz][1]) & (int)tame(n[hz][2]);
        }
        wave_lds_sync();  // earlier features' reads of nwt are done
        double *o = nwt + k * NW_PER_F;  // h = 2hp + hz
        if (NWCT == 32 || k < NWCT) {
#pragma unroll
            for (int hz = 0; hz < 2; hz++) {
                o[2 * (2 * hp + hz)] = n[hz][0];
                o[2 * (2 * hp + hz) + 1] = n[hz][1];
                o[8 + 2 * hz + hp] = n[hz][2];
            }
        }
        nwbad = __ballot(!ok);
        nwf0 = f0;
        wave_lds_sync();
    }

    // The table of feature f (its weights in nwt: nwf0 <= f < nwf0 + NWCT).  Returns `wide`:
    // some input is not tame, so products over this feature must renormalise after every factor.
    __device__ __forceinline__ bool build(const MixParams<C, FR> &r, int f) const {
        const int k = f - nwf0;
        // every parameter in [0, 1 + 2^-20): unsigned high words <= hi(1.0) (a sign bit, NaN or
        // inf fails).  Table entries are then <= ~1, so a product never overflows, and one that
        // underflows stays below 2^-1022 until the feature's check (see lik_mixture_kernel).
        uint32_t hmx = hiword(r.g);
#pragma unroll
        for (int i = 0; i < ZR; i++) hmx = max(hmx, hiword(r.z[i]));
#pragma unroll
        for (int fm = 0; fm < FR; fm++) hmx = max(hmx, hiword(r.fm[fm]));
        const bool wide = ((nwbad >> (2 * k)) & 3ull) != 0 || __ballot(hmx > 0x3FF00000u) != 0;
        // 1. normalised weights from nwt.  Slot i >= 1 holds zone classes only (zc >= G >= 1):
        //    wave-uniform weights of h = 1 (no family) and h = 3 (family).  Slot 0 mixes zc = 0
        //    (lanes lg == 0, h = 0 / 2) and zone classes (h = 1 / 3).
        //    Six 16-B reads: (c0, c1) of each h, and c2 of (h, h + 2) as one pair.
        const double *nk = static_cast<const double *>(__builtin_assume_aligned(nwt + k * NW_PER_F, 16));
        auto pair = [&](int at) { return *reinterpret_cast<const double2 *>(nk + at); };
        double u[2][3], p[2][3];
        const double2 cu = pair(10), cp = pair(8 + 2 * hz0);  // c2 of (h, h + 2), hz = 1 / hz0
#pragma unroll
        for (int hf = 0; hf < 2; hf++) {
            if (C == 2 && hf == 1) {
#pragma unroll
                for (int cc = 0; cc < 3; cc++) u[hf][cc] = p[hf][cc] = 0.0;
                continue;
            }
            const double2 a = pair(2 * (1 + 2 * hf)), q = pair(2 * (hz0 + 2 * hf));
            u[hf][0] = a.x;
            u[hf][1] = a.y;
            u[hf][2] = C == 3 ? (hf ? cu.y : cu.x) : 0.0;
            p[hf][0] = q.x;
            p[hf][1] = q.y;
            p[hf][2] = C == 3 ? (hf ? cp.y : cp.x) : 0.0;
        }
        // 2. table: the reference cell (n0*l0 + n1*l1) + n2*l2 for every class.  Branch-free:
        //    lanes without an entry write to their junk slot.  The family term of a class
        //    without family is n2 * l2 = (w2 * 0 / sum) * (0 or 1): +0 for tame inputs, left
        //    out then (x + 0 == x); kept for untamed ones, where it may be NaN.
        wave_lds_sync();
        const double l0 = r.g + naone;
#pragma unroll
        for (int i = 0; i < ZR; i++) {
            const int zc = lg + i * G;
            const bool valid = (lane < G * S1) && (zc <= Z);
            const double n00 = i == 0 ? p[0][0] : u[0][0], n01 = i == 0 ? p[0][1] : u[0][1];
            // zone lh: 0 for a site outside every zone (model.py:241-247), 1 for NA
            const double l1 = r.z[i] + naone;
            double *row = valid ? tab + (BK ? bk_row(zc, 0, FamC, S1) : (uint32_t)(zc * FamC * S1)) + lx : junk;
            const int rs = valid ? (BK ? 32 : S1) : 0;
            // fused multiply-adds: each entry within an ulp of the reference's per-cell value
            // (north_star's tolerance is 1e-9 relative on the log-likelihood)
#if SBZ_LIK_FMA
            double v = __builtin_fma(n01, l1, n00 * l0);
            if (C == 3 && wide) v = __builtin_fma(i == 0 ? p[0][2] : u[0][2], naone, v);
#else
            double v = n00 * l0 + n01 * l1;
            if (C == 3 && wide) v = v + (i == 0 ? p[0][2] : u[0][2]) * naone;
#endif
            row[0] = v;
            if (C == 3) {
                const double n10 = i == 0 ? p[1][0] : u[1][0], n11 = i == 0 ? p[1][1] : u[1][1];
                const double n12 = i == 0 ? p[1][2] : u[1][2];
#if SBZ_LIK_FMA
                const double a1 = __builtin_fma(n11, l1, n10 * l0);
#pragma unroll
                for (int fm = 0; fm < FR; fm++) {
                    double *dst = fm < Fam ? row + (fm + 1) * rs : junk;  // families past Fam: junk
                    *dst = __builtin_fma(n12, r.fm[fm] + naone, a1);
                }
#else
                const double a1 = n10 * l0 + n11 * l1;
#pragma unroll
                for (int fm = 0; fm < FR; fm++) {
                    double *dst = fm < Fam ? row + (fm + 1) * rs : junk;
                    *dst = a1 + n12 * (r.fm[fm] + naone);
                }
#endif
            }
        }
        wave_lds_sync();
        return wide;
    }

    __device__ __forceinline__ double at(uint32_t byte_addr) const {
        return *reinterpret_cast<const double *>(lds + byte_addr);
    }
};

// ---------------------------------------------------------------------------------------
// Dense mixture kernel: every site of the task is gathered from the table.
// The lane owns SPL sites (4*lane + 256*k + j); their class row offsets (bytes, < 64 KiB) live
// in registers, two per register.  Parameters and observations run one feature ahead (two
// register sets, P / O[f & 1]).
// ---------------------------------------------------------------------------------------
template <int C, int SPL, int FR, bool XS8, bool BK>
__global__ __launch_bounds__(WAVE, MIX_WAVES) void lik_mixture_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int NO = SPL / 4;  // observation words (4 sites each) per lane per feature
    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    MixTable<C, FR, BK> t(a, lds, b);
    const __amdgpu_buffer_rsrc_t robs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.obs_fm), (short)0, a.F * a.Np, 0x00020000);
    auto load_obs = [&](int f, int c0, uint32_t (&o)[NO]) {
#pragma unroll
        for (int k = 0; k < NO; k++)  // one lane offset; the word index goes to the scalar offset
            o[k] = __builtin_amdgcn_raw_buffer_load_b32(robs, lane * 4, f * a.Np + c0 + 256 * k, 0);
    };

    double m[4];  // independent product chains
    int e;
    // A lane's product fell below 2^-1022 (a zero or tiny cell): the wave re-runs the task with
    // per-factor renormalisation (`force`), which is exact for any normal double.
    uint64_t under;
    bool force = false;
    uint32_t base2[SPL / 2];  // per-site class row offsets (bytes, < 64 KiB), two per register
    MixParams<C, FR> P[2];    // parameter sets: feature f uses P[(f - fa) & 1]
    uint32_t O[2][NO];        // observation sets, same rotation

    // The product chains since the last check; every factor is <= ~1, so a product that left
    // the normal range is still below it here.  Then renormalise.
    auto flush = [&]() {
        const double mn = fmin(fmin(m[0], m[1]), fmin(m[2], m[3]));
        under |= __ballot(!(mn >= 0x1p-1022));
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (q < NO) renorm(m[q], e);
    };

    // One feature: build its table from `cur`, issue the loads of feature f + 1 into `fill` (the
    // sets feature f - 1 used), gather.  `live` = false for the padding feature.
    auto feature = [&](int f, int c0, bool live, const MixParams<C, FR> &cur, const uint32_t (&ob)[NO],
                       MixParams<C, FR> &fill, uint32_t (&ofill)[NO]) {
        const int fk = min(f, fb - 1);
        if (fk < t.nwf0 || fk >= t.nwf0 + t.NWCT) t.prep(fk, fb);  // uniform, once per NWCT features
        const bool wide = t.build(cur, fk) || force;
        __builtin_amdgcn_sched_barrier(0);
        t.load(min(f + 1, fb - 1), fill);
        load_obs(min(f + 1, fb - 1), c0, ofill);
        if (!live) return;
        auto cell_at = [&](int i) {  // cell i = 4k + j of the lane
            const int k = i >> 2, j = i & 3;
            const uint32_t bw = base2[2 * k + (j >> 1)];
            const uint32_t bs = (j & 1) ? (bw >> 16) : (bw & 0xffffu);
            const uint32_t xb = (ob[k] >> (8 * j)) & 0xffu;
            return bs + (XS8 ? xb : (xb << 3));
        };
        if (!wide) {
#if SBZ_GTREE
            if constexpr (SPL >= 8) {
                // groups of GT table reads issued back to back (sched_group_barrier: left alone,
                // the compiler interleaves each read with its multiply and a wait, ~4 reads in
                // flight), each half of a group multiplied as a tree into chains 2q and 2q + 1
                constexpr int GT = SPL < SBZ_GTREE ? SPL : SBZ_GTREE, H = GT / 2;
#pragma unroll
                for (int g = 0; g < SPL; g += GT) {
                    double v[GT];
#pragma unroll
                    for (int i = 0; i < GT; i++) v[i] = t.at(cell_at(g + i));
                    __builtin_amdgcn_sched_group_barrier(0x0100, GT, 0);  // the GT DS reads first
#pragma unroll
                    for (int h = H / 2; h >= 1; h >>= 1)
#pragma unroll
                        for (int i = 0; i < h; i++) {
                            v[i] = v[i] * v[i + h];
                            v[H + i] = v[H + i] * v[H + i + h];
                        }
                    m[(2 * (g / GT)) & 3] *= v[0];
                    m[(2 * (g / GT) + 1) & 3] *= v[H];
                    __builtin_amdgcn_sched_barrier(0);
                }
            } else
#endif
            {
#pragma unroll
                for (int k = 0; k < NO; k++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        m[k & 3] *= t.at(cell_at(4 * k + j));
                        // <= GIF reads in flight
                        if (j == 3 && (k & (GIF / 4 - 1)) == GIF / 4 - 1) __builtin_amdgcn_sched_barrier(0);
                    }
            }
            if ((f - fa) % RN == RN - 1) flush();
        } else {
            // untamed inputs: renormalise after every factor (exact for any normal double)
            flush();  // the products since the last check first
#pragma unroll
            for (int i = 0; i < SPL; i++) mul_exact(m[0], e, t.at(cell_at(i)));
        }
    };

#if SBZ_LIK_STAGGER
    // A/B of the phase-lock hypothesis: tasks of odd slot start SBZ_LIK_STAGGER x 1024 cycles late
    if (blockIdx.x & 1)
        for (int i = 0; i < SBZ_LIK_STAGGER; i++) __builtin_amdgcn_s_sleep(16);
#endif
    for (;;) {
        for (int q = 0; q < 4; q++) m[q] = 1.0;
        e = 0;
        under = 0;
        for (int c0 = 0; c0 < a.Np; c0 += SPL * WAVE) {
            // classes of this chunk's sites (cls = zc*FamC + fc, padding -> the neutral row); the
            // first feature's parameters and observations
            const uint8_t *zb = a.zone + (size_t)b * a.N;
            uint32_t zs[SPL];
            int4 pv[NO];
            uint32_t fw[NO];
#pragma unroll
            for (int k = 0; k < NO; k++) {
                const uint32_t p0 = (uint32_t)(c0 + 4 * lane + 256 * k);  // < Np (arrays padded)
                pv[k] = *reinterpret_cast<const int4 *>(a.perm + p0);
                fw[k] = *reinterpret_cast<const uint32_t *>(a.famc + p0);
            }
#pragma unroll
            for (int k = 0; k < NO; k++) {
                zs[4 * k + 0] = zb[(uint32_t)pv[k].x];
                zs[4 * k + 1] = zb[(uint32_t)pv[k].y];
                zs[4 * k + 2] = zb[(uint32_t)pv[k].z];
                zs[4 * k + 3] = zb[(uint32_t)pv[k].w];
            }
            t.load(fa, P[0]);
            load_obs(fa, c0, O[0]);
            if (t.pwf0 != fa) t.prep_issue(fa, fb);  // the first weights, with the zone bytes
#pragma unroll
            for (int i = 0; i < SPL; i++) {
                const int pos = c0 + 4 * lane + 256 * (i / 4) + (i % 4);
                const int z = (int)zs[i];
                const int fc = (int)((fw[i / 4] >> (8 * (i % 4))) & 0xffu);
                const int zc = z < t.Z ? z + 1 : 0;
                uint32_t off;
                if (BK) off = 8u * (pos < a.N ? bk_row(zc, fc, t.FamC, t.S1) : (uint32_t)(t.FamC * 32));
                else off = (uint32_t)((pos < a.N ? zc * t.FamC + fc : t.ncls) * t.S1 * 8);
                if (i & 1) base2[i >> 1] |= off << 16;
                else base2[i >> 1] = off;
            }
            for (int f = fa; f < fb; f += 2) {
                feature(f, c0, true, P[0], O[0], P[1], O[1]);
                feature(f + 1, c0, f + 1 < fb, P[1], O[1], P[0], O[0]);
            }
        }
        flush();
        if (force || under == 0) break;
        force = true;  // uniform: `under` is a ballot
    }
    const double v = ((log(m[0]) + log(m[1])) + (log(m[2]) + log(m[3]))) + (double)e * LN2;
    finish_chain(a, b, wave_sum(v));
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
    for (int s = lane; s < a.N; s += WAVE) {  // s: position in the family-sorted site order
        const int z = zb[a.perm[s]];
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
    finish_chain(a, b, tot);
}


// ---------------------------------------------------------------------------------------
// Source kernel, generic path (any S, Z, Fam within the ABI limits, and the SBZ_SRC_RC=0
// check): one lane per site, the cell w_norm[src] * l_src computed directly from the
// parameters in the reference's operation order (model.py:436-452, 241-247) and the caller's
// source bytes ([B][N][F] or [B][F][Np]) read in place, one log per cell.  A selected weight of
// exactly 0 sets the chain's -inf flag (model.py:181-182).
// ---------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(WAVE) void lik_source_generic_kernel(LikArgs a) {
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
    // the caller's sources: [B][N][F] by site, or [B][F][Np] by position
    const uint8_t *sb = a.src_pm ? a.src_pm + (size_t)b * a.F * a.Np : a.src_rm + (size_t)b * a.N * a.F;
    const int div = a.xs8 ? 8 : 1;
    double lsum = 0.0;
    uint32_t zw = 0;
    for (int s = lane; s < a.N; s += WAVE) {  // s: position in the family-sorted site order
        const int site = a.perm[s];
        const int z = zb[site];
        const bool hz = z < Z;
        const int fc = (C == 3) ? a.famc[s] : 0;
        const bool hf = fc > 0;
        for (int f = fa; f < fb; f++) {
            const int x = a.obs_fm[(size_t)f * a.Np + s] / div;
            const bool na = x == S;
            const int c = a.src_pm ? sb[(size_t)f * a.Np + s] : sb[(size_t)site * a.F + f];
            const double w0 = wb[(size_t)f * C] * 1.0;
            const double w1 = wb[(size_t)f * C + 1] * (hz ? 1.0 : 0.0);
            double sum = w0 + w1, w2 = 0.0;
            if (C == 3) {
                w2 = wb[(size_t)f * C + 2] * (hf ? 1.0 : 0.0);
                sum = sum + w2;
            }
            double wsel, lsel;
            if (c == 0) {
                wsel = w0 / sum;
                lsel = na ? 1.0 : pgb[(size_t)f * S + x];
            } else if (c == 1) {
                wsel = w1 / sum;
                lsel = na ? 1.0 : (hz ? pzb[(size_t)z * zfs + (size_t)f * S + x] : 0.0);
            } else {
                wsel = w2 / sum;
                lsel = na ? 1.0 : (hf ? pfb[(size_t)(fc - 1) * zfs + (size_t)f * S + x] : 0.0);
            }
            zw |= wsel == 0.0 ? 1u : 0u;
            lsum += log(wsel * lsel);
        }
    }
    const double tot = wave_sum(lsum);
    finish_chain(a, b, tot, __ballot(zw != 0) != 0);
}

// ---------------------------------------------------------------------------------------
// Source kernel, table form (lik_source_rc_kernel; the default where it applies).  Rows (each S1
// doubles): T0[h] (h = hz | hf << 1, w_norm[h][0] * l0) 0..3, T1[z][hf] (w_norm[1|hf<<1][1] * l1)
// from 4, T2[fam][hz] (w_norm[2|hz][2] * l2) from 4 + 2Z, the zero rows Z0[h] of a selected
// component the site lacks (weight w_c * 0 / sum_h, lh 0), the neutral row rn (padding).
//
// The sources come POSITION-MAJOR, [B][F][Np] component bytes in the context's family-sorted
// site order (sbz_loglik_batch_device_pm; the sampler keeps them so), read in place with the
// observations' layout: one dword = 4 positions of one feature.  A cell's table row depends on
// its component c and its site's class only, so per chunk each lane holds, for each of its
// 4-position groups, three ROW-MAP words M_c (byte j = the row of component c at position j of
// the group); per feature the group's row word is two v_perm_b32 byte selects of its source word:
// bit 0 of each c picks M0 / M1, bit 1 then picks M2 (c <= 2).  A cell then costs one
// multiply-add for its address (row * row_bytes + x * 8), one ds_read_b64 and one v_mul_f64.
// Per feature each lane loads (buffer loads, scalar per-feature offsets, one feature ahead)
// p_global[x], the p_zones rows lg, lg + G and the p_families rows lg, lg + G of its state
// x = lane % S1 (NA lanes read out of range: 0, plus `naone` = 1), and writes T0[h] and Z0[h]
// (h = lg, lg + G, .. < 4), the two T1 rows of each zone and the two T2 rows of each family.
// Normalised weights come from per-batch LDS (prep).  Inputs are checked as in the dense kernel
// (one unsigned max; products checked when renormalised, the task re-run per factor when one
// left the normal range, e.g. a zero weight's -inf cell).
// ---------------------------------------------------------------------------------------
constexpr int SRC_NWC = 32;  // features per normalised-weight batch
#ifndef SBZ_SRC_RC_WAVES
#define SBZ_SRC_RC_WAVES 2  // launch bound: waves per SIMD (3 spills: 262 vs 246 us per launch)
#endif
// PK: the sources come as 2-bit planes (source_to_pk_kernel, the by-site entry): per feature row
// and lane, one dword pair (lo, hi) per 8 position groups, bit 8 j + kk of lo / hi = bit 0 / 1 of
// the component at position 4 lane + 256 (8 kb + kk) + j of the chunk; pair (chunk, kb, lane) at
// byte ((chunk * NOB + kb) * 64 + lane) * 8 of the row (a.pk_row bytes).  A quarter of the bytes
// the by-position layout streams, and the same two selector words per group.
template <int C, int SPL, bool XS8, bool PK = false>
__global__ __launch_bounds__(WAVE, SBZ_SRC_RC_WAVES) void lik_source_rc_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int NO = SPL / 4;
    constexpr int KP = NO < 8 ? NO : 8;  // PK: position groups per dword pair
    constexpr int NOB = NO / KP;         // PK: dword pairs per lane, feature and chunk
    static_assert(!PK || NO >= 4, "2-bit planes need 16 sites per lane or more");
    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    if (fa >= fb) {
        finish_chain(a, b, 0.0);
        return;
    }
    const int S = a.S, S1 = a.S + 1, Z = a.Z;
    const int Fam = (C == 3) ? a.Fam : 0;
    const int off1 = 4, off2 = 4 + 2 * Z, rz = off2 + 2 * Fam, rn = rz + 4;
    const uint32_t row_bytes = (uint32_t)S1 * 8u;
    double *tab = reinterpret_cast<double *>(lds);
    double *nwt = tab + ((((rn + 1) * S1) + 1) & ~1);  // [SRC_NWC][8], 16-B aligned
    double *junk = nwt + SRC_NWC * 8 + lane;
    // zrow[r] = 1: the weight of row r is exactly 0 (written for `wide` features and read by their
    // per-factor gathers: the reference's any(weight == 0) -> -inf, model.py:181-182).  A zero
    // weight in a fast-path feature gives a zero product, which re-runs the task per factor.
    uint8_t *zrow = reinterpret_cast<uint8_t *>(nwt + SRC_NWC * 8 + WAVE);

    const int G = WAVE / S1, lx = lane % S1, lg = lane / S1;
    const bool na = lx == S, act = lane < G * S1;
    const uint32_t lxc = (uint32_t)min(lx, S - 1);
    const uint32_t zfs = (uint32_t)(a.F * S);
    const double naone = na ? 1.0 : 0.0;
    constexpr uint32_t OOB = 0x80000000u;
    const double *pgb = a.pg + (size_t)b * zfs;
    const double *zbase = Z > 0 ? a.pz + (size_t)b * Z * zfs : pgb;
    const double *fbase = Fam > 0 ? a.pf + (size_t)b * Fam * zfs : pgb;
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(pgb), (short)0, (int)(zfs * 8u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rzr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(zbase), (short)0,
                                                                         (int)((uint32_t)max(Z, 1) * zfs * 8u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(fbase), (short)0,
                                                                        (int)((uint32_t)max(Fam, 1) * zfs * 8u), 0x00020000);
    const __amdgpu_buffer_rsrc_t robs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.obs_fm), (short)0,
                                                                          a.F * a.Np, 0x00020000);
    const int src_row = PK ? a.pk_row : a.Np;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.src_pm + (size_t)b * a.F * src_row), (short)0, a.F * src_row, 0x00020000);
    // lane offsets (bytes) of its parameter rows; rows past Z / Fam read a valid row (unused)
    const uint32_t vg = na ? OOB : lxc * 8u;
    uint32_t vz[2], vf[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
        vz[i] = na ? OOB : ((uint32_t)min(lg + G * i, max(Z - 1, 0)) * zfs + lxc) * 8u;
        vf[i] = na ? OOB : ((uint32_t)min(lg + G * i, max(Fam - 1, 0)) * zfs + lxc) * 8u;
    }
    struct SrcParams {
        double g, z[2], fm[2];
    };
    auto load = [&](int f, SrcParams &r) {
        const int so = f * S * 8;
        r.g = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rg, (int)vg, so, 0));
#pragma unroll
        for (int i = 0; i < 2; i++) {
            r.z[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rzr, (int)vz[i], so, 0));
            r.fm[i] = C == 3 ? __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rf, (int)vf[i], so, 0)) : 0.0;
        }
    };
    auto load_words = [&](const __amdgpu_buffer_rsrc_t &rs, int f, int c0, uint32_t (&o)[NO]) {
#pragma unroll
        for (int k = 0; k < NO; k++) o[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, f * a.Np + c0 + 256 * k, 0);
    };
    // the sources of feature f in the chunk at c0: NO words (by position) or NOB (lo, hi) pairs
    auto load_src = [&](int f, int c0, uint32_t (&o)[NO]) {
        if constexpr (PK) {
            const int cb = c0 / (SPL * WAVE);
#pragma unroll
            for (int kb = 0; kb < NOB; kb++) {
                const unsigned long long v = __builtin_bit_cast(
                    unsigned long long,
                    __builtin_amdgcn_raw_buffer_load_b64(rsrc, lane * 8, f * a.pk_row + (cb * NOB + kb) * WAVE * 8, 0));
                o[2 * kb] = (uint32_t)v;
                o[2 * kb + 1] = (uint32_t)(v >> 32);
            }
        } else {
            load_words(rsrc, f, c0, o);
        }
    };

    for (int x = lane; x < S1; x += WAVE) tab[rn * S1 + x] = 1.0;  // padding positions
    bool force = false;  // per-factor re-run of the task (uniform)
    uint32_t zw = 0;     // per-factor features: this lane selected a weight of exactly 0
    // normalised weights of features f0 .. f0 + SRC_NWC: [k][q], q = h (w_norm[h][0]), 4 / 5 =
    // w_norm[1 / 3][1], 6 / 7 = w_norm[2 / 3][2]; lane 2k + hp computes feature k's h = 2hp + hz
    int nwf0 = -(1 << 30);
    uint64_t nwbad = 0;
    const double *wb = a.w + (size_t)b * a.F * C;
    auto prep = [&](int f0) {
        const int k = lane >> 1, hp = lane & 1;
        const uint32_t f = (uint32_t)min(f0 + k, fb - 1);
        const double w0r = wb[f * C], w1r = wb[f * C + 1], w2r = C == 3 ? wb[f * C + 2] : 0.0;
        int ok = 1;
        double n[2][3];
#pragma unroll
        for (int hz = 0; hz < 2; hz++) {
            const double w0 = w0r * 1.0, w1 = w1r * (hz ? 1.0 : 0.0);
            double sum = w0 + w1, w2 = 0.0;
            if (C == 3) {
                w2 = w2r * (hp ? 1.0 : 0.0);
                sum = sum + w2;
            }
            n[hz][0] = w0 / sum;
            n[hz][1] = w1 / sum;
            n[hz][2] = C == 3 ? w2 / sum : 0.0;
            ok &= (int)tame(n[hz][0]) & (int)tame(n[hz][1]) & (int)tame(n[hz][2]);
        }
        wave_lds_sync();  // earlier features' reads of nwt are done
        double *o = nwt + k * 8;
        o[2 * hp] = n[0][0];      // h = 2hp
        o[2 * hp + 1] = n[1][0];  // h = 2hp + 1
        o[4 + hp] = n[1][1];      // h = 1 / 3
        if (hp) {
            o[6] = n[0][2];       // h = 2
            o[7] = n[1][2];       // h = 3
        }
        nwbad = __ballot(!ok);
        nwf0 = f0;
        wave_lds_sync();
    };
    // the table of feature f; returns `wide`
    auto build = [&](const SrcParams &r, int f) -> bool {
        const int k = f - nwf0;
        uint32_t hmx = max(hiword(r.g), max(hiword(r.z[0]), hiword(r.z[1])));
        if (C == 3) hmx = max(hmx, max(hiword(r.fm[0]), hiword(r.fm[1])));
        const bool wide = ((nwbad >> (2 * k)) & 3ull) != 0 || __ballot(hmx > 0x3FF00000u) != 0;
        const double *q = nwt + k * 8;
        const double wz0 = q[4], wz1 = q[5], wf0 = q[6], wf1 = q[7];
        wave_lds_sync();  // the previous feature's gathers are done with the table
        const double l0 = r.g + naone;
        // T0[h], h = 0..3, from lane group lg (and lg + G, ... when fewer than 4 groups, S1 > 16),
        // and the zero row of h: a component the site lacks has weight w_c * 0 / sum_h (0, or NaN
        // when sum_h is 0) and lh 0 (model.py:241-247, 436-452)
        for (int h = lg; h < 4; h += G) {
            double *t0 = act ? tab + h * S1 + lx : junk;
            *t0 = q[h] * l0;
            double *t0z = act ? tab + (rz + h) * S1 + lx : junk;
            *t0z = q[h] * 0.0;
        }
        if (wide || force) {  // weights of exactly 0, by table row
            for (int r = lane; r <= rn; r += WAVE) {  // rn: the padding positions' neutral row
                const double wr = r < 4 ? q[r] : r < off2 ? q[4 + ((r - 4) & 1)]
                                : r < rz ? q[6 + ((r - off2) & 1)] : r < rn ? q[r - rz] * 0.0 : 1.0;
                zrow[r] = wr == 0.0 ? 1 : 0;
            }
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int zr = lg + G * i;
            const double l1 = r.z[i] + naone;
            double *tz = (act && zr < Z) ? tab + (off1 + 2 * zr) * S1 + lx : junk;
            const int sz = (act && zr < Z) ? S1 : 0;
            tz[0] = wz0 * l1;
            tz[sz] = wz1 * l1;
            if (C == 3) {
                const double l2 = r.fm[i] + naone;
                double *tf = (act && zr < Fam) ? tab + (off2 + 2 * zr) * S1 + lx : junk;
                const int sf = (act && zr < Fam) ? S1 : 0;
                tf[0] = wf0 * l2;
                tf[sf] = wf1 * l2;
            }
        }
        wave_lds_sync();
        return wide;
    };

    double m[4];
    int e;
    uint64_t under;
    SrcParams P[2];
    uint32_t O[2][NO], R[2][NO];
    uint32_t M0[NO], M1[NO], M2[NO];  // row maps of the lane's position groups (see above)
    // a product that left the normal range (0, tiny, or NaN: fmin would drop a NaN) re-runs the
    // task per factor, where every cell's row is checked for a zero weight
    auto flush = [&]() {
        constexpr double T = 0x1p-1022;
        under |= __ballot(!(m[0] >= T && m[1] >= T && m[2] >= T && m[3] >= T));
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (q < NO) renorm(m[q], e);
    };
    // the 4 table rows of position group k from its 4 component bytes
    auto rows_of = [&](int k, const uint32_t (&sb)[NO]) -> uint32_t {
        uint32_t s0, s1;  // bit 0 / bit 1 of the 4 components, each moved to bit 2 of its byte
        if constexpr (PK) {
            s0 = ((sb[2 * (k / KP)] >> (k % KP)) & 0x01010101u) << 2;
            s1 = ((sb[2 * (k / KP) + 1] >> (k % KP)) & 0x01010101u) << 2;
        } else {
            s0 = (sb[k] & 0x01010101u) << 2;
            s1 = (sb[k] & 0x02020202u) << 1;
        }
        const uint32_t r01 = __builtin_amdgcn_perm(M1[k], M0[k], s0 + 0x03020100u);
        if (C == 2) return r01;
        return __builtin_amdgcn_perm(M2[k], r01, s1 + 0x03020100u);
    };
    auto feature = [&](int f, int c0, bool live, const SrcParams &cur, const uint32_t (&ob)[NO],
                       const uint32_t (&sb)[NO], SrcParams &fill, uint32_t (&ofill)[NO], uint32_t (&sfill)[NO]) {
        const int fk = min(f, fb - 1);
        if (fk < nwf0 || fk >= nwf0 + SRC_NWC) prep(fk);
        const bool wide = build(cur, fk) || force;
        __builtin_amdgcn_sched_barrier(0);
        const int fn = min(f + 1, fb - 1);
        load(fn, fill);
        load_words(robs, fn, c0, ofill);
        load_src(fn, c0, sfill);
        if (!live) return;
        uint32_t rw[NO];
#pragma unroll
        for (int k = 0; k < NO; k++) rw[k] = rows_of(k, sb);
        auto addr = [&](int k, int j) {
            const uint32_t xb = (ob[k] >> (8 * j)) & 0xffu;
            const uint32_t rr = (rw[k] >> (8 * j)) & 0xffu;
            return rr * row_bytes + (XS8 ? xb : (xb << 3));
        };
        if (!wide) {
#if SBZ_SRC_GTREE
            if constexpr (SPL >= 8) {  // grouped reads and tree products, as lik_mixture_kernel
                constexpr int GT = SPL < SBZ_SRC_GTREE ? SPL : SBZ_SRC_GTREE, H = GT / 2;
#pragma unroll
                for (int g = 0; g < SPL; g += GT) {
                    double v[GT];
#pragma unroll
                    for (int i = 0; i < GT; i++)
                        v[i] = *reinterpret_cast<const double *>(lds + addr((g + i) >> 2, (g + i) & 3));
                    __builtin_amdgcn_sched_group_barrier(0x0100, GT, 0);
#pragma unroll
                    for (int h = H / 2; h >= 1; h >>= 1)
#pragma unroll
                        for (int i = 0; i < h; i++) {
                            v[i] = v[i] * v[i + h];
                            v[H + i] = v[H + i] * v[H + i + h];
                        }
                    m[(2 * (g / GT)) & 3] *= v[0];
                    m[(2 * (g / GT) + 1) & 3] *= v[H];
                    __builtin_amdgcn_sched_barrier(0);
                }
            } else
#endif
            {
#pragma unroll
                for (int k = 0; k < NO; k++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        m[k & 3] *= *reinterpret_cast<const double *>(lds + addr(k, j));
                        if (j == 3 && (k & 3) == 3) __builtin_amdgcn_sched_barrier(0);
                    }
            }
            if ((f - fa) % RN == RN - 1) flush();
        } else {
            flush();
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    mul_exact(m[0], e, *reinterpret_cast<const double *>(lds + addr(k, j)));
                    zw |= zrow[(rw[k] >> (8 * j)) & 0xffu];
                }
        }
    };

    for (;;) {
        m[0] = m[1] = m[2] = m[3] = 1.0;
        e = 0;
        under = 0;
        for (int c0 = 0; c0 < a.Np; c0 += SPL * WAVE) {
            // row maps of this chunk's positions: the chain's zone of each site and its family
            // class.  Component c -> T0[h] (c = 0), T1[z][hf] (c = 1, zoned sites), T2[fam][hz]
            // (c = 2, sites with a family), else the zero row of h; padding -> the neutral row.
            const uint8_t *zb = a.zone + (size_t)b * a.N;
            int4 pv[NO];
            uint32_t fw[NO];
#pragma unroll
            for (int k = 0; k < NO; k++) {
                const uint32_t p0 = (uint32_t)(c0 + 4 * lane + 256 * k);  // < Np (arrays padded)
                pv[k] = *reinterpret_cast<const int4 *>(a.perm + p0);
                fw[k] = *reinterpret_cast<const uint32_t *>(a.famc + p0);
            }
            uint32_t zs[NO][4];
#pragma unroll
            for (int k = 0; k < NO; k++) {
                zs[k][0] = zb[(uint32_t)pv[k].x];
                zs[k][1] = zb[(uint32_t)pv[k].y];
                zs[k][2] = zb[(uint32_t)pv[k].z];
                zs[k][3] = zb[(uint32_t)pv[k].w];
            }
            load(fa, P[0]);
            load_words(robs, fa, c0, O[0]);
            load_src(fa, c0, R[0]);
#pragma unroll
            for (int k = 0; k < NO; k++) {
                uint32_t m0 = 0, m1 = 0, m2 = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int pos = c0 + 4 * lane + 256 * k + j;
                    const int z = (int)zs[k][j];
                    const int fc = C == 3 ? (int)((fw[k] >> (8 * j)) & 0xffu) : 0;
                    const bool hz = z < Z, hf = fc > 0;
                    const uint32_t h = (hz ? 1u : 0u) | (hf ? 2u : 0u);
                    const uint32_t rl = (uint32_t)rz + h;  // a component the site lacks
                    uint32_t r0 = h;
                    uint32_t r1 = hz ? (uint32_t)(off1 + 2 * z) + (hf ? 1u : 0u) : rl;
                    uint32_t r2 = hf ? (uint32_t)(off2 + 2 * (fc - 1)) + (hz ? 1u : 0u) : rl;
                    if (pos >= a.N) r0 = r1 = r2 = (uint32_t)rn;
                    m0 |= r0 << (8 * j);
                    m1 |= r1 << (8 * j);
                    m2 |= r2 << (8 * j);
                }
                M0[k] = m0;
                M1[k] = m1;
                M2[k] = m2;
            }
            for (int f = fa; f < fb; f += 2) {
                feature(f, c0, true, P[0], O[0], R[0], P[1], O[1], R[1]);
                feature(f + 1, c0, f + 1 < fb, P[1], O[1], R[1], P[0], O[0], R[0]);
            }
        }
        flush();
        if (force || under == 0) break;
        force = true;  // uniform: `under` is a ballot
    }
    const double v = (log(m[0]) + log(m[1])) + (log(m[2]) + log(m[3])) + (double)e * LN2;
    const double tot = wave_sum(v);
    finish_chain(a, b, tot, __ballot(zw != 0) != 0);
}

// Source layout transposes between the reference layout [B][N][F] (site-major, row s = site s)
// and the position-major layout [B][F][Np] (row f = feature f, column p = site perm[p] of the
// context's family-sorted order; padding columns p >= N hold 0).  One workgroup moves a tile of
// RP_T positions x RP_F features through LDS: on the site-major side RP_F / 16 lanes per site row
// (16 feature bytes each, as 4-byte words when F is a multiple of 4), on the position-major side
// 4 lanes per feature row (16 position bytes each per 64-position subtile, one 16-B access).
// (Tile shapes measured in round 2)
constexpr int RP_T = 256;  // positions per workgroup (a multiple of 64)
constexpr int RP_F = 64;   // features per workgroup (a multiple of 16, RP_F / 16 divides 256)
template <bool TO_PM>
__global__ __launch_bounds__(256) void source_transpose_kernel(int N, int F, int Np, const int *perm,
                                                               const uint8_t *src, uint8_t *dst) {
    constexpr int RW = RP_F / 4 + 1;  // words per LDS row (odd: the position-major side's 4
                                      // position groups fall in distinct banks)
    constexpr int LR = RP_F / 16;     // lanes per site row
    constexpr int RPP = 256 / LR;     // rows per pass
    constexpr int NP = RP_T / RPP;    // passes
    __shared__ uint32_t tile[RP_T][RW];  // [position][feature word]
    uint8_t *tb = reinterpret_cast<uint8_t *>(&tile[0][0]);
    const int tid = threadIdx.x;
    const int p0 = blockIdx.x * RP_T, f0 = blockIdx.y * RP_F;
    const size_t b = blockIdx.z;
    const int l = tid % LR, rg = tid / LR;  // lane l of row group rg: features f0 + 16 l ..
    const int fq = f0 + 16 * l;
    const bool words = (F & 3) == 0 && fq + 16 <= F;
    const int q = tid & 3;  // position-major side: positions p0 + 64 t + 16 q .. of feature f0 + fr
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    if (TO_PM) {
        uint32_t w[NP][4];
        int row[NP];
#pragma unroll
        for (int t = 0; t < NP; t++) {
            const int p = p0 + RPP * t + rg;
            row[t] = p < N ? perm[p] : -1;
        }
#pragma unroll
        for (int t = 0; t < NP; t++) {
            if (row[t] >= 0 && fq < F) {
                const uint8_t *rp = src + (b * N + row[t]) * F;
                if (words) {
                    const uint32_t *wp = reinterpret_cast<const uint32_t *>(rp + fq);
#pragma unroll
                    for (int k = 0; k < 4; k++) w[t][k] = wp[k];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        uint32_t x = 0;
#pragma unroll
                        for (int j = 0; j < 4; j++) x |= (fq + 4 * k + j < F ? (uint32_t)rp[fq + 4 * k + j] : 0u) << (8 * j);
                        w[t][k] = x;
                    }
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++) w[t][k] = 0;
            }
        }
#pragma unroll
        for (int t = 0; t < NP; t++)
#pragma unroll
            for (int k = 0; k < 4; k++) tile[RPP * t + rg][4 * l + k] = w[t][k];
        __syncthreads();
        for (int fr = tid >> 2; fr < RP_F; fr += 64) {
            const int f = f0 + fr;
            if (f >= F) break;
            uint8_t *drow = dst + (b * F + f) * Np + p0 + 16 * q;
#pragma unroll
            for (int t = 0; t < RP_T / 64; t++) {
                if (p0 + 64 * t >= Np) break;
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    uint32_t x = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) x |= (uint32_t)tb[(64 * t + 16 * q + 4 * k + j) * (RW * 4) + fr] << (8 * j);
                    o[k] = x;
                }
                // Np is a multiple of 64, so the 16 bytes are 16-byte aligned and inside the row
                const u32x4 ov = {o[0], o[1], o[2], o[3]};
                *reinterpret_cast<u32x4 *>(drow + 64 * t) = ov;
            }
        }
    } else {
        for (int fr = tid >> 2; fr < RP_F; fr += 64) {
            const int f = f0 + fr;
            if (f >= F) break;
            const uint8_t *srow = src + (b * F + f) * Np + p0 + 16 * q;
#pragma unroll
            for (int t = 0; t < RP_T / 64; t++) {
                if (p0 + 64 * t >= Np) break;
                const u32x4 iv = *reinterpret_cast<const u32x4 *>(srow + 64 * t);
                const uint32_t o[4] = {iv.x, iv.y, iv.z, iv.w};
#pragma unroll
                for (int k = 0; k < 4; k++)
#pragma unroll
                    for (int j = 0; j < 4; j++) tb[(64 * t + 16 * q + 4 * k + j) * (RW * 4) + fr] = (uint8_t)(o[k] >> (8 * j));
            }
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < NP; t++) {
            const int p = p0 + RPP * t + rg;
            const int s = p < N ? perm[p] : -1;
            if (s < 0 || fq >= F) continue;
            uint8_t *rp = dst + (b * N + s) * F;
            if (words) {
                uint32_t *wp = reinterpret_cast<uint32_t *>(rp + fq);
#pragma unroll
                for (int k = 0; k < 4; k++) wp[k] = tile[RPP * t + rg][4 * l + k];
            } else {
                for (int i = 0; i < 16 && fq + i < F; i++) rp[fq + i] = tb[(RPP * t + rg) * (RW * 4) + 16 * l + i];
            }
        }
    }
}

// By-site sources [B][N][F] -> by-position [B][F][Np] (F a multiple of 4), the by-site entry's
// transpose: one workgroup moves a tile of TR_P positions x 128 features (whole 128-B segments of
// the site rows) through LDS laid out position-major, tile[p][fw] (row stride 33 words):
// - read: 8 consecutive lanes take one site row's 128 B (16 B each, as 4 dwords), so a wave
//   instruction reads 8 whole row segments; the writes tile[r][4 c + k] of a half-wave (rows
//   r0 .. r0 + 3, chunks c = 0..7) fall on banks r + 4 c + k: 32 distinct;
// - write: TR_P / 4 lanes per feature word; lane l reads the words of positions 4 l .. 4 l + 3,
//   transposes the 4 x 4 bytes in registers (v_perm_b32) and stores one dword per feature row:
//   each store is a coalesced TR_P-byte row segment.
// A tile (x, y) and its neighbour (x, y + 1) share the boundary lines of unaligned site rows; their
// linear block ids differ by gridDim.x (16 at Np = 2048), which keeps them on one XCD's L2.
// cfg5, 256 chains (524 MB moved): 138.7 us for the round-5 kernel (64-feature tiles, byte LDS
// reads), 92-94 us for this one at TR_P = 128 (5.6 TB/s; tools/ab_transpose.sh,
// profiles/r06_transpose_ab.txt).
#ifndef SBZ_TR_P
#define SBZ_TR_P 128  // positions per tile (tools/ab_transpose.sh: 128 over 256 and 64)
#endif
constexpr int TR_P = SBZ_TR_P, TR_F = 128, TR_W = TR_F / 4, TR_S = TR_W + 1, TR_R = TR_P / 32;
__global__ __launch_bounds__(256) void source_to_pm_kernel(int N, int F, int Np, const int *perm,
                                                           const uint8_t *src, uint8_t *dst) {
    __shared__ uint32_t tile[TR_P * TR_S];
    const int tid = threadIdx.x;
    const int p0 = blockIdx.x * TR_P, f0 = blockIdx.y * TR_F;
    const size_t b = blockIdx.z;
    const int c = tid & 7, rl = tid >> 3;  // 16-B chunk c of the rows of positions rl + 32 i
    int rows[TR_R];
#pragma unroll
    for (int i = 0; i < TR_R; i++) {
        const int p = p0 + rl + 32 * i;
        rows[i] = p < N ? perm[p] : -1;
    }
    // (16-B loads of dword-aligned chunks: global loads need only dword alignment on gfx950)
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    uint32_t w[TR_R][4];
#pragma unroll
    for (int i = 0; i < TR_R; i++) {
        const int fc = f0 + 16 * c;
        const uint8_t *rp = src + (b * N + (size_t)max(rows[i], 0)) * F + min(fc, F - 16);
        u32x4a v = {0u, 0u, 0u, 0u};
        if (rows[i] >= 0 && fc < F) v = *reinterpret_cast<const u32x4a *>(rp);
        // a chunk past the row's end (F - fc < 16 bytes, F a multiple of 4) was read from F - 16:
        // shift its words down and zero the rest
        const int sh = fc + 16 > F ? (fc + 16 - F) / 4 : 0;
        const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++) w[i][k] = (k + sh < 4 && fc + 4 * k < F) ? vv[min(k + sh, 3)] : 0u;
    }
#pragma unroll
    for (int i = 0; i < TR_R; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) tile[(rl + 32 * i) * TR_S + 4 * c + k] = w[i][k];
    __syncthreads();
    // writes: TR_P / 4 lanes per feature word; 256 / (TR_P / 4) words at a time
    constexpr int LPW = TR_P / 4, WPR = 256 / LPW;
    const int ql = tid % LPW, fw0 = tid / LPW;
    if (p0 + 4 * ql >= Np) return;  // (no barrier follows)
    for (int fw = fw0; fw < TR_W; fw += WPR) {
        const int fb = f0 + 4 * fw;
        if (fb >= F) break;  // uniform
        uint32_t q[4];  // positions 4 ql + j, bytes = features fb .. fb + 3
#pragma unroll
        for (int j = 0; j < 4; j++) q[j] = tile[(4 * ql + j) * TR_S + fw];
        // o_i: feature fb + i, bytes = positions 4 lane .. + 3
        const uint32_t a_lo = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u);  // q0.0 q1.0 q0.1 q1.1
        const uint32_t a_hi = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);  // q0.2 q1.2 q0.3 q1.3
        const uint32_t b_lo = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u);
        const uint32_t b_hi = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
        const uint32_t o[4] = {__builtin_amdgcn_perm(b_lo, a_lo, 0x05040100u),
                               __builtin_amdgcn_perm(b_lo, a_lo, 0x07060302u),
                               __builtin_amdgcn_perm(b_hi, a_hi, 0x05040100u),
                               __builtin_amdgcn_perm(b_hi, a_hi, 0x07060302u)};
#pragma unroll
        for (int i = 0; i < 4; i++)
            *reinterpret_cast<uint32_t *>(dst + (b * F + fb + i) * Np + p0 + 4 * ql) = o[i];
    }
}

// By-site sources [B][N][F] -> 2-bit planes by position (F a multiple of 4, SPL >= 16), the layout
// lik_source_rc_kernel<.., PK = true> reads: per feature row, dword pair q = (chunk * NOB + kb) * 64
// + lane holds, at bit 8 j + kk of its lo / hi word, bit 0 / 1 of the component at position
// chunk * 64 SPL + 4 lane + 256 (KP kb + kk) + j (KP = min(SPL / 4, 8) groups per pair).  The row
// is SPL / 2 ... 4 bytes per 16 positions: a quarter of the by-position layout's bytes at SPL = 32.
// One workgroup covers 64 / KP consecutive pairs (lanes) of one (chunk, kb) and 128 features: its
// 256 positions (KP runs of 256 / KP) are read as whole 128-B row segments into LDS as in
// source_to_pm_kernel; then thread (feature word fw, pair l) reads the KP x 4 words of its
// positions, transposes each 4 x 4 byte block (v_perm_b32) and slides bits 0 / 1 of each
// feature's bytes into its planes; 8 consecutive lanes store 8 consecutive pairs of one row.
// Padding positions (p >= N) hold 0 (the kernel maps them to the neutral row whatever they hold).
#ifndef SBZ_PK_P
#define SBZ_PK_P 256  // positions per tile
#endif
#ifndef SBZ_PK_F
#define SBZ_PK_F 64  // features per tile (32, 64 or 128; tools/ab_pack.sh: 64)
#endif
constexpr int PK_P = SBZ_PK_P, PK_F = SBZ_PK_F, PK_W = PK_F / 4, PK_S = PK_W + 1;
template <int KP>
__global__ __launch_bounds__(256) void source_to_pk_kernel(int N, int F, int Np, int spl, int pk_row,
                                                           const int *perm, const uint8_t *src, uint8_t *dst) {
    constexpr int LT = PK_P / (4 * KP);           // pairs (lanes) per tile
    constexpr int LPR = PK_F / 16, RPP = 256 / LPR, NPASS = PK_P / RPP;  // row loads: 16 B per lane
    __shared__ uint32_t tile[PK_P * PK_S];
    const int tid = threadIdx.x;
    const int q0 = blockIdx.x * LT;  // first pair of the tile: (chunk * NOB + kb) * 64 + l0
    const int nob = spl / 4 / KP;
    const int cb = q0 / 64, l0 = q0 % 64;
    const int chunk = cb / nob, kb = cb % nob;
    const int pbase = chunk * 64 * spl + 4 * l0 + 256 * KP * kb;
    const int f0 = blockIdx.y * PK_F;
    const size_t b = blockIdx.z;
    // tile row r: run kk = r / (4 LT), u = r % (4 LT) -> position pbase + 256 kk + u
    auto pos_of = [&](int r) { return pbase + 256 * (r / (4 * LT)) + r % (4 * LT); };
    const int c = tid % LPR, rl = tid / LPR;
    const int fc = f0 + 16 * c;
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    uint32_t w[NPASS][4];
#pragma unroll
    for (int i = 0; i < NPASS; i++) {
        const int p = pos_of(rl + RPP * i);
        const int row = p < N ? perm[p] : -1;
        u32x4a v = {0u, 0u, 0u, 0u};
        if (row >= 0 && fc < F) v = *reinterpret_cast<const u32x4a *>(src + (b * N + (size_t)row) * F + min(fc, F - 16));
        const int sh = fc + 16 > F ? (fc + 16 - F) / 4 : 0;  // a chunk past the row's end: see source_to_pm_kernel
        const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++) w[i][k] = (k + sh < 4 && fc + 4 * k < F) ? vv[min(k + sh, 3)] : 0u;
    }
#pragma unroll
    for (int i = 0; i < NPASS; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) tile[(rl + RPP * i) * PK_S + 4 * c + k] = w[i][k];
    __syncthreads();
    for (int t = tid; t < PK_W * LT; t += 256) {
        const int l = t % LT, fw = t / LT;
        const int fb = f0 + 4 * fw;
        if (fb >= F) break;  // t grows with fw
        uint32_t lo[4] = {0u, 0u, 0u, 0u}, hi[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int kk = 0; kk < KP; kk++) {
            uint32_t q[4];  // positions 4 l + j of run kk; bytes = features fb .. fb + 3
#pragma unroll
            for (int j = 0; j < 4; j++) q[j] = tile[(kk * 4 * LT + 4 * l + j) * PK_S + fw];
            const uint32_t a_lo = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u);
            const uint32_t a_hi = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);
            const uint32_t b_lo = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u);
            const uint32_t b_hi = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
            const uint32_t o[4] = {__builtin_amdgcn_perm(b_lo, a_lo, 0x05040100u),
                                   __builtin_amdgcn_perm(b_lo, a_lo, 0x07060302u),
                                   __builtin_amdgcn_perm(b_hi, a_hi, 0x05040100u),
                                   __builtin_amdgcn_perm(b_hi, a_hi, 0x07060302u)};
#pragma unroll
            for (int i = 0; i < 4; i++) {  // o[i]: feature fb + i, byte j = position 4 l + j
                lo[i] |= (o[i] & 0x01010101u) << kk;
                hi[i] |= ((o[i] >> 1) & 0x01010101u) << kk;
            }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (fb + i >= F) break;
            const unsigned long long v = (unsigned long long)lo[i] | ((unsigned long long)hi[i] << 32);
            *reinterpret_cast<unsigned long long *>(dst + (b * F + fb + i) * (size_t)pk_row + (size_t)(q0 + l) * 8) = v;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Host side: kernel choice and launch
// ------------------------------------------------------------------------------------------
template <int C, int FR, bool XS8, bool BK>
const void *mix_kernel_x(int spl) {
    switch (spl) {
        case 4: return reinterpret_cast<const void *>(&lik_mixture_kernel<C, 4, FR, XS8, BK>);
        case 8: return reinterpret_cast<const void *>(&lik_mixture_kernel<C, 8, FR, XS8, BK>);
        case 16: return reinterpret_cast<const void *>(&lik_mixture_kernel<C, 16, FR, XS8, BK>);
        default: return reinterpret_cast<const void *>(&lik_mixture_kernel<C, 32, FR, XS8, BK>);
    }
}

// The dense mixture kernel for (C, family registers, x*8 observations, banked layout, sites per
// lane).  The banked layout needs S + 1 <= 16, so its observations are always x*8.
const void *mix_kernel(int C, int fr, bool xs8, bool bk, int spl) {
    if (bk) {
        if (C == 3) return fr == 4 ? mix_kernel_x<3, 4, true, true>(spl) : mix_kernel_x<3, 8, true, true>(spl);
        return mix_kernel_x<2, 4, true, true>(spl);
    }
    if (C == 3) {
        if (fr == 4) return xs8 ? mix_kernel_x<3, 4, true, false>(spl) : mix_kernel_x<3, 4, false, false>(spl);
        return xs8 ? mix_kernel_x<3, 8, true, false>(spl) : mix_kernel_x<3, 8, false, false>(spl);
    }
    return xs8 ? mix_kernel_x<2, 4, true, false>(spl) : mix_kernel_x<2, 4, false, false>(spl);
}

template <int C, int FR, bool XS8, bool BK>
void configure_mix_x(std::vector<const void *> &v) {
    for (int spl = 4; spl <= 32; spl *= 2) v.push_back(mix_kernel_x<C, FR, XS8, BK>(spl));
}

template <int C, int FR>
void configure_mix(std::vector<const void *> &v) {
    configure_mix_x<C, FR, true, true>(v);
    configure_mix_x<C, FR, true, false>(v);
    configure_mix_x<C, FR, false, false>(v);
}

// lik_source_rc_kernel applies: G = 64 / S1 lanes groups cover 2G zone and family rows (the 4
// T0 rows are written by a strided loop over the groups, so any G >= 1), row indices are bytes
bool source_rc_applies(const sbz_dims &d, int C) {
    const int S1 = d.n_states + 1;
    if (S1 > WAVE) return false;
    const int G = WAVE / S1;
    const int Fam = C == 3 ? d.n_families : 0;
    return d.n_zones <= 2 * G && Fam <= 2 * G && 4 + 2 * d.n_zones + 2 * Fam + 4 < 256;
}
// table (T0 4, T1 2Z, T2 2Fam, zero rows 4, neutral 1) | nwt | junk | zrow (row bytes)
size_t source_rc_lds_bytes(const sbz_dims &d, int C) {
    const size_t S1 = (size_t)d.n_states + 1;
    const size_t Fam = C == 3 ? (size_t)d.n_families : 0;
    const size_t rows = 4 + 2 * (size_t)d.n_zones + 2 * Fam + 5;
    return ((((rows * S1) + 1) & ~(size_t)1) + (size_t)SRC_NWC * 8 + WAVE) * 8 + ((rows + 7) & ~(size_t)7);
}
template <int C>
const void *source_rc_kernel(int spl, bool xs8, bool pk = false) {
    if (pk) {  // 2-bit planes (sites per lane 16 or 32)
        if (spl == 16) return xs8 ? reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 16, true, true>)
                                  : reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 16, false, true>);
        return xs8 ? reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 32, true, true>)
                   : reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 32, false, true>);
    }
    if (xs8) {
        switch (spl) {
            case 4: return reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 4, true>);
            case 8: return reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 8, true>);
            case 16: return reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 16, true>);
            default: return reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 32, true>);
        }
    }
    switch (spl) {
        case 4: return reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 4, false>);
        case 8: return reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 8, false>);
        case 16: return reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 16, false>);
        default: return reinterpret_cast<const void *>(&lik_source_rc_kernel<C, 32, false>);
    }
}

template <int C>
void configure_source(std::vector<const void *> &v) {
    for (int spl = 4; spl <= 32; spl *= 2) {
        v.push_back(source_rc_kernel<C>(spl, true));
        v.push_back(source_rc_kernel<C>(spl, false));
        if (spl >= 16) {
            v.push_back(source_rc_kernel<C>(spl, true, true));
            v.push_back(source_rc_kernel<C>(spl, false, true));
        }
    }
}

// the by-site entry reorders its sources into 2-bit planes (source_to_pk_kernel)
bool source_pk_applies(const sbz_ctx *ctx) {
    return ctx->src_pack && ctx->spl >= 16 && ctx->d.n_features % 4 == 0 && ctx->d.n_features >= 16;
}
// bytes per feature row of the 2-bit planes: 8 per lane and pair, NOB pairs per chunk
int source_pk_row(const sbz_ctx *ctx) {
    const int no = ctx->spl / 4, kp = no < 8 ? no : 8;
    return ctx->Np / (64 * ctx->spl) * (no / kp) * 64 * 8;
}

// How the mixture branch runs for these dims: table path with FR family registers (banked or
// packed layout), or the generic per-cell path (fr == 0).
struct MixPlan {
    int fr = 0;
    bool bk = false;  // the banked table layout applies (S + 1 <= 16, fits 64 KiB)
};

size_t mix_lds_bytes(const sbz_dims &d, int C, bool bk) {
    const size_t S1 = (size_t)d.n_states + 1;
    const size_t Fam = C == 3 ? (size_t)d.n_families : 0;
    if (bk)  // the lines hold the table, the neutral row and the junk slots
        return ((size_t)bk_lines(d.n_zones, (int)Fam + 1, (int)S1) * 32 + (size_t)16 * NW_PER_F) * 8;
    const size_t ncls = (size_t)(d.n_zones + 1) * (Fam + 1);
    return ((ncls + 1) * S1 + WAVE + 1 + (size_t)NWC * NW_PER_F) * 8;
}

MixPlan plan_mixture(const sbz_dims &d, int C) {
    MixPlan p;
    const int S1 = d.n_states + 1;
    const int Fam = C == 3 ? d.n_families : 0;
    if (S1 > WAVE) return p;
    const int G = WAVE / S1;
    if (d.n_zones + 1 > ZR * G) return p;
    if ((d.n_zones + 1) * (Fam + 1) + 1 > 256) return p;  // class ids are bytes
    if (mix_lds_bytes(d, C, false) > 64 * 1024) return p; // row offsets are 16-bit
    if (C == 2 || Fam <= 4) p.fr = 4;
    else if (Fam <= 8) p.fr = 8;
    if (p.fr) p.bk = 2 * S1 <= 32 && mix_lds_bytes(d, C, true) <= 64 * 1024;
    return p;
}

// one resident round of single-wave tasks (occupancy x CUs) over the launch, so every wave
// streams its features with no tail of late tasks
int tasks_per_chain(sbz_ctx *ctx, const void *fn, size_t lds, int B) {
    if (ctx->mix_occ == 0 || ctx->mix_occ_fn != fn) {
        int occ = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, WAVE, lds);
        ctx->mix_occ = (e == hipSuccess && occ > 0) ? occ : 8;
        ctx->mix_occ_fn = fn;
    }
    // a chain's tasks all resident at once (occupancy x CUs), except for few sites per lane
    // (N <= 256): there the per-task set-up and the finish outweigh the per-feature work of more,
    // shorter tasks, and 4 tasks per CU measured fastest (cfg2 / cfg3 / cfg4 shapes: 28 / 22 / 16 us
    // at the occupancy, 12 / 15 / 12 at 4; profiles/r03_lik_tasks_per_cu.txt)
    const int per_cu = ctx->tasks_per_cu > 0 ? ctx->tasks_per_cu
                                             : (ctx->spl <= 4 ? std::min(4, ctx->mix_occ) : ctx->mix_occ);
    const int F = ctx->d.n_features;
    return std::max(1, std::min((F + 1) / 2, (ctx->n_cu * per_cu + B - 1) / B));
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
    if (!source_mode) {
        const MixPlan p = plan_mixture(d, C);
        return p.fr ? mix_lds_bytes(d, C, p.bk) : 0;
    }
    return source_rc_applies(d, C) ? source_rc_lds_bytes(d, C) : 0;
}

int lik_configure(sbz_ctx *ctx) {
    std::vector<const void *> fns;
    configure_mix<2, 4>(fns);
    configure_mix<3, 4>(fns);
    configure_mix<3, 8>(fns);
    configure_source<2>(fns);
    configure_source<3>(fns);
    for (const void *fn : fns) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
    }
    return SBZ_OK;
}

int launch_source_pack(sbz_ctx *ctx, int B, const uint8_t *src, uint8_t *dst) {
    const int no = ctx->spl / 4, kp = no < 8 ? no : 8;
    const int pairs = source_pk_row(ctx) / 8;
    const dim3 g(pairs / (PK_P / (4 * kp)), (ctx->d.n_features + PK_F - 1) / PK_F, B);
    if (kp == 8)
        source_to_pk_kernel<8><<<g, 256, 0, ctx->stream>>>(ctx->d.n_sites, ctx->d.n_features, ctx->Np, ctx->spl,
                                                            source_pk_row(ctx), ctx->d_perm, src, dst);
    else
        source_to_pk_kernel<4><<<g, 256, 0, ctx->stream>>>(ctx->d.n_sites, ctx->d.n_features, ctx->Np, ctx->spl,
                                                            source_pk_row(ctx), ctx->d_perm, src, dst);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "source_to_pk_kernel launch");
}

int launch_source_transpose(sbz_ctx *ctx, int B, const uint8_t *src, uint8_t *dst, bool to_pm) {
    if (B <= 0) return SBZ_OK;
    if (to_pm && ctx->d.n_features % 4 == 0 && ctx->d.n_features >= 16) {  // whole-line tiles
        const dim3 g((ctx->Np + TR_P - 1) / TR_P, (ctx->d.n_features + TR_F - 1) / TR_F, B);
        source_to_pm_kernel<<<g, 256, 0, ctx->stream>>>(ctx->d.n_sites, ctx->d.n_features, ctx->Np, ctx->d_perm,
                                                         src, dst);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "source_to_pm_kernel launch");
    }
    const dim3 grid((ctx->Np + RP_T - 1) / RP_T, (ctx->d.n_features + RP_F - 1) / RP_F, B);
    if (to_pm)
        source_transpose_kernel<true><<<grid, 256, 0, ctx->stream>>>(ctx->d.n_sites, ctx->d.n_features, ctx->Np,
                                                                     ctx->d_perm, src, dst);
    else
        source_transpose_kernel<false><<<grid, 256, 0, ctx->stream>>>(ctx->d.n_sites, ctx->d.n_features, ctx->Np,
                                                                      ctx->d_perm, src, dst);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "source_transpose_kernel launch");
}

int launch_loglik(sbz_ctx *ctx, int B, const uint8_t *zone, const double *w, const double *pg,
                  const double *pz, const double *pf, const uint8_t *source, bool source_pm,
                  double *out_ll) {
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
    a.perm = ctx->d_perm;
    a.zone = zone;
    a.w = w;
    a.pg = pg;
    a.pz = pz;
    a.pf = pf;

    // the kernel and its tasks per chain W
    const void *fn = nullptr;
    size_t lds = 0;
    const char *names = nullptr;
    bool src_rc = false, pk = false;
    int rc;
    if (!src_mode) {
        const MixPlan plan = plan_mixture(d, ctx->C);
        if (plan.fr) {
            const bool bk = plan.bk && ctx->lik_banked;
            fn = mix_kernel(ctx->C, plan.fr, ctx->xs8 != 0, bk, ctx->spl);
            lds = mix_lds_bytes(d, ctx->C, bk);
            const int W = tasks_per_chain(ctx, fn, lds, B);
            a.fpw = (F + W - 1) / W;
            names = "lik_mixture_kernel";
        } else {
            fn = ctx->C == 3 ? reinterpret_cast<const void *>(&lik_mixture_generic_kernel<3>)
                             : reinterpret_cast<const void *>(&lik_mixture_generic_kernel<2>);
            names = "lik_mixture_generic_kernel";
        }
    } else {
        src_rc = ctx->src_rc && source_rc_applies(d, ctx->C) && source_rc_lds_bytes(d, ctx->C) <= 64 * 1024;
        if (src_rc) {
            pk = !source_pm && source_pk_applies(ctx);
            fn = ctx->C == 3 ? source_rc_kernel<3>(ctx->spl, ctx->xs8 != 0, pk)
                             : source_rc_kernel<2>(ctx->spl, ctx->xs8 != 0, pk);
            lds = source_rc_lds_bytes(d, ctx->C);
            const int W = tasks_per_chain(ctx, fn, lds, B);
            a.fpw = (F + W - 1) / W;
            names = source_pm ? "lik_source_rc_kernel"
                    : pk ? "source_to_pk_kernel lik_source_rc_kernel<planes>"
                    : (F % 4 == 0 && F >= 16 ? "source_to_pm_kernel lik_source_rc_kernel" : "source_transpose_kernel lik_source_rc_kernel");
        } else {
            fn = ctx->C == 3 ? reinterpret_cast<const void *>(&lik_source_generic_kernel<3>)
                             : reinterpret_cast<const void *>(&lik_source_generic_kernel<2>);
            if (source_pm) a.src_pm = source;
            else a.src_rm = source;
            names = "lik_source_generic_kernel";
        }
    }
    if (lds == 0) {
        // generic paths: one wave per (chain, feature range), enough tasks to fill 256 CUs x 32 waves
        const int W = std::max(1, std::min(F, (256 * 32 + B - 1) / B));
        a.fpw = (F + W - 1) / W;
    }
    a.W = (F + a.fpw - 1) / a.fpw;

    rc = ensure(ctx, ctx->partial, (size_t)B * a.W * sizeof(double));
    if (rc) return rc;
    a.partial = static_cast<double *>(ctx->partial.ptr);
    for (DevBuf *buf : {&ctx->ticket, &ctx->zflag}) {  // 0 between launches
        if (buf->bytes < (size_t)B * sizeof(unsigned) || !buf->ptr) {
            rc = ensure(ctx, *buf, (size_t)B * sizeof(unsigned));
            if (rc) return rc;
            hipError_t e = hipMemsetAsync(buf->ptr, 0, buf->bytes, ctx->stream);
            if (e != hipSuccess) return hip_fail(ctx, e, "hipMemsetAsync(ticket)");
        }
    }
    a.ticket = static_cast<unsigned *>(ctx->ticket.ptr);
    a.zflag = src_mode ? static_cast<unsigned *>(ctx->zflag.ptr) : nullptr;
    a.out = out_ll;

    hipStream_t st = ctx->stream;
    // A launch that never ran leaves no ticket armed, but one that failed after some tasks
    // finished would leave the chains' tickets non-zero and corrupt every later sum: re-zero them.
    auto launch_failed = [&](hipError_t e, const char *what) {
        (void)hipMemsetAsync(ctx->ticket.ptr, 0, ctx->ticket.bytes, st);
        (void)hipMemsetAsync(ctx->zflag.ptr, 0, ctx->zflag.bytes, st);
        return hip_fail(ctx, e, what);
    };
    if (src_rc) {
        if (source_pm) {
            a.src_pm = source;
        } else if (pk) {  // the reference layout: reordered into 2-bit planes by position first
            a.pk_row = source_pk_row(ctx);
            rc = ensure(ctx, ctx->src_t, (size_t)B * F * a.pk_row);
            if (rc) return rc;
            rc = launch_source_pack(ctx, B, source, static_cast<uint8_t *>(ctx->src_t.ptr));
            if (rc) return rc;
            a.src_pm = static_cast<const uint8_t *>(ctx->src_t.ptr);
        } else {  // the reference layout: transposed to the position-major one first
            rc = ensure(ctx, ctx->src_t, (size_t)B * F * ctx->Np);
            if (rc) return rc;
            rc = launch_source_transpose(ctx, B, source, static_cast<uint8_t *>(ctx->src_t.ptr), true);
            if (rc) return rc;
            a.src_pm = static_cast<const uint8_t *>(ctx->src_t.ptr);
        }
    }
    ctx->last_kernels = names;
    void *args[] = {&a};
    hipError_t e = hipLaunchKernel(fn, dim3(a.W, B), dim3(WAVE), args, lds, st);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return launch_failed(e, "likelihood launch");
    return SBZ_OK;
}

}  // namespace sbz
