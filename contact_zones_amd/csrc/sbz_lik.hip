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
#include <type_traits>
#include <vector>

#include "sbz_internal.h"

namespace sbz {

namespace {

constexpr double LN2 = 0.69314718055994530941723212145818;
constexpr int WAVE = 64;
constexpr int ZR = 2;  // zone classes per lane held in registers
constexpr int NW_BYTES = 16 * 8;  // nw[4][4] doubles ahead of the source-kernel table

__device__ __forceinline__ bool safe_factor(double v) {
    return v == 0.0 || (v >= 0x1p-120 && v <= 0x1p120);
}

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
// producer stores every byte sc1 (relaxed agent-scope atomic store, 8 B), (3) the storing lane
// (the only lane that stores) runs s_waitcnt vmcnt(0) before its agent-scope atomic add to the
// chain's one unsharded counter, (4) the consumer is the task whose add returned W-1, and it loads
// only after that add has returned; buffers come from hipMalloc, one single-wave task per
// workgroup.  The release/acquire form (a release on every ticket add, an acquire on the winner)
// writes back the XCD's L2 once per task: ~1.7 us per fence, measured ~2x the kernel here.
// tests/test_gpu_likelihood.py::test_partials_handoff_stress re-checks the hand-off under uneven
// load across all XCDs; the host re-zeroes the tickets when a launch fails (launch_loglik).
//
// `zw` (source branch): the task saw a selected normalised weight of exactly 0.  The reference
// then returns -inf whatever the other cells hold (model.py:181-182, NaN cells included), so the
// flag travels beside the partials (zflag[b], same sc1 hand-off) and overrides the sum.
__device__ __forceinline__ void finish_chain(const LikArgs &a, int b, double tot,
                                             bool leader = threadIdx.x == 0, bool zw = false) {
    if (!leader) return;
    if (a.W == 1) {
        a.out[b] = zw ? -INFINITY : tot;
        return;
    }
    double *pb = a.partial + (size_t)b * a.W;
    __hip_atomic_store(&pb[blockIdx.x], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (zw) __hip_atomic_store(&a.zflag[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev =
        __hip_atomic_fetch_add(&a.ticket[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev != (unsigned)a.W - 1) return;
    asm volatile("" ::: "memory");
    double s = 0.0;
    for (int t = 0; t < a.W; t++)
        s += __hip_atomic_load(&pb[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.zflag != nullptr && __hip_atomic_load(&a.zflag[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        s = -INFINITY;
        __hip_atomic_store(&a.zflag[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    a.out[b] = s;
    __hip_atomic_store(&a.ticket[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
// Mixture tables (shared by the dense and zone-sparse mixture kernels).  Requires S + 1 <= 64,
// Z + 1 <= ZR * (64 / (S + 1)), Fam <= FR and (Z+1)(Fam+1) + 1 <= 256 (checked on the host;
// otherwise lik_mixture_generic_kernel runs).
//
// A task is (chain b, features [fa, fb)).  LDS (bytes from the dynamic base):
//   table      T[ncls + 1][S1] doubles, class = zc*FamC + fc; the last row is neutral (1.0).
//              Rows 0..FamC-1 (zc = 0) are the no-zone classes T0[fc][x].
//   junk       64 doubles (writes of lanes without an entry)
// Lane (lx = lane % S1, lg = lane / S1) builds the entries of state x = lx for the zone
// classes zc = lg + i*G, i < ZR (G = 64 / S1), every family class.  It loads exactly the
// parameters those entries need (p_global[f][x], p_zones[zc-1][f][x], p_fam[fm][f][x]; uniform
// row base + 32-bit lane offset) straight into registers, SBZ_PIPE - 1 features ahead; the
// normalised weights are computed by lanes 0..11 (one division each) and broadcast to SGPRs
// with v_readlane.  Every global load is unconditional (indices clamped): a load under a
// branch makes the compiler's vmcnt bookkeeping conservative at the join, and a feature's
// gathers would then wait for the next feature's loads.
// ---------------------------------------------------------------------------------------
#ifndef SBZ_ABLATE
#define SBZ_ABLATE 0  // diagnostic builds only: 1 = skip gathers, 2 = skip table build,
                      // 4 = skip tame checks, 8 = skip NA selects, 16 = every gather reads
                      // the first table row (no bank conflicts), 32 = constant normalised
                      // weights (no LDS weight reads) (wrong results)
#endif
#ifndef SBZ_MIX_WAVES
#define SBZ_MIX_WAVES 3  // launch bound: minimum waves per SIMD of the dense mixture kernel
#endif
#ifndef SBZ_ZS_WAVES
#define SBZ_ZS_WAVES 3  // launch bound: minimum waves per SIMD of the zone-sparse kernel
#endif
#ifndef SBZ_PIPE
#define SBZ_PIPE 2  // parameter / observation register sets: loads run SBZ_PIPE - 1 features ahead
#endif
#ifndef SBZ_LDS_FENCE
// 1: s_waitcnt lgkmcnt(0) around the table build.  0: compiler barrier only — a wave's LDS
// instructions execute in issue order, so within a single-wave workgroup a read issued after a
// write (by any lane) sees it, and a write issued after a read cannot overtake it.
#define SBZ_LDS_FENCE 1
#endif
#ifndef SBZ_DB_LAUNDER
#define SBZ_DB_LAUNDER 0  // double-buffered kernel: launder the row offsets each feature
#endif
#ifndef SBZ_DB_GBAR
#define SBZ_DB_GBAR 1  // double-buffered kernel: scheduling barrier every 8 gathers (VGPR bound)
#endif
#ifndef SBZ_TAME
// 1: a feature's inputs are "tame" when every parameter lies in [0, 1 + 2^-20) (one unsigned max
//    over the high words); products that still leave the normal range (tiny or zero cells) are
//    caught after the fact and the task is re-run with per-factor renormalisation.
// 0: every input checked against [2^-60, 2^60] or 0 before the feature (round-1 form).
#define SBZ_TAME 1
#endif
#ifndef SBZ_RN
// SBZ_TAME = 1: the dense kernel's product chains are checked and renormalised once per SBZ_RN
// features (8 * SBZ_RN factors per chain; every factor <= ~1, so nothing overflows, and an
// underflow is caught by the check and re-run exactly)
#define SBZ_RN 4
#endif
#ifndef SBZ_GIF
#define SBZ_GIF 16  // dense kernel: table reads in flight per wave (scheduling barrier every SBZ_GIF)
#endif
#ifndef SBZ_PAIR
// dense kernel, packed layout (experiment): tables of two features built back to back into two
// 4-KiB LDS tables, then both features gathered together (one build phase and twice the
// independent reads per pair)
#define SBZ_PAIR 0
#endif
#ifndef SBZ_PAIR_ASM
#define SBZ_PAIR_ASM 1
#endif
#ifndef SBZ_GPIPE
#define SBZ_GPIPE 0  // dense kernel: software-pipelined gather groups of SBZ_GIF reads
#endif
#ifndef SBZ_NCH
#define SBZ_NCH 4  // dense kernel: independent product chains per lane (4 or 8)
#endif
#ifndef SBZ_OBS_X4
#define SBZ_OBS_X4 0  // dense kernel: observations as 16-B loads (4 words of 4 sites per lane)
#endif
#ifndef SBZ_ASM_ADDR
#define SBZ_ASM_ADDR 0  // cell addresses by inline v_add_u32_sdwa (row offsets stay packed)
#endif
#ifndef SBZ_LIK_STAMP
// diagnostic builds only: the dense kernel returns, instead of each chain's log-likelihood, the
// s_memtime cycles its waves spent in phase a.F4 (0 weights, 1 table build, 2 load issue,
// 3 gathers + renorm, 4 task set-up, 5 whole task), summed over the chain's tasks
#define SBZ_LIK_STAMP 0
#endif
__device__ __forceinline__ uint64_t lik_stamp() {
    uint64_t t = 0;
    if (SBZ_LIK_STAMP) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
        __builtin_amdgcn_sched_barrier(0);
    }
    return t;
}
constexpr int NS = SBZ_PIPE;

// Banked table layout (dense kernel, S + 1 <= 16).  The table lives in 256-B LDS lines, one
// line per LDS bank sweep (64 banks x 4 B).  The no-zone rows T0[fc] (read by ~80 % of the
// sites, mostly one family per 32-lane group after the family sort) own slots [0, S1) of lines
// 0 .. FamC-1; every zone row (zc, fc) has a line of its own and sits in slots [S1, 2 S1) or
// [32 - S1, 32) by zone parity, so a zoned lane never lands on a bank the group's hot row
// uses, and zoned lanes of different zones spread over both halves.  Simulated on the bench
// data: 3.3 LDS cycles per ds_read_b64 against 4.1 for the packed [class][x] layout.
// Line FamC slots [0, S1) hold the neutral row (padding sites), lines FamC+1.. slots [0, S1)
// the junk slots of lanes without an entry.
__host__ __device__ constexpr int bk_lines(int Z, int FamC, int S1) {
    return Z * FamC > FamC + 1 + (WAVE + S1 - 1) / S1 ? Z * FamC : FamC + 1 + (WAVE + S1 - 1) / S1;
}
// first double of row (zc, fc), zc = zone + 1 (0 = no zone)
__host__ __device__ __forceinline__ uint32_t bk_row(int zc, int fc, int FamC, int S1) {
    return zc == 0 ? (uint32_t)fc * 32u
                   : (uint32_t)(((zc - 1) * FamC + fc) * 32 + S1 + ((zc - 1) & 1) * (32 - 2 * S1));
}

__device__ __forceinline__ void lds_phase() {
#if SBZ_LDS_FENCE
    wave_lds_sync();
#else
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#endif
}

// A parameter or normalised weight is "tame" if it is 0 or in [2^-60, 2^60]: every table entry
// is then a sum of <= 3 products of tame values, i.e. 0 or in [2^-120, 3*2^120], and 8 such
// factors times a mantissa in [0.5, 1) stay in the normal range.  Otherwise (tiny / huge /
// negative / NaN inputs) the wave renormalises after every factor for that feature.
__device__ __forceinline__ bool tame(double v) { return v == 0.0 || (v >= 0x1p-60 && v <= 0x1p60); }
// Byte address of cell j (0..3) of a 4-site group: its 16-bit row offset (WORD_(j&1) of the
// packed pair) plus its observation byte x*8 (BYTE_j of the observation word), one
// v_add_u32_sdwa.  Written out so the row offsets stay packed two per register: the compiler
// otherwise hoists the loop-invariant unpack out of the feature loop into 32 registers.
__device__ __forceinline__ uint32_t cell_addr(uint32_t bw, uint32_t ow, int j) {
    uint32_t r;
    switch (j) {
        case 0: asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:BYTE_0"
                    : "=v"(r) : "v"(bw), "v"(ow)); break;
        case 1: asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_1"
                    : "=v"(r) : "v"(bw), "v"(ow)); break;
        case 2: asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:BYTE_2"
                    : "=v"(r) : "v"(bw), "v"(ow)); break;
        default: asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_3"
                     : "=v"(r) : "v"(bw), "v"(ow)); break;
    }
    return r;
}
__device__ __forceinline__ uint32_t hiword(double v) {
    return (uint32_t)((unsigned long long)__double_as_longlong(v) >> 32);
}

// One feature's parameters as one lane needs them (the weights come from MixTable::prep).
template <int C, int FR>
struct MixParams {
    double g;       // p_global[f][lxc]
    double z[ZR];   // p_zones[zc_i - 1][f][lxc]
    double fm[FR];  // p_fam[fm][f][lxc]
};

// Normalised weights are computed for NWC features at a time (MixTable::prep) and kept in LDS.
#ifndef SBZ_NWC
#define SBZ_NWC 32
#endif
constexpr int NWC = SBZ_NWC;
// Per feature, h = hz | hf << 1: (c0, c1) of h at [2h, 2h + 1]; c2 of h at 8 + 2 * hz + hf, so
// c2 of (h, h + 2) is one 16-B pair.  Every read of build() is a ds_read_b128.
constexpr int NW_PER_F = 12;

// Double-buffered layout (DB, lik_mixture_db_kernel): two tables of DB_TAB_BYTES each, so the
// table of feature f+1 is built while feature f is gathered; every zone class has FR + 1 family
// rows (rows >= Fam unused) so the build has no branches.
constexpr int DB_TAB_BYTES = 4096;

// BK: banked table layout (bk_row).  PH: the SBZ_TAME = 1 input check, for kernels that catch
// under-flowing products after the fact (the dense kernel); the others check every input.
template <int C, int FR, bool DB = false, int SLOT = -1, bool BK = false, bool PH = false>
struct MixTable {
    // features per normalised-weight batch: 16 in the banked layout, so that 12 tasks per CU
    // (3 waves per SIMD) fit the 160 KiB of LDS at the bench shape
    static constexpr int NWCT = BK ? 16 : NWC;
    static constexpr bool PRT = SBZ_PAIR && PH && !BK && !DB;  // two 512-double tables
    int tbo = 0;  // PRT: doubles from `tab` to the table being built
    // SLOT >= 0: this wave loads and builds only zone-class slot SLOT (i = SLOT of the ZR
    // slots); the wave-specialised kernel splits the table between two builder waves this way.
    static constexpr bool has(int i) { return SLOT < 0 || i == SLOT; }
    static constexpr int RPZ_DB = (C == 3) ? FR + 1 : 1;  // rows per zone class (DB layout)
    int lane, S, S1, FamC, RPZ, Z, Fam, ncls, G, lx, lg, row_bytes;
    uint32_t lxc;
    bool na;
    uint32_t zfs;
    unsigned char *lds;
    double *tab, *junk;
    double *nwt;       // [NWC][NW_PER_F] normalised weights of features nwf0 .. nwf0 + NWC
    int nwf0;          // first feature of the weights in nwt (wave-uniform)
    uint64_t nwbad;    // bits 2k, 2k+1: feature nwf0 + k has an untamed normalised weight
    int hz0;           // has-zone flag of the lane's slot-0 class (lg > 0)
    const double *pgb, *zbase, *fbase, *wb;
    uint32_t pzo[ZR];  // lane offset of its p_zones rows (elements)
    // PH (dense kernel): the parameter loads are buffer loads whose per-feature and per-family
    // advance is a scalar offset, so a feature's loads need no address arithmetic at all.  The
    // NA column's lanes, and the zone loads of the no-zone class, use an out-of-range offset:
    // the load returns 0, and adding `naone` (1 on the NA column, else 0) gives the reference's
    // lh of 1 for NA cells (model.py:247) and 0 for the zone lh outside every zone, with no
    // selects (p + 0 == p for every p but -0).
    __amdgpu_buffer_rsrc_t rg, rz, rf;
    uint32_t vg_off, vz_off[ZR];
    double naone;

    __device__ __forceinline__ MixTable(const LikArgs &a, unsigned char *lds_, int b,
                                        double *tab0 = nullptr, double *tab1 = nullptr)
        : lds(lds_) {
        lane = threadIdx.x % WAVE;
        S = a.S;
        S1 = a.S + 1;
        FamC = a.FamC;
        RPZ = DB ? RPZ_DB : FamC;
        Z = a.Z;
        Fam = (C == 3) ? a.Fam : 0;
        ncls = (Z + 1) * RPZ;
        G = WAVE / S1;
        lx = lane % S1;
        lg = lane / S1;
        na = (SBZ_ABLATE & 8) ? false : lx == S;
        lxc = (uint32_t)min(lx, S - 1);  // the NA column and idle lanes read state 0
        // LDS: non-DB  [table | junk | nwt] from the dynamic base;
        //      DB      two static tables (tab0, tab1), [junk | nwt] from the dynamic base
        tab = DB ? tab0 : reinterpret_cast<double *>(lds);
        double *dyn = DB ? reinterpret_cast<double *>(lds) : tab + (PRT ? 1024 : (ncls + 1) * S1);
        junk = dyn + lane;
        // nwt 16-B aligned (one 8-B pad slot in the LDS budget)
        nwt = dyn + WAVE + (DB ? 0 : (((ncls + 1) * S1) & 1));
        if (BK) {
            junk = tab + (FamC + 1 + lane / S1) * 32 + lane % S1;
            nwt = tab + bk_lines(Z, FamC, S1) * 32;
        }
        nwf0 = -(1 << 30);
        nwbad = 0;
        hz0 = lg > 0 ? 1 : 0;
        row_bytes = S1 * 8;
        zfs = (uint32_t)(a.F * S);
        pgb = a.pg + (size_t)b * zfs;
        zbase = Z > 0 ? a.pz + (size_t)b * Z * zfs : pgb;
        fbase = Fam > 0 ? a.pf + (size_t)b * Fam * zfs : pgb;
        wb = a.w + (size_t)b * a.F * C;
#pragma unroll
        for (int i = 0; i < ZR; i++)
            pzo[i] = (uint32_t)(max(min(lg + i * G, Z), 1) - 1) * zfs + lxc;
        if constexpr (PH) {
            constexpr uint32_t OOB = 0x80000000u;  // beyond every buffer: the load returns 0
            vg_off = na ? OOB : lxc * 8u;
#pragma unroll
            for (int i = 0; i < ZR; i++) vz_off[i] = (na || lg + i * G == 0) ? OOB : pzo[i] * 8u;
            naone = na ? 1.0 : 0.0;
            rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(pgb), (short)0, (int)(zfs * 8u), 0x00020000);
            rz = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(zbase), (short)0,
                                                   (int)((uint32_t)max(Z, 1) * zfs * 8u), 0x00020000);
            rf = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(fbase), (short)0,
                                                   (int)((uint32_t)max(Fam, 1) * zfs * 8u), 0x00020000);
        }
        if (SBZ_ABLATE & 2)  // diagnostic build without table builds: a constant table
            for (int q = lane; q < (BK ? bk_lines(Z, FamC, S1) * 32 : (ncls + 1) * S1); q += WAVE) tab[q] = 0.5;
        for (int x = lane; x < S1; x += WAVE) {  // neutral row (both buffers)
            tab[(BK ? FamC * 32 : ncls * S1) + x] = 1.0;
            if (PRT) tab[512 + ncls * S1 + x] = 1.0;
            if (DB) tab1[ncls * S1 + x] = 1.0;
        }
    }

    __device__ __forceinline__ void load(int f, MixParams<C, FR> &r) const {
        const uint32_t fo = (uint32_t)f * (uint32_t)S;
        if constexpr (PH) {
            const int so = (int)(fo * 8u);
            r.g = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rg, (int)vg_off, so, 0));
#pragma unroll
            for (int i = 0; i < ZR; i++)
                if (has(i))
                    r.z[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rz, (int)vz_off[i], so, 0));
#pragma unroll
            for (int fm = 0; fm < FR; fm++)
                r.fm[fm] = __builtin_bit_cast(
                    double, __builtin_amdgcn_raw_buffer_load_b64(
                                rf, (int)vg_off, so + (int)((uint32_t)min(fm, max(Fam - 1, 0)) * zfs * 8u), 0));
            return;
        }
        r.g = pgb[fo + lxc];
#pragma unroll
        for (int i = 0; i < ZR; i++)
            if (has(i)) r.z[i] = zbase[fo + pzo[i]];
#pragma unroll
        for (int fm = 0; fm < FR; fm++)
            r.fm[fm] = fbase[(uint32_t)min(fm, max(Fam - 1, 0)) * zfs + fo + lxc];
    }

    // normalize_weights (model.py:451-452): w*has / ((w0*h0 + w1*h1) + w2*h2) for the 4 classes
    // h = hz | hf << 1 of features f0 .. f0 + NWC (clamped to fb - 1), into nwt.  Lane 2k + hp
    // computes feature k's h = 2hp and 2hp + 1 (one division per weight, as the reference).
    // Runs once per NWC features instead of once per feature.
    // PH: the weights of the next batch are loaded one batch ahead (prep_issue), so prep does
    // not wait a memory round trip; a batch other than the one in flight loads on the spot.
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
        double w0r, w1r, w2r;
        if (PH) {
            if (pwf0 != f0) prep_issue(f0, fb);
            w0r = pw0;
            w1r = pw1;
            w2r = pw2;
            prep_issue(f0 + NWCT, fb);
        } else {
            const uint32_t f = (uint32_t)min(f0 + k, fb - 1);
            w0r = wb[f * C];
            w1r = wb[f * C + 1];
            w2r = C == 3 ? wb[f * C + 2] : 0.0;
        }
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
        lds_phase();  // earlier features' reads of nwt are done
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
        lds_phase();
    }

    // The table of feature f (its weights in nwt: nwf0 <= f < nwf0 + NWC).  Returns `wide`:
    // some input is not tame, so products over this feature must renormalise after every factor.
    __device__ __forceinline__ bool build(const MixParams<C, FR> &r, int f, double *dbtab = nullptr) const {
        const int k = f - nwf0;
        int ok;
        if constexpr (PH) {
            // every parameter in [0, 1 + 2^-20): unsigned high words <= hi(1.0) (a sign bit, NaN or
            // inf fails).  Table entries are then <= ~1, so a product never overflows, and one that
            // underflows stays below 2^-1022 until the feature's check (see lik_mixture_kernel).
            uint32_t hmx = hiword(r.g);
#pragma unroll
            for (int i = 0; i < ZR; i++)
                if (has(i)) hmx = max(hmx, hiword(r.z[i]));
#pragma unroll
            for (int fm = 0; fm < FR; fm++) hmx = max(hmx, hiword(r.fm[fm]));
            ok = hmx <= 0x3FF00000u;
        } else {
            ok = (int)tame(r.g);
#pragma unroll
            for (int i = 0; i < ZR; i++)
                if (has(i)) ok &= (int)tame(r.z[i]);
#pragma unroll
            for (int fm = 0; fm < FR; fm++) ok &= (int)tame(r.fm[fm]);
        }
#if SBZ_ABLATE & 4
        ok = 1;  // diagnostic build: no tame checks
#endif
        const bool wide = ((nwbad >> (2 * k)) & 3ull) != 0 || __ballot(!ok) != 0;
        // 1. normalised weights from nwt.  Slot i >= 1 holds zone classes only (zc >= G >= 1):
        //    wave-uniform weights of h = 1 (no family) and h = 3 (family).  Slot 0 mixes zc = 0
        //    (lanes lg == 0, h = 0 / 2) and zone classes (h = 1 / 3).
        //    Six 16-B reads: (c0, c1) of each h, and c2 of (h, h + 2) as one pair.
        const double *nk = static_cast<const double *>(__builtin_assume_aligned(nwt + k * NW_PER_F, 16));
        auto pair = [&](int at) {
            if (SBZ_ABLATE & 32) return double2{0.25 + at, 0.5};  // diagnostic: no LDS weight reads
            return *reinterpret_cast<const double2 *>(nk + at);
        };
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
        // DB: no fences — a wave's LDS operations complete in issue order, and the buffer being
        // written was last read by the gathers of feature f - 1, issued earlier.
        if (!DB) lds_phase();
        double *const tb = DB ? dbtab : tab + (PRT ? tbo : 0);
        const double l0 = PH ? r.g + naone : na ? 1.0 : r.g;
        const double nad = PH ? naone : na ? 1.0 : 0.0;  // l2 of a class without family
#pragma unroll
        for (int i = 0; i < ZR; i++) {
#if SBZ_ABLATE & 2
            break;  // diagnostic build: skip the table build
#endif
            if (!has(i)) continue;
            const int zc = lg + i * G;
            const bool valid = (lane < G * S1) && (zc <= Z);
            const double n00 = i == 0 ? p[0][0] : u[0][0], n01 = i == 0 ? p[0][1] : u[0][1];
            // zone lh: 0 for a site outside every zone (model.py:241-247), 1 for NA
            const double l1 = PH ? r.z[i] + naone : na ? 1.0 : ((i > 0 || zc > 0) ? r.z[i] : 0.0);
            double *row = valid ? tb + (BK ? bk_row(zc, 0, FamC, S1) : (uint32_t)(zc * RPZ * S1)) + lx : junk;
            const int rs = valid ? (BK ? 32 : S1) : 0;
            double v = n00 * l0 + n01 * l1;
            if (C == 3 && DB) {
                // the reference's third term, l2 = 0 (no family) or 1 (NA): +0 for tame inputs
                v = v + (i == 0 ? p[0][2] : u[0][2]) * nad;
            } else if (C == 3 && wide) {
                v = v + (i == 0 ? p[0][2] : u[0][2]) * nad;
            }
            row[0] = v;
            if (C == 3) {
                const double n10 = i == 0 ? p[1][0] : u[1][0], n11 = i == 0 ? p[1][1] : u[1][1];
                const double n12 = i == 0 ? p[1][2] : u[1][2];
                const double a1 = n10 * l0 + n11 * l1;
#pragma unroll
                for (int fm = 0; fm < FR; fm++) {
                    const double lf = PH ? r.fm[fm] + naone : na ? 1.0 : r.fm[fm];
                    if (PH) {  // families past Fam write to the junk slot: no branch
                        double *dst = fm < Fam ? row + (fm + 1) * rs : junk;
                        *dst = a1 + n12 * lf;
                    } else if (DB || fm < Fam) {
                        row[(fm + 1) * rs] = a1 + n12 * lf;
                    }
                }
            }
        }
        if (!DB) lds_phase();
        return wide;
    }

    __device__ __forceinline__ double at(uint32_t byte_addr) const {
        return *reinterpret_cast<const double *>(lds + byte_addr);
    }
};

// ---------------------------------------------------------------------------------------
// Dense mixture kernel: every site of the task is gathered from the table.
// The lane owns SPL sites (4*lane + 256*k + j); their class row offsets live in registers.
// ---------------------------------------------------------------------------------------
template <int C, int SPL, int FR, bool XS8, bool BK>
__global__ __launch_bounds__(WAVE, SBZ_MIX_WAVES) void lik_mixture_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int NO = SPL / 4;  // observation words (4 sites each) per lane per feature
    constexpr bool PH = SBZ_TAME != 0;
    constexpr int NCH = (SBZ_NCH == 8 && NO >= 8) ? 8 : 4;
    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    MixTable<C, FR, false, -1, BK, PH> t(a, lds, b);

    // SBZ_OBS_X4 (NO a multiple of 4): word k of a lane holds positions
    // c0 + 1024 (k / 4) + 16 lane + 4 (k % 4) + 0..3, one 16-B load per 4 words; otherwise
    // positions c0 + 256 k + 4 lane + 0..3, one dword load per word.
    constexpr bool X4 = SBZ_OBS_X4 && PH && NO % 4 == 0;
    auto wpos = [&](int c0, int k) {
        return X4 ? c0 + 1024 * (k / 4) + 16 * lane + 4 * (k % 4) : c0 + 4 * lane + 256 * k;
    };
    const __amdgpu_buffer_rsrc_t robs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.obs_fm), (short)0, a.F * a.Np, 0x00020000);
    auto load_obs = [&](int f, int c0, uint32_t (&o)[NO]) {
#pragma unroll
        for (int k = 0; k < NO; k++)  // one lane offset; the word index goes to the scalar offset
            if (!X4) o[k] = __builtin_amdgcn_raw_buffer_load_b32(robs, lane * 4, f * a.Np + c0 + 256 * k, 0);
        if (X4) {
#pragma unroll
            for (int q = 0; q < NO / 4; q++) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(robs, lane * 16, f * a.Np + c0 + 1024 * q, 0);
                o[4 * q] = v[0];
                o[4 * q + 1] = v[1];
                o[4 * q + 2] = v[2];
                o[4 * q + 3] = v[3];
            }
        }
    };

    double m[NCH];  // independent product chains (SBZ_NCH)
    int e;
    // PH: a lane's product fell below 2^-1022 (a zero or tiny cell): the wave re-runs the task
    // with per-factor renormalisation (`force`), which is exact for any normal double.
    uint64_t under;
    bool force = false;
    uint32_t base2[SPL / 2];  // per-site class row offsets (bytes, < 64 KiB), two per register
    MixParams<C, FR> P[NS];   // parameter sets: feature f uses P[(f - fa) % NS]
    uint32_t O[NS][NO];       // observation sets, same rotation

    uint64_t cyc[6] = {0, 0, 0, 0, 0, 0};  // SBZ_LIK_STAMP: cycles per phase
    const uint64_t tstart = lik_stamp();
    // PH: the product chains since the last check; every factor is <= ~1, so a product that left
    // the normal range is still below it here.  Then renormalise.
    auto flush = [&]() {
        if (PH) {
            double mn = fmin(fmin(m[0], m[1]), fmin(m[2], m[3]));
#pragma unroll
            for (int q = 4; q < NCH; q++) mn = fmin(mn, m[q]);
            under |= __ballot(!(mn >= 0x1p-1022));
        }
#pragma unroll
        for (int q = 0; q < NCH; q++)
            if (q < NO) renorm(m[q], e);
    };

    // One feature: build its table from `cur`, issue the loads of feature f + NS - 1 into
    // `fill` (the sets feature f - 1 used), gather.  `live` = false for padding features.
    auto feature = [&](int f, int c0, bool live, const MixParams<C, FR> &cur, const uint32_t (&ob)[NO],
                       MixParams<C, FR> &fill, uint32_t (&ofill)[NO]) {
        const int fk = min(f, fb - 1);
        uint64_t t0 = lik_stamp();
        if (fk < t.nwf0 || fk >= t.nwf0 + t.NWCT) t.prep(fk, fb);  // uniform, once per NWCT features
        uint64_t t1 = lik_stamp();
        const bool wide = t.build(cur, fk) || (PH && force);
        uint64_t t2 = lik_stamp();
        __builtin_amdgcn_sched_barrier(0);
        t.load(min(f + NS - 1, fb - 1), fill);
        load_obs(min(f + NS - 1, fb - 1), c0, ofill);
        uint64_t t3 = lik_stamp();
        if (SBZ_LIK_STAMP) {
            cyc[0] += t1 - t0;
            cyc[1] += t2 - t1;
            cyc[2] += t3 - t2;
        }
        if (SBZ_ABLATE & 1 || !live) {
            // padding feature (or diagnostic build): no gathers
        } else if (!wide) {
            auto cell_at = [&](int i) {  // cell i = 4k + j of the lane
                const int k = i >> 2, j = i & 3;
                const uint32_t bw = base2[2 * k + (j >> 1)];
                const uint32_t bs = (SBZ_ABLATE & 16) ? 0u : (j & 1) ? (bw >> 16) : (bw & 0xffffu);
                const uint32_t xb = (ob[k] >> (8 * j)) & 0xffu;
                return (XS8 && PH && SBZ_ASM_ADDR && !(SBZ_ABLATE & 16)) ? cell_addr(bw, ob[k], j)
                                                                         : bs + (XS8 ? xb : (xb << 3));
            };
            if (SBZ_GPIPE) {
                // software-pipelined gathers: the reads of group g + 1 are issued before the
                // products of group g, so 2 * SBZ_GIF reads are in flight
                constexpr int GQ = SBZ_GIF < SPL ? SBZ_GIF : SPL, NG = SPL / GQ;
                double va[GQ], vb[GQ];
#pragma unroll
                for (int q = 0; q < GQ; q++) va[q] = t.at(cell_at(q));
#pragma unroll
                for (int g = 0; g < NG; g++) {
                    if (g + 1 < NG) {
#pragma unroll
                        for (int q = 0; q < GQ; q++) vb[q] = t.at(cell_at((g + 1) * GQ + q));
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < GQ; q++) m[((g * GQ + q) >> 2) & (NCH - 1)] *= va[q];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < GQ; q++) va[q] = vb[q];
                }
            } else {
#pragma unroll
                for (int k = 0; k < NO; k++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        m[k & (NCH - 1)] *= t.at(cell_at(4 * k + j));
                        // <= SBZ_GIF reads in flight
                        if (j == 3 && (k & (SBZ_GIF / 4 - 1)) == SBZ_GIF / 4 - 1) __builtin_amdgcn_sched_barrier(0);
                    }
            }
            if (!PH || SBZ_RN == 1 || (f - fa) % SBZ_RN == SBZ_RN - 1) flush();
        } else {
            // untamed inputs: renormalise after every factor (exact for any normal double)
            if (PH) flush();  // the products since the last check first
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t bw = base2[2 * k + (j >> 1)];
                    const uint32_t bs = (j & 1) ? (bw >> 16) : (bw & 0xffffu);
                    const uint32_t xb = (ob[k] >> (8 * j)) & 0xffu;
                    mul_exact(m[0], e, t.at((XS8 && PH && SBZ_ASM_ADDR) ? cell_addr(bw, ob[k], j) : bs + (XS8 ? xb : (xb << 3))));
                }
        }
        if (SBZ_LIK_STAMP) cyc[3] += lik_stamp() - t3;
    };

    constexpr bool PR = SBZ_PAIR && PH && !BK && NS == 2;
    // PR: features f (table at 0) and f + 1 (table at 4096 B) with P[0] / O[0] and P[1] / O[1]
    auto feature_pair = [&](int f, int c0) {
        const int fk0 = min(f, fb - 1), fk1 = min(f + 1, fb - 1);
        if (fk0 < t.nwf0 || fk0 >= t.nwf0 + t.NWCT) t.prep(fk0, fb);
        t.tbo = 0;
        const bool wa = t.build(P[0], fk0) || force;
        if (fk1 < t.nwf0 || fk1 >= t.nwf0 + t.NWCT) t.prep(fk1, fb);
        t.tbo = 512;
        const bool wb = t.build(P[1], fk1) || force;
        __builtin_amdgcn_sched_barrier(0);
        t.load(min(f + 2, fb - 1), P[0]);
        t.load(min(f + 3, fb - 1), P[1]);
        const bool live1 = f + 1 < fb;
        auto addr = [&](const uint32_t (&ob)[NO], int i) {
            const int k = i >> 2, j = i & 3;
            const uint32_t bw = base2[2 * k + (j >> 1)];
            if (SBZ_PAIR_ASM) return cell_addr(bw, ob[k], j);
            return ((j & 1) ? (bw >> 16) : (bw & 0xffffu)) + ((ob[k] >> (8 * j)) & 0xffu);
        };
        if (!wa && !wb) {
#pragma unroll
            for (int i = 0; i < SPL; i++) {
                m[(i >> 2) & 3] *= t.at(addr(O[0], i));
                if (live1) m[(i >> 2) & 3] *= t.at(addr(O[1], i) + 4096u);
                if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);
            }
            if (SBZ_RN <= 2 || ((f - fa) >> 1) % (SBZ_RN / 2) == SBZ_RN / 2 - 1) flush();
        } else {
            flush();
#pragma unroll
            for (int i = 0; i < SPL; i++) {
                m[0] *= t.at(addr(O[0], i));
                if (wa) renorm(m[0], e);
            }
            if (live1) {
#pragma unroll
                for (int i = 0; i < SPL; i++) {
                    m[1] *= t.at(addr(O[1], i) + 4096u);
                    if (wb) renorm(m[1], e);
                }
            }
            flush();
        }
        load_obs(min(f + 2, fb - 1), c0, O[0]);
        load_obs(min(f + 3, fb - 1), c0, O[1]);
    };

  for (;;) {
    for (int q = 0; q < NCH; q++) m[q] = 1.0;
    e = 0;
    under = 0;
    for (int c0 = 0; c0 < a.Np; c0 += SPL * WAVE) {
        const uint64_t ts = lik_stamp();
        // classes of this chunk's sites (cls = zc*FamC + fc, padding -> the neutral row); the
        // first NS - 1 features' parameters and observations
        {
            const uint8_t *zb = a.zone + (size_t)b * a.N;
            uint32_t zs[SPL];
            int4 pv[NO];
            uint32_t fw[NO];
#pragma unroll
            for (int k = 0; k < NO; k++) {
                const uint32_t p0 = (uint32_t)wpos(c0, k);  // < Np (arrays padded)
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
#pragma unroll
            for (int j = 0; j < (PR ? NS : NS - 1); j++) {
                t.load(min(fa + j, fb - 1), P[j]);
                load_obs(min(fa + j, fb - 1), c0, O[j]);
            }
            if (PH && t.pwf0 != fa) t.prep_issue(fa, fb);  // the first weights, with the zone bytes
#pragma unroll
            for (int i = 0; i < SPL; i++) {
                const int pos = wpos(c0, i / 4) + (i % 4);
                const int z = (int)zs[i];
                const int fc = (int)((fw[i / 4] >> (8 * (i % 4))) & 0xffu);
                const int zc = z < t.Z ? z + 1 : 0;
                uint32_t off;
                if (BK) off = 8u * (pos < a.N ? bk_row(zc, fc, t.FamC, t.S1) : (uint32_t)(t.FamC * 32));
                else off = (uint32_t)((pos < a.N ? zc * t.FamC + fc : t.ncls) * t.row_bytes);
                if (i & 1) base2[i >> 1] |= off << 16;
                else base2[i >> 1] = off;
            }
        }
        if (SBZ_LIK_STAMP) cyc[4] += lik_stamp() - ts;
        if (PR) {
            for (int f = fa; f < fb; f += 2) feature_pair(f, c0);
        } else {
            for (int f = fa; f < fb; f += NS) {
#pragma unroll
                for (int j = 0; j < NS; j++)
                    feature(f + j, c0, f + j < fb, P[j], O[j], P[(j + NS - 1) % NS], O[(j + NS - 1) % NS]);
            }
        }
    }
    if (PH) flush();
    if (!PH || force || under == 0) break;
    force = true;  // uniform: `under` is a ballot
  }
    double v = (log(m[0]) + log(m[1])) + (log(m[2]) + log(m[3]));
#pragma unroll
    for (int q = 4; q < NCH; q++) v = v + log(m[q]);
    v = v + (double)e * LN2;
    double tot = wave_sum(v);
    if (SBZ_LIK_STAMP) {
        cyc[5] = lik_stamp() - tstart;
        uint64_t c = cyc[0];
#pragma unroll
        for (int q = 1; q < 6; q++) c = a.F4 == q ? cyc[q] : c;
        tot = (double)c;
    }
    finish_chain(a, b, tot);
}

// ---------------------------------------------------------------------------------------
// Dense mixture kernel, double-buffered (opt-in, SBZ_LIK_KERNEL=db; needs the table to fit
// DB_TAB_BYTES).  Measured at cfg5: 99 us per launch vs 95 us for lik_mixture_kernel — without
// the LDS fences and with one parameter set, but at 168 VGPRs, and with the build after the
// gathers (letting the compiler interleave them spilled), so it is not the default.
// Step f gathers feature f from one table buffer, then builds feature f + 1's table into the
// other with no LDS fence between them (distinct static LDS arrays; the buffer address folds
// into the ds_read offset).  One parameter register set: feature f + 2's parameters load right
// after build(f + 1) consumed f + 1's.
// ---------------------------------------------------------------------------------------
template <int C, int SPL, int FR>
__global__ __launch_bounds__(WAVE, SBZ_MIX_WAVES) void lik_mixture_db_kernel(LikArgs a) {
    __shared__ __attribute__((aligned(16))) double tab0[DB_TAB_BYTES / 8];
    __shared__ __attribute__((aligned(16))) double tab1[DB_TAB_BYTES / 8];
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int NO = SPL / 4;  // observation words (4 sites each) per lane per feature
    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    MixTable<C, FR, true> t(a, lds, b, tab0, tab1);

    auto load_obs = [&](int f, int c0, uint32_t (&o)[NO]) {
        const uint32_t *op = reinterpret_cast<const uint32_t *>(a.obs_fm + (size_t)f * a.Np + c0);
#pragma unroll
        for (int k = 0; k < NO; k++) o[k] = op[(uint32_t)(lane + 64 * k)];
    };

    double m[4] = {1.0, 1.0, 1.0, 1.0};  // four independent product chains
    int e = 0;
    uint32_t base2[SPL / 2];  // per-site class row offsets (bytes, < DB_TAB_BYTES), two per register
    MixParams<C, FR> P;       // parameters of the next table to build
    uint32_t O[2][NO];        // observations of the feature being gathered / the next one

    auto cell = [&](auto jc, uint32_t off) -> double {
        constexpr int J = decltype(jc)::value;
        const unsigned char *tb = reinterpret_cast<const unsigned char *>(J ? tab1 : tab0);
        return *reinterpret_cast<const double *>(tb + off);
    };
    auto gather = [&](auto jc, const uint32_t (&ob)[NO], bool wide) {
        if (SBZ_ABLATE & 1) return;
        if (!wide) {
            // launder the packed row offsets: otherwise LICM hoists each word's low half out of
            // the feature loop and keeps 16 more VGPRs live (the SDWA add selects the half)
            // Compiler memory barriers pin the reads here in groups of 8: LDS reads cannot fault
            // and the static tables alias nothing else, so they would otherwise be speculated
            // above earlier branches and all 32 results kept live.
            asm volatile("" ::: "memory");
#if SBZ_DB_LAUNDER
#pragma unroll
            for (int i = 0; i < SPL / 2; i++) asm volatile("" : "+v"(base2[i]));
#endif
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t bw = base2[2 * k + (j >> 1)];
                    const uint32_t bs = (j & 1) ? (bw >> 16) : (bw & 0xffffu);
                    m[k & 3] *= cell(jc, bs + ((ob[k] >> (8 * j)) & 0xffu));
#if SBZ_DB_GBAR
                    // <= 8 reads in flight: the group's products are inputs of the barrier, so
                    // its multiplies complete before the next group's reads are issued
                    if (j == 3 && (k & 1))
                        asm volatile("" : "+v"(m[0]), "+v"(m[1]), "+v"(m[2]), "+v"(m[3])::"memory");
#endif
                }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (q < NO) renorm(m[q], e);
        } else {
            // untamed inputs: renormalise after every factor (exact for any normal double).
            // The base words pass through an empty asm so the compiler cannot treat this path's
            // addresses as common with the fast path's and hoist all 32 above the branch.
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    uint32_t bw = base2[2 * k + (j >> 1)];
                    asm volatile("" : "+v"(bw));
                    const uint32_t bs = (j & 1) ? (bw >> 16) : (bw & 0xffffu);
                    m[0] *= cell(jc, bs + ((ob[k] >> (8 * j)) & 0xffu));
                    renorm(m[0], e);
                }
        }
    };

    for (int c0 = 0; c0 < a.Np; c0 += SPL * WAVE) {
        // classes of this chunk's sites (cls = zc*RPZ + fc, padding -> the neutral row)
        {
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
#pragma unroll
            for (int i = 0; i < SPL; i++) {
                const int pos = c0 + 4 * lane + 256 * (i / 4) + (i % 4);
                const int z = (int)zs[i];
                const int fc = (int)((fw[i / 4] >> (8 * (i % 4))) & 0xffu);
                const int cls = pos < a.N ? ((z < t.Z ? z + 1 : 0) * t.RPZ + fc) : t.ncls;
                const uint32_t off = (uint32_t)(cls * t.row_bytes);
                if (i & 1) base2[i >> 1] |= off << 16;
                else base2[i >> 1] = off;
            }
        }
        // prologue: feature fa's table into buffer 0, feature fa + 1's parameters
        __builtin_amdgcn_sched_barrier(0);
        t.load(fa, P);
        load_obs(fa, c0, O[0]);
        if (fa < t.nwf0 || fa >= t.nwf0 + NWC) t.prep(fa, fb);
        bool wide = t.build(P, fa, tab0);
        t.load(min(fa + 1, fb - 1), P);

        // step J: gather feature f from buffer J; build feature f + 1 into buffer 1 - J
        auto step = [&](auto jc, int f) {
            constexpr int J = decltype(jc)::value;
            const int fn = min(f + 1, fb - 1);
            if (fn < t.nwf0 || fn >= t.nwf0 + NWC) t.prep(fn, fb);  // uniform, once per NWC
            gather(jc, O[J], wide);
            const bool wn = t.build(P, fn, J ? tab0 : tab1);
            t.load(min(f + 2, fb - 1), P);
            load_obs(fn, c0, O[1 - J]);
            wide = wn;
        };
        int f = fa;
        for (; f + 1 < fb; f += 2) {
            step(std::integral_constant<int, 0>(), f);
            step(std::integral_constant<int, 1>(), f + 1);
        }
        if (f < fb) gather(std::integral_constant<int, 0>(), O[0], wide);  // odd tail
    }
    double v = (log(m[0]) + log(m[1])) + (log(m[2]) + log(m[3]));
    v = v + (double)e * LN2;
    const double tot = wave_sum(v);
    finish_chain(a, b, tot);
}

// ---------------------------------------------------------------------------------------
// Dense mixture kernel, wave-specialised (SBZ_LIK_KERNEL=ws; the default where the table fits
// DB_TAB_BYTES and obs hold x*8).  A task (chain b, features [fa, fb)) is one workgroup of
// 1 + NG waves on separate SIMDs:
//   wave 0      the builder: loads the parameters and builds feature f + 1's table (MixTable,
//               DB row layout) into one of two static LDS buffers, plus its `wide` flag;
//   waves 1..NG the gatherers: each owns SPL sites per lane of the chunk and multiplies feature
//               f's cells out of the other buffer.
// One s_barrier per feature hands the buffers over: the builder writes buffer (k+1)&1 in step k,
// which the gatherers last read in step k-1, before the previous barrier.  Table build and
// gathers, which the single-wave kernel runs back to back, overlap on two SIMDs, and each role
// keeps only its own registers live (the gatherers hold no parameters, the builder no sites).
// ---------------------------------------------------------------------------------------
#ifndef SBZ_WS_WAVES
#define SBZ_WS_WAVES 4  // launch bound: minimum waves per SIMD of the wave-specialised kernel
#endif

// s_barrier after this wave's LDS operations completed; a compiler memory barrier on both sides
// (the bare builtin is not one) and, unlike __syncthreads(), no vmcnt drain: prefetched global
// loads stay in flight.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// bytes of one builder's [junk | nwt] region (16-B multiple)
__host__ __device__ constexpr size_t mix_db_lds_bytes_d() { return ((size_t)WAVE + 2 + (size_t)NWC * NW_PER_F) * 8; }

template <int C, int SPL, int FR, int NG, int NB>
__global__ __launch_bounds__(WAVE *(NB + NG), SBZ_WS_WAVES) void lik_mixture_ws_kernel(LikArgs a) {
    __shared__ __attribute__((aligned(16))) double tab0[DB_TAB_BYTES / 8];
    __shared__ __attribute__((aligned(16))) double tab1[DB_TAB_BYTES / 8];
    __shared__ int wflag[2][NB];
    __shared__ double red[NG];
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // builder: junk | nwt
    constexpr int NO = SPL / 4;  // observation words (4 sites each) per lane per feature
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    const int lane = threadIdx.x % WAVE;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    const int nf = fb - fa;
    const int chunk = NG * SPL * WAVE;

    auto builder = [&](auto slot) {
        constexpr int SL = decltype(slot)::value;
        constexpr int BW = SL < 0 ? 0 : SL;  // builder index
        MixTable<C, FR, true, SL> t(a, lds + BW * mix_db_lds_bytes_d(), b, tab0, tab1);
        MixParams<C, FR> P;
        for (int c0 = 0; c0 < a.Np; c0 += chunk) {
            t.load(fa, P);
            if (fa < t.nwf0 || fa >= t.nwf0 + NWC) t.prep(fa, fb);
            bool wide = t.build(P, fa, tab0);
            t.load(min(fa + 1, fb - 1), P);
            if (t.lane == 0) wflag[0][BW] = wide;
            lds_barrier();
            for (int k = 0; k < nf; k++) {
                const int fn = fa + k + 1;
                if (fn < fb) {
                    if (fn < t.nwf0 || fn >= t.nwf0 + NWC) t.prep(fn, fb);
                    wide = t.build(P, fn, (k & 1) ? tab0 : tab1);
                    t.load(min(fn + 1, fb - 1), P);
                    if (t.lane == 0) wflag[(k + 1) & 1][BW] = wide;
                }
                lds_barrier();
            }
        }
        lds_barrier();  // the gatherers' partials
    };
    if (wv < NB) {
        if constexpr (NB == 1) {
            builder(std::integral_constant<int, -1>());
        } else {
            if (wv == 0) builder(std::integral_constant<int, 0>());
            else builder(std::integral_constant<int, 1>());
        }
        return;
    }

    // ------------------------------ gatherers ------------------------------
    const int g = wv - NB;
    auto wide_of = [&](int j) {
        int w = wflag[j][0];
#pragma unroll
        for (int i = 1; i < NB; i++) w |= wflag[j][i];
        return w != 0;
    };
    const int Z = a.Z;
    const int RPZ = MixTable<C, FR, true>::RPZ_DB;
    static_assert(NB == 1 || ZR == 2, "two builder waves split the ZR = 2 zone-class slots");
    const int ncls = (Z + 1) * RPZ;
    const uint32_t row_bytes = (uint32_t)(a.S + 1) * 8u;
    double m[4] = {1.0, 1.0, 1.0, 1.0};  // four independent product chains
    int e = 0;
    uint32_t base2[SPL / 2];  // per-site class row offsets (bytes, < DB_TAB_BYTES), two per register
    uint32_t O[2][NO];        // observations of the feature being gathered / the next one

    auto load_obs = [&](int f, int s0, uint32_t (&o)[NO]) {
        const uint32_t *op = reinterpret_cast<const uint32_t *>(a.obs_fm + (size_t)f * a.Np + s0);
#pragma unroll
        for (int k = 0; k < NO; k++) o[k] = op[(uint32_t)(lane + 64 * k)];
    };
    auto cell = [&](auto jc, uint32_t off) -> double {
        constexpr int J = decltype(jc)::value;
        const unsigned char *tb = reinterpret_cast<const unsigned char *>(J ? tab1 : tab0);
        return *reinterpret_cast<const double *>(tb + off);
    };
    auto gather = [&](auto jc, const uint32_t (&ob)[NO], bool wide) {
        if (SBZ_ABLATE & 1) return;
        if (!wide) {
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t bw = base2[2 * k + (j >> 1)];
                    const uint32_t bs = (j & 1) ? (bw >> 16) : (bw & 0xffffu);
                    m[k & 3] *= cell(jc, bs + ((ob[k] >> (8 * j)) & 0xffu));
                    // <= 8 reads in flight: the group's products are inputs of the barrier
                    if (j == 3 && (k & 1))
                        asm volatile("" : "+v"(m[0]), "+v"(m[1]), "+v"(m[2]), "+v"(m[3])::"memory");
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
                    uint32_t bw = base2[2 * k + (j >> 1)];
                    asm volatile("" : "+v"(bw));
                    const uint32_t bs = (j & 1) ? (bw >> 16) : (bw & 0xffffu);
                    m[0] *= cell(jc, bs + ((ob[k] >> (8 * j)) & 0xffu));
                    renorm(m[0], e);
                }
        }
    };

    for (int c0 = 0; c0 < a.Np; c0 += chunk) {
        const int s0 = c0 + g * SPL * WAVE;  // this gatherer's first position
        {
            const uint8_t *zb = a.zone + (size_t)b * a.N;
            uint32_t zs[SPL];
            int4 pv[NO];
            uint32_t fw[NO];
#pragma unroll
            for (int k = 0; k < NO; k++) {
                const uint32_t p0 = (uint32_t)(s0 + 4 * lane + 256 * k);  // < Np (arrays padded)
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
#pragma unroll
            for (int i = 0; i < SPL; i++) {
                const int pos = s0 + 4 * lane + 256 * (i / 4) + (i % 4);
                const int z = (int)zs[i];
                const int fc = (int)((fw[i / 4] >> (8 * (i % 4))) & 0xffu);
                const int cls = pos < a.N ? ((z < Z ? z + 1 : 0) * RPZ + fc) : ncls;
                const uint32_t off = (uint32_t)cls * row_bytes;
                if (i & 1) base2[i >> 1] |= off << 16;
                else base2[i >> 1] = off;
            }
        }
        load_obs(fa, s0, O[0]);
        lds_barrier();  // feature fa's table
        int k = 0;
        for (; k + 1 < nf; k += 2) {
            load_obs(fa + k + 1, s0, O[1]);
            gather(std::integral_constant<int, 0>(), O[0], wide_of(0));
            lds_barrier();
            load_obs(min(fa + k + 2, fb - 1), s0, O[0]);
            gather(std::integral_constant<int, 1>(), O[1], wide_of(1));
            lds_barrier();
        }
        if (k < nf) {  // odd tail: buffer 0
            gather(std::integral_constant<int, 0>(), O[0], wide_of(0));
            lds_barrier();
        }
    }
    double v = (log(m[0]) + log(m[1])) + (log(m[2]) + log(m[3]));
    v = v + (double)e * LN2;
    const double tot = wave_sum(v);
    if (lane == 0) red[g] = tot;
    lds_barrier();
    if (g == 0) {
        double s = red[0];
#pragma unroll
        for (int i = 1; i < NG; i++) s += red[i];
        finish_chain(a, b, s, lane == 0);
    }
}

// ---------------------------------------------------------------------------------------
// Zone-sparse mixture kernel.  A site outside every zone has class (0, fc), so over those
// sites   sum log T0[fc][x] = sum_{fc,x} n_out[fc][x] * log T0[fc][x].
// With n_all[f][fc][x] (all sites, counted once when the context opens) and the chain's list
// of zoned sites (zone_list_kernel):
//   sum_sites log T = sum_{fc,x} n_all * log T0  +  log prod_zoned T[cls][x]
//                                                 -  log prod_zoned T0[fc][x]
// One log per (fc, x) entry instead of one gather per site: the gathers shrink to the zoned
// sites (two each).  Identical to the per-cell sum up to rounding (~1e-15 relative).
// When a T0 entry with a non-zero count is 0 (the subtraction would be inf - inf) or an input
// is untamed, the feature takes the exact slow path: zoned sites by a per-factor renormalised
// product, the other sites by one log per cell.
// The lane owns ZSPL zoned sites per chunk (lane + 64k); more zoned sites -> more chunks
// (the tables are rebuilt per chunk).
// ---------------------------------------------------------------------------------------
constexpr int CP = 128;  // count entries per feature (FamC * S1 <= CP)

template <int C, int ZSPL, int FR, bool XS8>
__global__ __launch_bounds__(WAVE, SBZ_ZS_WAVES) void lik_zoned_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;
    const int fb = min(a.F, fa + a.fpw);
    MixTable<C, FR> t(a, lds, b);
    const int NC = t.FamC * t.S1;
    const int nz = a.nzs[b];
    const uint32_t *zlb = a.zl + (size_t)b * a.N;
    const uint32_t neutral = (uint32_t)(t.ncls * t.row_bytes);

    double m1[2] = {1.0, 1.0}, m0[2] = {1.0, 1.0};  // products over zoned sites of T and T0
    int e = 0;                                      // exponent of m1 / m0
    double acc = 0.0;                               // sum n_all * log T0 (and slow-path logs)
    uint32_t site[ZSPL], desc[ZSPL];                // zoned site; row offsets T | T0 << 16
    MixParams<C, FR> P[NS];
    uint32_t O[NS][ZSPL];                           // zoned sites' observation bytes (x or x*8)
    int CN[NS][2];                                  // n_all of entries lane, lane + 64

    auto load_zobs = [&](int f, uint32_t (&o)[ZSPL]) {
        const uint8_t *op = a.obs_fm + (size_t)f * a.Np;
#pragma unroll
        for (int k = 0; k < ZSPL; k++) o[k] = op[site[k]];
    };
    auto load_cnt = [&](int f, int (&c)[2]) {
        const int *cp = a.cnt + (size_t)f * CP;
        c[0] = cp[lane];
        c[1] = cp[lane + WAVE];
    };
    // slow path: sum over the chain's non-zoned sites of log T0[fc][x] (one log per cell)
    auto outside_logs = [&](int f) {
        const uint8_t *zb = a.zone + (size_t)b * a.N;
        const uint8_t *op = a.obs_fm + (size_t)f * a.Np;
        double sacc = 0.0;
        for (int s = lane; s < a.N; s += WAVE) {
            const uint32_t xb = op[s];
            const uint32_t row = (uint32_t)(a.famc[s] * t.row_bytes);
            const double v = t.at(row + (XS8 ? xb : (xb << 3)));
            sacc += zb[a.perm[s]] < (uint32_t)t.Z ? 0.0 : log(v);
        }
        return sacc;
    };

    auto feature = [&](int f, bool live, bool first, int zb0, const MixParams<C, FR> &cur,
                       const uint32_t (&ob)[ZSPL], const int (&cc)[2], MixParams<C, FR> &fill,
                       uint32_t (&ofill)[ZSPL], int (&cfill)[2]) {
        const int fk = min(f, fb - 1);
        if (fk < t.nwf0 || fk >= t.nwf0 + NWC) t.prep(fk, fb);
        const bool wide = t.build(cur, fk);
        __builtin_amdgcn_sched_barrier(0);
        t.load(min(f + NS - 1, fb - 1), fill);
        load_zobs(min(f + NS - 1, fb - 1), ofill);
        load_cnt(min(f + NS - 1, fb - 1), cfill);
        if (live) {
            // counts term against the no-zone rows T0 = tab[0 .. NC)
            double cl = 0.0;
            int zero_hit = 0;
#pragma unroll
            for (int q = 0; q < 2; q++) {
                if (q == 1 && NC <= WAVE) break;
                const int l = lane + WAVE * q;
                const double v = t.tab[min(l, NC - 1)];
                const bool use = l < NC && cc[q] > 0;
                zero_hit |= use && v == 0.0;  // checked in every chunk: T0 is gathered per chunk
                if (first) cl += use ? (double)cc[q] * log(v) : 0.0;
            }
            const bool slow = wide || __ballot(zero_hit) != 0;
            if (SBZ_ABLATE & 1) {
                acc += cl;
            } else if (!slow) {
                acc += cl;
#pragma unroll
                for (int k = 0; k < ZSPL; k++) {
                    if (zb0 + WAVE * k < nz) {  // uniform: slot k holds a zoned site in some lane
                        const uint32_t d = desc[k];
                        m1[k & 1] *= t.at((d & 0xffffu) + (XS8 ? ob[k] : (ob[k] << 3)));
                        m0[k & 1] *= t.at((d >> 16) + (XS8 ? ob[k] : (ob[k] << 3)));
                    }
                }
                int e1a, e1b, e0a, e0b;
                e1a = __builtin_amdgcn_frexp_exp(m1[0]);
                m1[0] = __builtin_amdgcn_frexp_mant(m1[0]);
                e1b = __builtin_amdgcn_frexp_exp(m1[1]);
                m1[1] = __builtin_amdgcn_frexp_mant(m1[1]);
                e0a = __builtin_amdgcn_frexp_exp(m0[0]);
                m0[0] = __builtin_amdgcn_frexp_mant(m0[0]);
                e0b = __builtin_amdgcn_frexp_exp(m0[1]);
                m0[1] = __builtin_amdgcn_frexp_mant(m0[1]);
                e += (e1a + e1b) - (e0a + e0b);
            } else {
                // exact slow path (rare: zero / untamed table entries)
#pragma unroll
                for (int k = 0; k < ZSPL; k++) {
                    const uint32_t d = desc[k];
                    m1[0] *= t.at((d & 0xffffu) + (XS8 ? ob[k] : (ob[k] << 3)));
                    renorm(m1[0], e);
                }
                if (first) acc += outside_logs(f);
            }
        }
    };

    const int nchunk = max(1, (nz + WAVE * ZSPL - 1) / (WAVE * ZSPL));
    for (int ch = 0; ch < nchunk; ch++) {
        const int zb0 = ch * WAVE * ZSPL;
#pragma unroll
        for (int k = 0; k < ZSPL; k++) {
            const int j = zb0 + lane + WAVE * k;
            const uint32_t ent = zlb[min(j, a.N - 1)];
            const uint32_t cls = ent >> 24;
            const uint32_t fc = cls - (cls / (uint32_t)t.FamC) * (uint32_t)t.FamC;
            const bool in = j < nz;
            site[k] = in ? (ent & 0xffffffu) : 0u;
            desc[k] = in ? ((uint32_t)(cls * t.row_bytes) | ((uint32_t)(fc * t.row_bytes) << 16))
                         : (neutral | (neutral << 16));
        }
#pragma unroll
        for (int j = 0; j < NS - 1; j++) {
            t.load(min(fa + j, fb - 1), P[j]);
            load_zobs(min(fa + j, fb - 1), O[j]);
            load_cnt(min(fa + j, fb - 1), CN[j]);
        }
        for (int f = fa; f < fb; f += NS) {
#pragma unroll
            for (int j = 0; j < NS; j++) {
                const int jf = (j + NS - 1) % NS;
                feature(f + j, f + j < fb, ch == 0, zb0, P[j], O[j], CN[j], P[jf], O[jf], CN[jf]);
            }
        }
    }
    double v = (log(m1[0]) + log(m1[1])) - (log(m0[0]) + log(m0[1]));
    v = v + (double)e * LN2;
    v = v + acc;
    const double tot = wave_sum(v);
    finish_chain(a, b, tot);
}

// ---------------------------------------------------------------------------------------
// Zone-sparse mixture kernel, direct (SBZ_LIK_KERNEL=zd).  Same decomposition as
// lik_zoned_kernel,
//   ll_f = sum_{fc,x} n_all[f][fc][x] log T0[fc][x] + log prod_zoned T - log prod_zoned T0,
// but without a class table: the feature's parameter column (p_global, p_zones, a row of
// ones for "no family", p_fam; the NA column is 1.0) is staged in ~1 KB of LDS and a zoned
// cell gathers its three l_c and forms T = (n0 l0 + n1 l1) + n2 l2 and T0 = n0' l0 + n2' l2 in
// registers (reference operation order; a +0 term of a tame input is left out, x + 0 == x).
// One lane per (fc, x) count entry takes the log of T0.  Zoned observations come as one dword
// (4 features) per site from the site-major obs8 rows.  The no-zone sites, 80 % at the bench's
// cfg5, cost no gathers at all.
// Features whose inputs are not all tame, or with a zero / non-finite T0 entry that has a
// non-zero count, take the exact slow path (every site of the feature, one log per cell).
// Requires: xs8, 2 (Z + 2 + Fam)(S + 1) <= 320, FamC * (S + 1) <= 64 (host check at launch).
// HFM: 0 no zoned site has a family (C == 2 or no families), 1 all sites have one, 2 mixed.
// ---------------------------------------------------------------------------------------
#ifndef SBZ_ZD_WAVES
#define SBZ_ZD_WAVES 2
#endif
constexpr int ZD_NT = 5;  // LDS-DMA dword loads per column image: 2 (Z + 2 + Fam)(S + 1) <= 320
constexpr int ZD_FB = 4;  // features per batch (one observation dword)

__device__ __forceinline__ double uniform_f64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

template <int C, int ZSPL, int HFM>
__global__ __launch_bounds__(WAVE, SBZ_ZD_WAVES) void lik_zdirect_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x;
    const int b = blockIdx.y;
    const int fa = blockIdx.x * a.fpw;  // fpw % 4 == 0
    const int fb = min(a.F, fa + a.fpw);
    const int S = a.S, S1 = S + 1, Z = a.Z, Fam = C == 3 ? a.Fam : 0, FamC = a.FamC;
    const int RL = Z + 2 + Fam;                      // rows: pg, pz[0..Z), ones, pf[0..Fam)
    const int NT = (2 * RL * S1 + WAVE - 1) / WAVE;  // LDS-DMA dword loads per column (<= ZD_NT)
    const int RLS = NT * (WAVE / 2);                 // one column image, doubles
    double *stg = reinterpret_cast<double *>(lds);   // [2][ZD_FB][RLS] column images
    double *nwt = stg + 2 * ZD_FB * RLS;
    const int NC = FamC * S1;
    const int nz = a.nzs[b];
    const uint32_t zfs = (uint32_t)(a.F * S);

    // weights: NWC features at a time, layout as MixTable::prep
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
        wave_lds_sync();
        double *o = nwt + k * NW_PER_F;
#pragma unroll
        for (int hz = 0; hz < 2; hz++) {
            o[2 * (2 * hp + hz)] = n[hz][0];
            o[2 * (2 * hp + hz) + 1] = n[hz][1];
            o[8 + 2 * hz + hp] = n[hz][2];
        }
        nwbad = __ballot(!ok);
        nwf0 = f0;
        wave_lds_sync();
    };

    // LDS-DMA sources: dword t*64 + lane of a column image is double (r, x) = ((t*64 + lane) / 2
    // as r * S1 + x), half (lane & 1).  NA column, "no family" row and padding read a.ones,
    // which advances with the feature like a parameter row (F * S + 8 ones).
    const char *dsrc[ZD_NT];
#pragma unroll
    for (int t = 0; t < ZD_NT; t++) {
        const int i = t * WAVE + lane, dr = i >> 1, r = dr / S1, x = dr - r * S1;
        const double *p;
        if (r >= RL || x == S || r == Z + 1) p = a.ones;
        else if (r == 0) p = a.pg + (size_t)b * zfs + x;
        else if (r <= Z) p = a.pz + ((size_t)b * Z + (r - 1)) * zfs + x;
        else p = a.pf + ((size_t)b * Fam + (r - Z - 2)) * zfs + x;
        dsrc[t] = reinterpret_cast<const char *>(p) + 4 * (i & 1);
    }
    auto dma_column = [&](int f, double *img) {
        const size_t fo = (size_t)f * S * 8;
#pragma unroll
        for (int t = 0; t < ZD_NT; t++)
            if (t < NT)  // uniform
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(dsrc[t] + fo),
                    (__attribute__((address_space(3))) void *)(img + t * (WAVE / 2)), 4, 0, 0);
    };
    auto dma = [&](int fg, int buf) {
#pragma unroll
        for (int j = 0; j < ZD_FB; j++) dma_column(min(fg + j, fb - 1), stg + (buf * ZD_FB + j) * RLS);
    };
    // count lane: entry (fc, x) = (lane / S1, lane % S1)
    const int cfc = min(lane, NC - 1) / S1, cx = min(lane, NC - 1) - cfc * S1;
    const uint32_t c_l2 = (uint32_t)((Z + 1 + cfc) * S1 + cx);
    const bool c_hf = C == 3 && cfc > 0;

    double m1[2] = {1.0, 1.0}, m0[2] = {1.0, 1.0};
    int e = 0;
    double acc = 0.0;
    uint64_t slowm = 0;  // features [fa, fb) for the exact slow path (fpw <= 64)
    uint32_t desc[ZSPL], obase[ZSPL];
    uint32_t hfm = 0;  // HFM == 2: bit q = the lane's slot-q site has a family

    auto load_c = [&](int fg, int (&c)[ZD_FB]) {
#pragma unroll
        for (int j = 0; j < ZD_FB; j++) c[j] = a.cnt[(size_t)min(fg + j, fb - 1) * CP + min(lane, NC - 1)];
    };
    auto load_o = [&](int fg, uint32_t (&o)[ZSPL]) {
#pragma unroll
        for (int k = 0; k < ZSPL; k++)
            o[k] = *reinterpret_cast<const uint32_t *>(a.obs8 + obase[k] + (uint32_t)fg);
    };
    auto at = [&](uint32_t byte) { return *reinterpret_cast<const double *>(lds + byte); };
    // cc[j] with a loop-variable j, without a dynamically indexed register array
    auto ccj = [](const int (&c)[ZD_FB], int j) { return j == 0 ? c[0] : j == 1 ? c[1] : j == 2 ? c[2] : c[3]; };

    // One batch of ZD_FB = 4 features (one observation dword per zoned site): the batch's four
    // column images landed in buffer buf during the previous batch; issue the next batch's DMA
    // into the other buffer, then count terms and zoned cells.
    auto batch = [&](int fg, int buf, bool first, int zb0, const int (&cc)[ZD_FB], const uint32_t (&ob)[ZSPL],
                     int (&cfill)[ZD_FB], uint32_t (&ofill)[ZSPL]) {
        if (fg + ZD_FB - 1 >= nwf0 + NWC) prep(fg);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this batch's images have landed
        wave_lds_sync();  // and the previous batch's reads of the other buffer are done
        dma(fg + ZD_FB, buf ^ 1);
        load_c(fg + ZD_FB, cfill);
        load_o(min(fg + ZD_FB, fb - 1) & ~3, ofill);
        const double *sbuf = stg + buf * ZD_FB * RLS;
        uint32_t slowb = 0;  // bit j: feature fg + j takes the slow path (or is padding)
        double cl = 0.0;
#pragma unroll 1
        for (int j = 0; j < ZD_FB; j++) {
            const double *sj = sbuf + j * RLS;
            int ok = 1;
#pragma unroll
            for (int k = 0; k < (ZD_NT + 1) / 2; k++) ok &= (int)tame(sj[min(lane + WAVE * k, RLS - 1)]);
            const bool wide = ((nwbad >> (2 * (fg + j - nwf0))) & 3ull) != 0 || __ballot(!ok) != 0;
            const double *nk = static_cast<const double *>(
                __builtin_assume_aligned(nwt + (fg + j - nwf0) * NW_PER_F, 16));
            const double2 n0p = *reinterpret_cast<const double2 *>(nk + 0);
            const double2 n2p = *reinterpret_cast<const double2 *>(nk + 4);
            const double2 c2p = *reinterpret_cast<const double2 *>(nk + 8);
            double t0 = (c_hf ? n2p.x : n0p.x) * sj[cx];
            if (C == 3) t0 = t0 + (c_hf ? c2p.y * sj[c_l2] : 0.0);
            const bool use = lane < NC && ccj(cc, j) > 0;
            const bool bad = use && !(t0 > 0.0 && t0 < __builtin_huge_val());
            const bool sl = fg + j >= fb || wide || __ballot(bad) != 0;
            slowb |= sl ? 1u << j : 0u;
            if (first && use && !sl) cl += (double)ccj(cc, j) * log(t0);
            __builtin_amdgcn_sched_barrier(0);  // one log's temporaries at a time
        }
        acc += cl;
#pragma unroll 1
        for (int j = 0; j < ZD_FB; j++) {
            if ((slowb >> j) & 1u) {
                if (first && fg + j < fb) slowm |= 1ull << (fg + j - fa);  // after the main loop
                continue;
            }
            const double *nk = static_cast<const double *>(
                __builtin_assume_aligned(nwt + (fg + j - nwf0) * NW_PER_F, 16));
            // the weights are wave-uniform: into SGPRs
            auto pair = [&](int i) {
                const double2 v = *reinterpret_cast<const double2 *>(nk + i);
                return make_double2(uniform_f64(v.x), uniform_f64(v.y));
            };
            const double2 n0p = pair(0), n2p = pair(4), c2p = pair(8);  // h = 0, 2; c2 of (0, 2)
            const double2 z1 = pair(2), z3 = pair(6), c2z = pair(10);   // h = 1, 3; c2 of (1, 3)
            const uint32_t sb = (uint32_t)((buf * ZD_FB + j) * RLS * 8);
            const int sh = 8 * j;
            // groups of 4 slots: every gather of the group is issued before the arithmetic
#pragma unroll
            for (int g = 0; g < ZSPL; g += 4) {
                if (zb0 + WAVE * g >= nz) break;  // uniform
                double L0[4], L1[4], L2[4];
#pragma unroll
                for (int q = g; q < g + 4; q++) {
                    if (zb0 + WAVE * q >= nz) break;  // uniform
                    const uint32_t x8 = sb + ((ob[q] >> sh) & 0xffu);
                    const uint32_t d = desc[q];
                    L0[q - g] = at(x8);
                    L1[q - g] = at((d & 0xffffu) + x8);
                    if (HFM != 0) L2[q - g] = at((d >> 16) + x8);
                }
#pragma unroll
                for (int q = g; q < g + 4; q++) {
                    if (zb0 + WAVE * q >= nz) break;  // uniform
                    const double l0 = L0[q - g], l1 = L1[q - g];
                    double T, T0;
                    if (HFM == 0) {
                        T = z1.x * l0 + z1.y * l1;
                        T0 = n0p.x * l0;
                    } else if (HFM == 1) {
                        const double l2 = L2[q - g];
                        T = (z3.x * l0 + z3.y * l1) + c2z.y * l2;
                        T0 = n2p.x * l0 + c2p.y * l2;
                    } else {
                        const double l2 = L2[q - g];
                        const bool h = (hfm >> q) & 1u;
                        T = (h ? z3.x : z1.x) * l0 + (h ? z3.y : z1.y) * l1;
                        T0 = (h ? n2p.x : n0p.x) * l0;
                        if (h) {
                            T = T + c2z.y * l2;
                            T0 = T0 + c2p.y * l2;
                        }
                    }
                    m1[q & 1] *= T;
                    m0[q & 1] *= T0;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            int e1a, e1b, e0a, e0b;
            e1a = __builtin_amdgcn_frexp_exp(m1[0]);
            m1[0] = __builtin_amdgcn_frexp_mant(m1[0]);
            e1b = __builtin_amdgcn_frexp_exp(m1[1]);
            m1[1] = __builtin_amdgcn_frexp_mant(m1[1]);
            e0a = __builtin_amdgcn_frexp_exp(m0[0]);
            m0[0] = __builtin_amdgcn_frexp_mant(m0[0]);
            e0b = __builtin_amdgcn_frexp_exp(m0[1]);
            m0[1] = __builtin_amdgcn_frexp_mant(m0[1]);
            e += (e1a + e1b) - (e0a + e0b);
        }
    };

    const int nchunk = max(1, (nz + WAVE * ZSPL - 1) / (WAVE * ZSPL));
    const uint32_t *zlb = a.zl + (size_t)b * a.N;
    for (int ch = 0; ch < nchunk; ch++) {
        const int zb0 = ch * WAVE * ZSPL;
        hfm = 0;
#pragma unroll
        for (int q = 0; q < ZSPL; q++) {
            const int jj = zb0 + lane + WAVE * q;
            const uint32_t ent = jj < nz ? zlb[min(jj, a.N - 1)] : 0u;  // beyond nz: stale
            const uint32_t cls = ent >> 24;
            const uint32_t zc = cls / (uint32_t)FamC;
            const uint32_t fc = cls - zc * (uint32_t)FamC;
            if (HFM == 2) hfm = fc > 0 ? (hfm | (1u << q)) : hfm;
            // a slot beyond nz reads the all-NA row N of obs8: l0 = l1 = l2 = 1, so its factor
            // T / T0 is (sum of normalised weights) / (sum of normalised weights) = 1 +- 1 ulp
            const int site = jj < nz ? a.perm[ent & 0xffffffu] : a.N;
            obase[q] = (uint32_t)site * (uint32_t)a.F4;
            desc[q] = (uint32_t)(zc * S1 * 8) | ((uint32_t)((Z + 1 + fc) * S1 * 8) << 16);
        }
        if (fa < nwf0 || fa + ZD_FB - 1 >= nwf0 + NWC) prep(fa);
        int Cc[ZD_FB], Cn[ZD_FB];
        uint32_t Oc[ZSPL], On[ZSPL];
        wave_lds_sync();
        dma(fa, 0);
        load_c(fa, Cc);
        load_o(fa, Oc);
        int buf = 0;
#pragma unroll 1
        for (int fg = fa; fg < fb; fg += ZD_FB) {
            batch(fg, buf, ch == 0, zb0, Cc, Oc, Cn, On);
#pragma unroll
            for (int j = 0; j < ZD_FB; j++) Cc[j] = Cn[j];
#pragma unroll
            for (int q = 0; q < ZSPL; q++) Oc[q] = On[q];
            buf ^= 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) prefetch
    }
    // exact slow path (rare: untamed inputs, or a zero T0 entry with a non-zero count): every
    // site of the feature, the reference cell, one log each
    while (slowm) {
        const int f = fa + __builtin_ctzll(slowm);
        slowm &= slowm - 1;
        if (f < nwf0 || f >= nwf0 + NWC) prep(f);
        wave_lds_sync();
        dma_column(f, stg);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_lds_sync();
        const double *nk = nwt + (f - nwf0) * NW_PER_F;
        const uint8_t *zb = a.zone + (size_t)b * a.N;
        const uint8_t *op = a.obs_fm + (size_t)f * a.Np;
        double sacc = 0.0;
        for (int p = lane; p < a.N; p += WAVE) {
            const int z = zb[a.perm[p]];
            const int fc = C == 3 ? a.famc[p] : 0;
            const uint32_t x8 = op[p];  // xs8
            const bool na = x8 == (uint32_t)(S * 8);
            const int hz = z < Z ? 1 : 0, hf = fc > 0 ? 1 : 0;
            const int h = hz | (hf << 1);
            const double n0 = nk[2 * h], n1 = nk[2 * h + 1];
            const double l0 = at(x8);
            const double l1 = hz ? at((uint32_t)((1 + z) * S1 * 8) + x8) : (na ? 1.0 : 0.0);
            double v = n0 * l0 + n1 * l1;
            if (C == 3) {
                const double l2 = hf ? at((uint32_t)((Z + 1 + fc) * S1 * 8) + x8) : (na ? 1.0 : 0.0);
                v = v + nk[8 + 2 * hz + hf] * l2;
            }
            sacc += log(v);
        }
        acc += sacc;
    }
    double v = (log(m1[0]) + log(m1[1])) - (log(m0[0]) + log(m0[1]));
    v = v + (double)e * LN2;
    v = v + acc;
    const double tot = wave_sum(v);
    finish_chain(a, b, tot);
}

// Per-chain ordered list of zoned sites for lik_zoned_kernel: zl[b][j] = position | cls << 24
// (position in the family-sorted site order, cls = (z+1)*FamC + fc), j < nzs[b].  One wave per
// chain.
__global__ void zone_list_kernel(int N, int Z, int FamC, const uint8_t *zone, const uint8_t *famc,
                                 const int *perm, uint32_t *zl, int *nzs) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const uint8_t *zb = zone + (size_t)b * N;
    uint32_t *out = zl + (size_t)b * N;
    int count = 0;
    for (int s0 = 0; s0 < N; s0 += WAVE) {
        const int s = s0 + lane;
        const int z = s < N ? zb[perm[s]] : SBZ_NONE;
        const bool in = z < Z;
        const uint64_t mask = __ballot(in);
        if (in) {
            const int pos = count + (int)__builtin_amdgcn_mbcnt_hi(
                                        (uint32_t)(mask >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
            out[pos] = (uint32_t)s | ((uint32_t)((z + 1) * FamC + famc[s]) << 24);
        }
        count += __popcll(mask);
    }
    if (lane == 0) nzs[b] = count;
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
// Source kernel: cell = w_norm[src] * l_src.  Rows (each S1 doubles):
//   T0[h]            h = hz | hf<<1     w_norm[h][0] * l0                      rows 0..3
//   T1[z][hf]        has_zone           w_norm[1|hf<<1][1] * l1                rows 4..4+2Z-1
//   T2[fam][hz]      has_family         w_norm[hz|2][2] * l2                   rows 4+2Z..
//   Z0[h]            selected component the site lacks: weight w_c * 0 / sum_h (0, or NaN when
//                    sum_h = 0), lh 0
//   N1               neutral row (padded sites)
// A selected weight of exactly 0 makes the chain -inf whatever the other cells hold
// (model.py:181-182): zrow[r] flags such rows per feature, and a feature with one runs the
// per-cell path, which checks every cell's row.
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
        finish_chain(a, b, 0.0);
        return;
    }
    const int S = a.S, S1 = a.S + 1, Z = a.Z;
    const int Fam = (C == 3) ? a.Fam : 0;
    const int off1 = 4, off2 = 4 + 2 * Z, rz = 4 + 2 * Z + 2 * Fam, rn = rz + 4;
    uint8_t *zrow = lds + NW_BYTES + (size_t)(rn + 1) * S1 * 8;
    const size_t zfs = (size_t)a.F * S;
    const double *pgb = a.pg + (size_t)b * zfs;
    const double *pzb = a.pz + (size_t)b * Z * zfs;
    const double *pfb = (C == 3) ? a.pf + (size_t)b * Fam * zfs : nullptr;
    const double *wb = a.w + (size_t)b * a.F * C;
    const uint8_t *zb = a.zone + (size_t)b * a.N;
    const int row_bytes = S1 * 8;
    const int shift = a.xs8 ? 0 : 3;

    for (int x = lane; x < S1; x += WAVE) tab[rn * S1 + x] = 1.0;

    double m = 1.0;
    int e = 0;
    uint32_t zw = 0;
    for (int c0 = 0; c0 < a.Np; c0 += SPL * WAVE) {
        uint32_t rows[SPL];
#pragma unroll
        for (int k = 0; k < SPL / 4; k++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int s = c0 + 4 * lane + 256 * k + j;  // position (family-sorted order)
                uint32_t r = (uint32_t)rn * 0x01010101u;
                if (s < a.N) {
                    const int z = zb[a.perm[s]];
                    const bool hz = z < Z;
                    const int fc = (C == 3) ? a.famc[s] : 0;
                    const bool hf = fc > 0;
                    const int r0 = (hz ? 1 : 0) | (hf ? 2 : 0);
                    const int r1 = hz ? off1 + 2 * z + (hf ? 1 : 0) : rz + r0;
                    const int r2 = hf ? off2 + 2 * (fc - 1) + (hz ? 1 : 0) : rz + r0;
                    r = (uint32_t)r0 | ((uint32_t)r1 << 8) | ((uint32_t)r2 << 16) | ((uint32_t)(rz + r0) << 24);
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
                    tab[(rz + h) * S1 + x] = nw[h * 4 + 0] * 0.0;
                }
                for (int z = 0; z < Z; z++) {
                    const double l1 = na ? 1.0 : pzb[z * zfs + off];
                    const double v0 = nw[1 * 4 + 1] * l1, v1 = nw[3 * 4 + 1] * l1;
                    bad |= (int)!safe_factor(v0) | (int)!safe_factor(v1);
                    tab[(off1 + 2 * z) * S1 + x] = v0;
                    tab[(off1 + 2 * z + 1) * S1 + x] = v1;
                }
                for (int i = 0; i < Fam; i++) {
                    const double l2 = na ? 1.0 : pfb[i * zfs + off];
                    const double v0 = nw[2 * 4 + 2] * l2, v1 = nw[3 * 4 + 2] * l2;
                    bad |= (int)!safe_factor(v0) | (int)!safe_factor(v1);
                    tab[(off2 + 2 * i) * S1 + x] = v0;
                    tab[(off2 + 2 * i + 1) * S1 + x] = v1;
                }
            }
            for (int r = lane; r <= rn; r += WAVE) {  // weights of exactly 0, by table row
                const double wr = r < 4 ? nw[r * 4] : r < off2 ? nw[(1 | (((r - 4) & 1) << 1)) * 4 + 1]
                                : r < rz ? nw[(2 | ((r - off2) & 1)) * 4 + 2] : r < rn ? nw[(r - rz) * 4] * 0.0 : 1.0;
                zrow[r] = wr == 0.0 ? 1 : 0;
                bad |= wr == 0.0;
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
                    const uint32_t rr = (rows[4 * k + j] >> (8 * (c < (uint32_t)C ? c : 3u))) & 0xff;
                    const int addr = NW_BYTES + (int)rr * row_bytes +
                                     (int)(((o[k] >> (8 * j)) & 0xff) << shift);
                    if (wide) {
                        mul_exact(m, e, *reinterpret_cast<const double *>(lds + addr));
                        zw |= zrow[rr];
                    } else {
                        m *= *reinterpret_cast<const double *>(lds + addr);
                    }
                }
                if (k & 1) renorm(m, e);
            }
            renorm(m, e);
            wave_lds_sync();
        }
    }
    const double v = log(m) + (double)e * LN2;
    const double tot = wave_sum(v);
    finish_chain(a, b, tot, lane == 0, __ballot(zw != 0) != 0);
}

// ---------------------------------------------------------------------------------------
// Source kernel, table form (lik_source_rc_kernel; the default where it applies).  Same rows as
// lik_source_kernel (T0[h] 0..3, T1[z][hf] from 4, T2[fam][hz] from 4 + 2Z, the zero row rz, the
// neutral row rn), but the repack writes each cell's ROW INDEX (its source byte mapped through
// the chain's zone and the site's family, repack_source_kernel with `rows`), so a cell costs one
// multiply-add for its address, one ds_read_b64 and one v_mul_f64.  Per feature each lane loads
// (buffer loads, scalar per-feature offsets, one feature ahead) p_global[x], the p_zones rows
// lg, lg + G and the p_families rows lg, lg + G of its state x = lane % S1 (NA lanes read
// out of range: 0, plus `naone` = 1), and writes T0[lg] (lg < 4), the two T1 rows of each zone
// and the two T2 rows of each family.  Normalised weights come from per-batch LDS (prep).  Inputs
// are checked as in the dense kernel (one unsigned max; products checked when renormalised, the
// task re-run per factor when one left the normal range, e.g. a zero weight's -inf cell).
// ---------------------------------------------------------------------------------------
constexpr int SRC_NWC = 32;  // features per normalised-weight batch
template <int C, int SPL, bool XS8>
__global__ __launch_bounds__(WAVE, 3) void lik_source_rc_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int NO = SPL / 4;
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
    const int row_bytes = S1 * 8;
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
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.src_fm + (size_t)b * a.F * a.Np), (short)0, a.F * a.Np, 0x00020000);
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
    // a product that left the normal range (0, tiny, or NaN: fmin would drop a NaN) re-runs the
    // task per factor, where every cell's row is checked for a zero weight
    auto flush = [&]() {
        constexpr double T = 0x1p-1022;
        under |= __ballot(!(m[0] >= T && m[1] >= T && m[2] >= T && m[3] >= T));
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (q < NO) renorm(m[q], e);
    };
    auto feature = [&](int f, int c0, bool live, const SrcParams &cur, const uint32_t (&ob)[NO],
                       const uint32_t (&rb)[NO], SrcParams &fill, uint32_t (&ofill)[NO], uint32_t (&rfill)[NO]) {
        const int fk = min(f, fb - 1);
        if (fk < nwf0 || fk >= nwf0 + SRC_NWC) prep(fk);
        const bool wide = build(cur, fk) || force;
        __builtin_amdgcn_sched_barrier(0);
        const int fn = min(f + 1, fb - 1);
        load(fn, fill);
        load_words(robs, fn, c0, ofill);
        load_words(rsrc, fn, c0, rfill);
        if (!live) return;
        auto addr = [&](int k, int j) {
            const uint32_t xb = (ob[k] >> (8 * j)) & 0xffu;
            const uint32_t rr = (rb[k] >> (8 * j)) & 0xffu;
            return rr * (uint32_t)row_bytes + (XS8 ? xb : (xb << 3));
        };
        if (!wide) {
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    m[k & 3] *= *reinterpret_cast<const double *>(lds + addr(k, j));
                    if (j == 3 && (k & 3) == 3) __builtin_amdgcn_sched_barrier(0);
                }
            if ((f - fa) % SBZ_RN == SBZ_RN - 1) flush();
        } else {
            flush();
#pragma unroll
            for (int k = 0; k < NO; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    mul_exact(m[0], e, *reinterpret_cast<const double *>(lds + addr(k, j)));
                    zw |= zrow[(rb[k] >> (8 * j)) & 0xffu];
                }
        }
    };

    for (;;) {
        m[0] = m[1] = m[2] = m[3] = 1.0;
        e = 0;
        under = 0;
        for (int c0 = 0; c0 < a.Np; c0 += SPL * WAVE) {
            load(fa, P[0]);
            load_words(robs, fa, c0, O[0]);
            load_words(rsrc, fa, c0, R[0]);
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
    finish_chain(a, b, tot, lane == 0, __ballot(zw != 0) != 0);
}

// Row-major source [B][N][F] -> feature-major [B][F][Np] in the family-sorted site order
// (padded sites -> component 0).  One workgroup transposes a tile of RP_T positions x RP_F
// features through LDS.  Read side: RP_F / 16 lanes per site row, each loading 16 feature bytes
// as 4-byte words (F a multiple of 4); every pass's loads are issued before the first is used.
// Write side: 4 lanes per feature, each storing 16 position bytes per 64-position subtile.
#ifndef SBZ_RP_T
#define SBZ_RP_T 256
#endif
#ifndef SBZ_RP_NT
#define SBZ_RP_NT 0  // non-temporal loads (1) / stores (2) in the repack
#endif
#ifndef SBZ_RP_F
#define SBZ_RP_F 64
#endif
constexpr int RP_T = SBZ_RP_T;  // positions per workgroup (a multiple of 64)
constexpr int RP_F = SBZ_RP_F;  // features per workgroup (a multiple of 16, RP_F / 16 divides 256)
// With `zone` (lik_source_rc_kernel) each byte is the cell's table row instead: the source
// component c mapped through the chain's zone of the site and its family class (rows as in
// lik_source_rc_kernel; a component the site lacks, or c >= C -> the zero row; padding -> the
// neutral row).
__global__ __launch_bounds__(256) void repack_source_kernel(int N, int F, int Np, const int *perm,
                                                            const uint8_t *src, uint8_t *dst,
                                                            const uint8_t *zone = nullptr,
                                                            const uint8_t *famc = nullptr, int Z = 0,
                                                            int Fam = 0, int C = 3) {
    constexpr int RW = RP_F / 4 + 1;  // words per LDS row (odd: the write side's 4 position
                                      // groups fall in distinct banks)
    constexpr int LR = RP_F / 16;     // lanes per site row
    constexpr int RPP = 256 / LR;     // rows per pass
    constexpr int NP = RP_T / RPP;    // passes
    __shared__ uint32_t tile[RP_T][RW];  // [position][feature word]
    const int tid = threadIdx.x;
    const int p0 = blockIdx.x * RP_T, f0 = blockIdx.y * RP_F;
    const size_t b = blockIdx.z;
    const int l = tid % LR, rg = tid / LR;  // lane l of row group rg: features f0 + 16 l ..
    const int fq = f0 + 16 * l;
    const bool words = (F & 3) == 0 && fq + 16 <= F;
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
                for (int k = 0; k < 4; k++) w[t][k] = (SBZ_RP_NT & 1) ? __builtin_nontemporal_load(wp + k) : wp[k];
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
    const int off2 = 4 + 2 * Z, rz = off2 + 2 * Fam, rn = rz + 4;
#pragma unroll
    for (int t = 0; t < NP; t++) {
        if (zone) {
            // row map of this position: byte c = table row of component c (c = 3: c >= C)
            uint32_t map;
            if (row[t] >= 0) {
                const int z = zone[b * N + row[t]];
                const bool hz = z < Z;
                const int fc = (C == 3) ? famc[p0 + RPP * t + rg] : 0;
                const bool hf = fc > 0;
                const uint32_t r0 = (hz ? 1u : 0u) | (hf ? 2u : 0u);
                const uint32_t rl = (uint32_t)rz + r0;  // a component the site lacks: zero row of h
                const uint32_t r1 = hz ? (uint32_t)(4 + 2 * z + (hf ? 1 : 0)) : rl;
                const uint32_t r2 = (C == 3 && hf) ? (uint32_t)(off2 + 2 * (fc - 1) + (hz ? 1 : 0)) : rl;
                map = r0 | (r1 << 8) | (r2 << 16) | (rl << 24);
            } else {
                map = (uint32_t)rn * 0x01010101u;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t x = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t c = min((w[t][k] >> (8 * j)) & 0xffu, 3u);
                    x |= ((map >> (8 * c)) & 0xffu) << (8 * j);
                }
                w[t][k] = x;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) tile[RPP * t + rg][4 * l + k] = w[t][k];
    }
    __syncthreads();
    const uint8_t *tb = reinterpret_cast<const uint8_t *>(&tile[0][0]);
    const int q = tid & 3;  // positions p0 + 64 t + 16 q .. of feature f0 + fr
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
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4 *dp = reinterpret_cast<u32x4 *>(drow + 64 * t);
            const u32x4 ov = {o[0], o[1], o[2], o[3]};
            if (SBZ_RP_NT & 2)
                __builtin_nontemporal_store(ov, dp);
            else
                *dp = ov;
        }
    }
}

// The mixture table kernel for these template choices (dense or zone-sparse).
template <int C, int FR>
const void *mix_db_kernel_x(int spl) {
    switch (spl) {
        case 4: return reinterpret_cast<const void *>(&lik_mixture_db_kernel<C, 4, FR>);
        case 8: return reinterpret_cast<const void *>(&lik_mixture_db_kernel<C, 8, FR>);
        case 16: return reinterpret_cast<const void *>(&lik_mixture_db_kernel<C, 16, FR>);
        default: return reinterpret_cast<const void *>(&lik_mixture_db_kernel<C, 32, FR>);
    }
}

const void *mix_db_kernel(int C, int fr, int spl) {
    if (C == 3) return fr == 4 ? mix_db_kernel_x<3, 4>(spl) : mix_db_kernel_x<3, 8>(spl);
    return mix_db_kernel_x<2, 4>(spl);
}

// The wave-specialised kernel for SPL sites per gatherer lane (spl / ng), NG gatherers and NB
// builders.
template <int C, int FR, int NG, int NB>
const void *mix_ws_kernel_x(int spl) {
    switch (spl) {
        case 4: return reinterpret_cast<const void *>(&lik_mixture_ws_kernel<C, 4, FR, NG, NB>);
        case 8: return reinterpret_cast<const void *>(&lik_mixture_ws_kernel<C, 8, FR, NG, NB>);
        case 16: return reinterpret_cast<const void *>(&lik_mixture_ws_kernel<C, 16, FR, NG, NB>);
        default: return reinterpret_cast<const void *>(&lik_mixture_ws_kernel<C, 32, FR, NG, NB>);
    }
}

template <int C, int FR>
const void *mix_ws_kernel_c(int spl, int ng, int nb) {
    if (nb == 2) return ng == 1 ? mix_ws_kernel_x<C, FR, 1, 2>(spl) : mix_ws_kernel_x<C, FR, 2, 2>(spl);
    return ng == 1 ? mix_ws_kernel_x<C, FR, 1, 1>(spl) : mix_ws_kernel_x<C, FR, 2, 1>(spl);
}

const void *mix_ws_kernel(int C, int fr, int spl, int ng, int nb) {
    if (C == 3) return fr == 4 ? mix_ws_kernel_c<3, 4>(spl, ng, nb) : mix_ws_kernel_c<3, 8>(spl, ng, nb);
    return mix_ws_kernel_c<2, 4>(spl, ng, nb);
}

template <int C, int FR, bool XS8, bool BK = false>
const void *mix_kernel_x(bool zoned, int spl, int zspl) {
    if (zoned) {
        switch (zspl) {
            case 4: return reinterpret_cast<const void *>(&lik_zoned_kernel<C, 4, FR, XS8>);
            case 16: return reinterpret_cast<const void *>(&lik_zoned_kernel<C, 16, FR, XS8>);
            default: return reinterpret_cast<const void *>(&lik_zoned_kernel<C, 8, FR, XS8>);
        }
    }
    switch (spl) {
        case 4: return reinterpret_cast<const void *>(&lik_mixture_kernel<C, 4, FR, XS8, BK>);
        case 8: return reinterpret_cast<const void *>(&lik_mixture_kernel<C, 8, FR, XS8, BK>);
        case 16: return reinterpret_cast<const void *>(&lik_mixture_kernel<C, 16, FR, XS8, BK>);
        default: return reinterpret_cast<const void *>(&lik_mixture_kernel<C, 32, FR, XS8, BK>);
    }
}

const void *mix_kernel(int C, int fr, bool xs8, bool zoned, int spl, int zspl, bool bk = false) {
    if (bk && !zoned) {  // banked layout: S + 1 <= 16, so observations are always x*8
        if (C == 3) return fr == 4 ? mix_kernel_x<3, 4, true, true>(false, spl, zspl)
                                   : mix_kernel_x<3, 8, true, true>(false, spl, zspl);
        return mix_kernel_x<2, 4, true, true>(false, spl, zspl);
    }
    if (C == 3) {
        if (fr == 4) return xs8 ? mix_kernel_x<3, 4, true>(zoned, spl, zspl) : mix_kernel_x<3, 4, false>(zoned, spl, zspl);
        return xs8 ? mix_kernel_x<3, 8, true>(zoned, spl, zspl) : mix_kernel_x<3, 8, false>(zoned, spl, zspl);
    }
    return xs8 ? mix_kernel_x<2, 4, true>(zoned, spl, zspl) : mix_kernel_x<2, 4, false>(zoned, spl, zspl);
}

const void *zd_kernel(int C, int zspl, int hfm) {
    if (C == 3) {
        if (zspl == 4)
            return hfm == 0 ? reinterpret_cast<const void *>(&lik_zdirect_kernel<3, 4, 0>)
                 : hfm == 1 ? reinterpret_cast<const void *>(&lik_zdirect_kernel<3, 4, 1>)
                            : reinterpret_cast<const void *>(&lik_zdirect_kernel<3, 4, 2>);
        return hfm == 0 ? reinterpret_cast<const void *>(&lik_zdirect_kernel<3, 8, 0>)
             : hfm == 1 ? reinterpret_cast<const void *>(&lik_zdirect_kernel<3, 8, 1>)
                        : reinterpret_cast<const void *>(&lik_zdirect_kernel<3, 8, 2>);
    }
    return zspl == 4 ? reinterpret_cast<const void *>(&lik_zdirect_kernel<2, 4, 0>)
                     : reinterpret_cast<const void *>(&lik_zdirect_kernel<2, 8, 0>);
}

// LDS of lik_zdirect_kernel: staged rows, 16-B pad, normalised weights
size_t zd_lds_bytes(const sbz_dims &d, int C) {
    const size_t S1 = (size_t)d.n_states + 1;
    const size_t Fam = C == 3 ? (size_t)d.n_families : 0;
    const size_t nt = (2 * ((size_t)d.n_zones + 2 + Fam) * S1 + WAVE - 1) / WAVE;
    return (2 * (size_t)ZD_FB * nt * (WAVE / 2) + (size_t)NWC * NW_PER_F) * 8;
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
    v.push_back(reinterpret_cast<const void *>(&lik_zoned_kernel<C, 4, FR, XS8>));
    v.push_back(reinterpret_cast<const void *>(&lik_zoned_kernel<C, 8, FR, XS8>));
    v.push_back(reinterpret_cast<const void *>(&lik_zoned_kernel<C, 16, FR, XS8>));
    v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 4, FR, XS8, false>));
    v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 8, FR, XS8, false>));
    v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 16, FR, XS8, false>));
    v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 32, FR, XS8, false>));
    if (XS8) {
        v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 4, FR, true, true>));
        v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 8, FR, true, true>));
        v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 16, FR, true, true>));
        v.push_back(reinterpret_cast<const void *>(&lik_mixture_kernel<C, 32, FR, true, true>));
        for (int nb = 1; nb <= 2; nb++)
            for (int ng = 1; ng <= 2; ng++)
                for (int spl = 4; spl <= 32; spl *= 2) v.push_back(mix_ws_kernel(C, FR, spl, ng, nb));
        v.push_back(reinterpret_cast<const void *>(&lik_mixture_db_kernel<C, 4, FR>));
        v.push_back(reinterpret_cast<const void *>(&lik_mixture_db_kernel<C, 8, FR>));
        v.push_back(reinterpret_cast<const void *>(&lik_mixture_db_kernel<C, 16, FR>));
        v.push_back(reinterpret_cast<const void *>(&lik_mixture_db_kernel<C, 32, FR>));
    }
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

void configure_zd(std::vector<const void *> &v) {
    for (int zspl = 4; zspl <= 8; zspl *= 2) {
        v.push_back(zd_kernel(2, zspl, 0));
        for (int hfm = 0; hfm < 3; hfm++) v.push_back(zd_kernel(3, zspl, hfm));
    }
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
const void *source_rc_kernel(int spl, bool xs8) {
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
    }
    v.push_back(reinterpret_cast<const void *>(&lik_source_kernel<C, 4>));
    v.push_back(reinterpret_cast<const void *>(&lik_source_kernel<C, 8>));
    v.push_back(reinterpret_cast<const void *>(&lik_source_kernel<C, 16>));
    v.push_back(reinterpret_cast<const void *>(&lik_source_kernel<C, 32>));
}

// How the mixture branch runs for these dims: table path with FR family registers, or the
// generic per-cell path (fr == 0).
struct MixPlan {
    int fr = 0;
    bool db = false;  // the double-buffered kernel applies (obs as x*8, table <= DB_TAB_BYTES)
    bool bk = false;  // the banked table layout applies (S + 1 <= 16, fits 64 KiB)
};

size_t mix_lds_bytes(const sbz_dims &d, int C, bool bk = false) {
    const size_t S1 = (size_t)d.n_states + 1;
    const size_t Fam = C == 3 ? (size_t)d.n_families : 0;
    if (bk)  // the lines hold the table, the neutral row and the junk slots
        return ((size_t)bk_lines(d.n_zones, (int)Fam + 1, (int)S1) * 32 + (size_t)16 * NW_PER_F) * 8;
    const size_t ncls = (size_t)(d.n_zones + 1) * (Fam + 1);
    if (SBZ_PAIR) return (1024 + WAVE + 1 + (size_t)NWC * NW_PER_F) * 8;  // (experiment: tables <= 4 KiB)
    return ((ncls + 1) * S1 + WAVE + 1 + (size_t)NWC * NW_PER_F) * 8;
}

// dynamic LDS of lik_mixture_db_kernel (the two tables are static): junk + nwt
size_t mix_db_lds_bytes() { return ((size_t)WAVE + 2 + (size_t)NWC * NW_PER_F) * 8; }
// dynamic LDS of lik_mixture_ws_kernel: junk + nwt per builder wave
size_t mix_ws_lds_bytes() { return 2 * mix_db_lds_bytes(); }

MixPlan plan_mixture(const sbz_dims &d, int C, bool xs8 = false) {
    MixPlan p;
    const int S1 = d.n_states + 1;
    const int Fam = C == 3 ? d.n_families : 0;
    if (S1 > WAVE) return p;
    const int G = WAVE / S1;
    if (d.n_zones + 1 > ZR * G) return p;
    if ((d.n_zones + 1) * (Fam + 1) + 1 > 256) return p;  // class ids are bytes
    if (mix_lds_bytes(d, C) > 64 * 1024) return p;       // row offsets are 16-bit
    if (C == 2 || Fam <= 4) p.fr = 4;
    else if (Fam <= 8) p.fr = 8;
    if (p.fr) {
        const int rpz = C == 3 ? p.fr + 1 : 1;
        const size_t tab = ((size_t)(d.n_zones + 1) * rpz + 1) * S1 * 8;
        p.db = xs8 && tab <= (size_t)DB_TAB_BYTES;
        p.bk = 2 * S1 <= 32 && mix_lds_bytes(d, C, true) <= 64 * 1024;
    }
    return p;
}

}  // namespace

bool lik_counts_apply(const sbz_dims &d) {
    const bool inh = (d.flags & SBZ_INHERITANCE) != 0;
    const int C = inh ? 3 : 2;
    const int FamC = inh ? d.n_families + 1 : 1;
    return plan_mixture(d, C).fr != 0 && FamC * (d.n_states + 1) <= CP && d.n_sites < (1 << 24);
}

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
    if (!source_mode) {
        const MixPlan p = plan_mixture(d, C);
        return p.fr ? mix_lds_bytes(d, C, p.bk) : 0;
    }
    const size_t rows = 4 + 2 * (size_t)d.n_zones + (inh ? 2 * (size_t)d.n_families : 0) + 5;
    return NW_BYTES + rows * S1 * sizeof(double) + ((rows + 7) & ~(size_t)7);  // table | zrow
}

int lik_configure(sbz_ctx *ctx) {
    std::vector<const void *> fns;
    configure_mix<2>(fns);
    configure_mix<3>(fns);
    configure_source<2>(fns);
    configure_source<3>(fns);
    configure_zd(fns);
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
    a.perm = ctx->d_perm;
    a.zone = zone;
    a.w = w;
    a.pg = pg;
    a.pz = pz;
    a.pf = pf;
    if (SBZ_LIK_STAMP) {  // diagnostic build: the phase the dense kernel reports
        const char *v = getenv("SBZ_STAMP_PHASE");
        a.F4 = v ? atoi(v) : 5;
    }

    MixPlan plan;
    bool zoned = false, ws = false, zd = false, src_rc = false;
    int block = WAVE;
    const void *mix_fn = nullptr;
    size_t lds = 0;
    int rc;
    if (!src_mode) {
        plan = plan_mixture(d, ctx->C, ctx->xs8 != 0);
        if (plan.fr) {
            zoned = ctx->d_cnt != nullptr && ctx->lik_kernel == 2;
            {
                const int Fam = ctx->C == 3 ? d.n_families : 0;
                zd = ctx->d_cnt != nullptr && ctx->d_obs8 != nullptr && ctx->lik_kernel == 5 &&
                     2 * (d.n_zones + 2 + Fam) * (d.n_states + 1) <= WAVE * ZD_NT &&
                     ctx->FamC * (d.n_states + 1) <= WAVE;
            }
            // (the <C=3, SPL=32, FR=8> instantiation of the double-buffered kernel spills)
            const bool bk = plan.bk && ctx->lik_kernel == 1 && ctx->lik_banked;
            const bool db = plan.db && !zoned && ctx->lik_kernel == 3 &&
                            !(ctx->C == 3 && plan.fr == 8 && ctx->spl == 32);
            // wave-specialised: a builder wave and ng gatherer waves of spl / ng sites per lane
            int ng = ctx->ws_ng;
            while (ng > 1 && ctx->spl / ng < 4) ng--;
            ws = plan.db && !zoned && ctx->lik_kernel == 4;
            if (zoned || zd) {
                rc = ensure(ctx, ctx->zl, (size_t)B * d.n_sites * sizeof(uint32_t));
                if (rc) return rc;
                rc = ensure(ctx, ctx->nzs, (size_t)B * sizeof(int));
                if (rc) return rc;
                zone_list_kernel<<<B, WAVE, 0, ctx->stream>>>(
                    d.n_sites, d.n_zones, ctx->FamC, zone, ctx->d_famc, ctx->d_perm,
                    static_cast<uint32_t *>(ctx->zl.ptr), static_cast<int *>(ctx->nzs.ptr));
                a.zl = static_cast<const uint32_t *>(ctx->zl.ptr);
                a.nzs = static_cast<const int *>(ctx->nzs.ptr);
                a.cnt = ctx->d_cnt;
            }
            lds = zd ? zd_lds_bytes(d, ctx->C) : ws ? mix_ws_lds_bytes() : db ? mix_db_lds_bytes()
                                                                             : mix_lds_bytes(d, ctx->C, bk);
            if (zd) {
                a.obs8 = ctx->d_obs8;
                a.F4 = ctx->F4;
                a.ones = ctx->d_ones;
                mix_fn = zd_kernel(ctx->C, ctx->zspl, ctx->C == 3 ? ctx->hfm : 0);
            } else if (ws) {
                block = WAVE * (ctx->ws_nb + ng);
                mix_fn = mix_ws_kernel(ctx->C, plan.fr, ctx->spl / ng, ng, ctx->ws_nb);
            } else {
                mix_fn = db ? mix_db_kernel(ctx->C, plan.fr, ctx->spl)
                            : mix_kernel(ctx->C, plan.fr, ctx->xs8 != 0, zoned, ctx->spl, ctx->zspl, bk);
            }
            // Long tasks: one resident round of single-wave tasks (occupancy x CUs) over the
            // launch, so every wave streams its features with no tail of late tasks.
            if (ctx->mix_occ == 0 || ctx->mix_occ_fn != mix_fn) {
                int occ = 0;
                hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, mix_fn, block, lds);
                ctx->mix_occ = (e == hipSuccess && occ > 0) ? occ : 8;
                ctx->mix_occ_fn = mix_fn;
            }
            const int per_cu = ctx->tasks_per_cu > 0 ? ctx->tasks_per_cu : ctx->mix_occ;
            const int W = std::max(1, std::min((F + 1) / 2, (ctx->n_cu * per_cu + B - 1) / B));
            a.fpw = (F + W - 1) / W;
            if (zd) {
                // dword observation groups; <= 64 features per task (the slow-path feature mask)
                a.fpw = std::min(64, (a.fpw + 3) / 4 * 4);
            }
        }
    } else {
        src_rc = ctx->src_rc && source_rc_applies(d, ctx->C) &&
                 source_rc_lds_bytes(d, ctx->C) <= 64 * 1024;
        lds = src_rc ? source_rc_lds_bytes(d, ctx->C) : lik_lds_bytes(d, true);
        if (lds > 64 * 1024)
            return fail(ctx, SBZ_EINVAL, "source-mode table needs " + std::to_string(lds) +
                                             " B of LDS per wave (> 64 KiB)");
        if (src_rc) {
            // one resident round of single-wave tasks, as the dense mixture kernel
            mix_fn = ctx->C == 3 ? source_rc_kernel<3>(ctx->spl, ctx->xs8 != 0)
                                 : source_rc_kernel<2>(ctx->spl, ctx->xs8 != 0);
            if (ctx->mix_occ == 0 || ctx->mix_occ_fn != mix_fn) {
                int occ = 0;
                hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, mix_fn, WAVE, lds);
                ctx->mix_occ = (e == hipSuccess && occ > 0) ? occ : 8;
                ctx->mix_occ_fn = mix_fn;
            }
            const int per_cu = ctx->tasks_per_cu > 0 ? ctx->tasks_per_cu : ctx->mix_occ;
            const int W = std::max(1, std::min((F + 1) / 2, (ctx->n_cu * per_cu + B - 1) / B));
            a.fpw = (F + W - 1) / W;
        }
    }
    if ((src_mode && !src_rc) || (!src_mode && !plan.fr)) {
        // one wave per (chain, feature range): enough tasks to fill 256 CUs x 32 waves
        int W = std::max(1, std::min(F, (256 * 32 + B - 1) / B));
        a.fpw = (F + W - 1) / W;
    }
    a.W = (F + a.fpw - 1) / a.fpw;

    rc = ensure(ctx, ctx->partial, (size_t)B * a.W * sizeof(double));
    if (rc) return rc;
    a.partial = static_cast<double *>(ctx->partial.ptr);
    if (ctx->ticket.bytes < (size_t)B * sizeof(unsigned) || !ctx->ticket.ptr) {
        rc = ensure(ctx, ctx->ticket, (size_t)B * sizeof(unsigned));
        if (rc) return rc;
        hipError_t e = hipMemsetAsync(ctx->ticket.ptr, 0, ctx->ticket.bytes, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipMemsetAsync(ticket)");
    }
    a.ticket = static_cast<unsigned *>(ctx->ticket.ptr);
    a.out = out_ll;
    if (src_mode) {
        if (ctx->zflag.bytes < (size_t)B * sizeof(unsigned) || !ctx->zflag.ptr) {
            rc = ensure(ctx, ctx->zflag, (size_t)B * sizeof(unsigned));
            if (rc) return rc;
            hipError_t e = hipMemsetAsync(ctx->zflag.ptr, 0, ctx->zflag.bytes, ctx->stream);
            if (e != hipSuccess) return hip_fail(ctx, e, "hipMemsetAsync(zflag)");
        }
        a.zflag = static_cast<unsigned *>(ctx->zflag.ptr);
    }

    if (src_mode) {
        const size_t bytes = (size_t)B * F * ctx->Np;
        rc = ensure(ctx, ctx->src_t, bytes);
        if (rc) return rc;
        const dim3 rgrid((ctx->Np + RP_T - 1) / RP_T, (F + RP_F - 1) / RP_F, B);
        if (src_rc)  // row codes for lik_source_rc_kernel
            repack_source_kernel<<<rgrid, 256, 0, ctx->stream>>>(
                d.n_sites, F, ctx->Np, ctx->d_perm, source, static_cast<uint8_t *>(ctx->src_t.ptr), zone,
                ctx->d_famc, d.n_zones, ctx->C == 3 ? d.n_families : 0, ctx->C);
        else
            repack_source_kernel<<<rgrid, 256, 0, ctx->stream>>>(d.n_sites, F, ctx->Np, ctx->d_perm, source,
                                                                static_cast<uint8_t *>(ctx->src_t.ptr));
        a.src_fm = static_cast<const uint8_t *>(ctx->src_t.ptr);
    }

    dim3 grid(a.W, B);
    hipStream_t st = ctx->stream;
    // A launch that never ran leaves no ticket armed, but one that failed after some tasks
    // finished would leave the chains' tickets non-zero and corrupt every later sum: re-zero them.
    auto launch_failed = [&](hipError_t e, const char *what) {
        (void)hipMemsetAsync(ctx->ticket.ptr, 0, ctx->ticket.bytes, st);
        if (ctx->zflag.ptr) (void)hipMemsetAsync(ctx->zflag.ptr, 0, ctx->zflag.bytes, st);
        return hip_fail(ctx, e, what);
    };
    ctx->last_kernels = src_rc ? "repack_source_kernel lik_source_rc_kernel"
                      : src_mode ? "repack_source_kernel lik_source_kernel"
                      : !plan.fr ? "lik_mixture_generic_kernel"
                      : zd ? "lik_zdirect_kernel" : zoned ? "zone_list_kernel lik_zoned_kernel"
                      : ws ? "lik_mixture_ws_kernel" : "lik_mixture_kernel";
    if (src_rc) {
        void *args[] = {&a};
        hipError_t e = hipLaunchKernel(mix_fn, grid, dim3(WAVE), args, lds, st);
        if (e != hipSuccess) return launch_failed(e, "source kernel launch");
    } else if (src_mode) {
        if (ctx->C == 3) launch_source<3>(ctx->spl, grid, lds, st, a);
        else launch_source<2>(ctx->spl, grid, lds, st, a);
    } else if (!plan.fr) {
        if (ctx->C == 3) lik_mixture_generic_kernel<3><<<grid, WAVE, 0, st>>>(a);
        else lik_mixture_generic_kernel<2><<<grid, WAVE, 0, st>>>(a);
    } else {
        void *args[] = {&a};
        hipError_t e = hipLaunchKernel(mix_fn, grid, dim3(block), args, lds, st);
        if (e != hipSuccess) return launch_failed(e, "mixture kernel launch");
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return launch_failed(e, "likelihood launch");
    return SBZ_OK;
}

}  // namespace sbz
