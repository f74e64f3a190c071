// sbz_mh.hip — batched Metropolis-Hastings for the sBayes zone model on CDNA4 (gfx950).
//
// One workgroup of 8 waves (two per SIMD of a CU) runs one chain for n_steps without leaving the
// kernel:
// MCMCGenerative.step (sbayes/sampling/mcmc_generative.py:282-351) with the operators of
// ZoneMCMC / ZoneMCMCWarmup (sbayes/sampling/zone_sampling.py) for SAMPLE_SOURCE = false; priors
// zero, 'counts' on p_global / p_families and 'uniform' / 'quadratic' zone size (sbz_set_priors):
//   shrink_zone :866-933 (warm-up :1498-1574)   grow_zone :788-864 (:1418-1496)
//   swap_zone :704-786 (:1328-1416)             alter_weights :408-452
//   alter_p_global :454-493   alter_p_zones :495-535   alter_p_families :571-612
//   dirichlet_proposal :537-569 (q = exp(scipy dirichlet._logpdf) then log)
//   gibbsish_sample_zones :619-702 (warm-up :1323-1326; weight 0 in the reference's own table,
//   mcmc_setup.py:77, so it runs only when a caller gives it a weight)
// Every decision is uniform: all lanes of all the waves draw the same values and take the same
// branches; the 512 threads share the per-site / per-feature work.
//
// State: the chain's zone assignment lives in LDS for the whole run (written back at the end);
// parameters stay in HBM and are updated in place on acceptance.  The log-likelihood is updated
// incrementally, ll += delta: a zone move changes the F cells of one or two sites, a parameter
// move the cells of one feature whose state is one of the two altered states (sites of the zone
// / family for p_zones / p_families; every site for weights).  Cells are computed in the
// reference's operation order (normalize_weights model.py:436-452, combine model.py:174-176).
//
// Draws: a replay tape (the reference's decisions, tests/golden/make_golden_mh.py) gives
// bit-exact trajectories; otherwise Philox4x32-10 keyed by (seed, global chain id).
#include <cmath>
#include <cstdint>
#include <string>

#include "sbz_mh_common.h"

namespace sbz {

// A/B knobs (profiles/r04_sampler_micro.txt): loads per thread and round of the planned columns
// (16 makes cfg5's one round trip, but the wider unroll costs the rest of the kernel registers:
// 5.25 vs 5.09 us per step).  A parameter move's delta takes one log of mn / mo (5.05 us per
// step against 5.25 for two library logs; two flog()s: 5.01 against 4.85 for one library log,
// profiles/r04_flog_ab.txt); SBZ_MH_DLOG picks flog or the library log for it.
#ifndef SBZ_MH_COLR
#define SBZ_MH_COLR 8
#endif
#ifndef SBZ_MH_DLOG
#define SBZ_MH_DLOG 1
#endif

namespace {

// Philox mode: step t of a launch draws its uniforms from the counter window
// [ctr0 + WIN t, ctr0 + WIN (t + 1)) (operator at slot 0, the move's draws from slot 1 on, the
// Dirichlet lane streams keyed by the slot that follows them, the acceptance uniform at slot
// WIN - 1), so every step's operator, feature, pair and Dirichlet draws are known in advance.
// The kernel computes the proposals of the parameter moves among the next LA steps at once, one
// plan per lane or lane group (gammas, lgamma / log terms and densities of all plans in parallel
// lanes of the workgroup), and
// a step whose plan is still valid (no earlier step of the batch accepted a change of the same
// parameter row) skips its proposal phase.  A plan that went stale is recomputed in place, from
// the same draws, so the trajectory does not depend on LA (tests/test_gpu_sampler.py).
constexpr int WIN = 8;
constexpr int LA = 24;  // most plans per batch (ten lgamma / log threads per plan: NT >= 10 LA)
constexpr int MAX_NWV = 8;

// The plans of one batch, shared by the workgroup's waves (written between barriers); the
// validity flags are per wave, so a wave invalidates its own copy without a barrier.
struct Plans {
    int op[LA], comp[LA], row[LA], f[LA], ia[LA], ib[LA];
    int ci0[LA], ci1[LA];  // column positions of the altered pair
    int off[LA];           // offset of the altered row in its array (w / p_global / p_zones / p_fam)
    uint32_t fm[LA];       // bit j: later plan j moves a parameter of the same feature
    int ok[MAX_NWV][LA];
    uint64_t cd[LA];  // Philox counter of the Dirichlet lane streams
    double c0[LA], c1[LA], sum[LA], t0[LA], t1[LA], a0[LA], a1[LA], n0[LA], n1[LA];
    double g[LA][2], v[LA][10];
    double nv0[LA], nv1[LA], lq[LA], lqb[LA], dprior[LA];
    double lu[LA];  // log of each step's acceptance uniform (every step of the batch)
};

// LDS layout of one chain's workgroup (byte offsets from the dynamic base), shared by the kernel
// and mh_lds_bytes.  Site scans: thread t owns KT consecutive sites c * CH + t * KT + j of chunk
// c (CH = NT * KT sites per chunk, nsc chunks); zos / nb / lst are padded to NpS = nsc * CH.
struct MhLayout {
    int KT, CH, nsc, NpS, nent, ncol;
    uint32_t col, zsize, red, nb, zos, selc, lst, wtab, wnw, tdl, gdl, fpr, rowp, ipos, plans, plcol,
        plnw, geo, gib;
    size_t total;
    __host__ __device__ MhLayout(int N, int Np, int S, int Z, int Fam, int C, int FamC, int NT,
                                 bool with_geo = false, int la = 1, bool with_gib = false, int ntab = 1) {
        KT = Np / NT;
        KT = KT < 4 ? 4 : (KT > 32 ? 32 : KT);
        CH = NT * KT;
        nsc = (Np + CH - 1) / CH;
        NpS = nsc * CH;
        nent = ((Z + 1) * FamC + 1) * (S + 1);
        ncol = (1 + Z + (C == 3 ? Fam : 0)) * S + C;
        size_t o = 0;
        auto take = [&](size_t bytes) {
            const size_t at = o;
            o = (o + bytes + 15) & ~(size_t)15;
            return (uint32_t)at;
        };
        col = take((size_t)ncol * 8);
        zsize = take((size_t)(Z + 1) * 4);
        red = take(64 * 8);              // block reductions: [2][16] doubles + [2][16] ints + misc
        nb = take((size_t)NpS * 2);
        zos = take((size_t)NpS);
        selc = take((size_t)nsc * 16 * 4);  // per chunk: selected sites per wave of the last scan
        lst = take((size_t)NpS * 2);
        // a parameter move's cell-ratio tables, per table slot (ntab, one per wave of a group) a
        // dense one (weights moves) and a sparse one (1.0 but the changed entries), its normalised
        // weights [NWV][2][4][4], the entries decomposed once (tdl), the grouped moves' deltas
        // (two slots of 8), each family class's position range [FamC][2]
        wtab = take((size_t)ntab * 2 * nent * 8);
        wnw = take((size_t)(NT / 64) * 32 * 8);
        tdl = take((size_t)nent * 4);
        gdl = take(16 * 8);
        fpr = take((size_t)FamC * 8);
        rowp = take((size_t)Np * 4);
        ipos = take((size_t)N * 2);
        // geo prior scratch (geo_zone_prior): key [N] doubles, mem [N] u16, cnt + redd / redi [16]
        plans = take(sizeof(Plans));
        // the planned steps' parameter columns [la][ncol] and normalised weights [la][2][4][4]
        plcol = take(la > 1 ? (size_t)la * ncol * 8 : 0);
        plnw = take(la > 1 ? (size_t)la * 32 * 8 : 0);
        geo = with_geo ? take(geo_scratch_bytes(N)) : o;
        // gibbsish_sample_zones: per available site its two log marginals [N] + [N] doubles and
        // its in / out flags [N] bytes
        gib = with_gib ? take((size_t)N * 17) : o;
        total = o;
    }
};

// s_barrier after the wave's LDS operations complete.  Unlike __syncthreads() this does not
// drain the vector-memory counter, so prefetched global loads stay in flight across it.
__device__ __forceinline__ void bsync() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One chain per workgroup of NWV waves (8: two per SIMD of the CU).  Every wave runs the same
// control flow: all draws and decisions are computed redundantly and identically by every wave
// (wave-uniform, from the same LDS / HBM state), and the per-site / per-feature work of a step is
// split over all NWV * 64 threads, with block reductions in a fixed order (deterministic).
// Shared state is written by thread 0 and published by a barrier.
template <int C, int NWV>
__global__ __launch_bounds__(NWV * 64) void mh_kernel(MhArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int NT = NWV * WAVE;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid >> 6;
    const int b = blockIdx.x;
    const int N = a.N, F = a.F, S = a.S, Z = a.Z, Fam = (C == 3) ? a.Fam : 0;
    const sbz_chains &ch = a.ch;

    const MhLayout L(N, a.Np, S, Z, a.Fam, C, a.FamC, NT, a.geo_cost != nullptr, a.la, a.gib != 0, a.ntab);
    const int KT = L.KT, CH = L.CH, nsc = L.nsc, ncol = L.ncol;
    double *col = reinterpret_cast<double *>(lds + L.col);  // staged parameter column
    int *zsize = reinterpret_cast<int *>(lds + L.zsize);     // [Z]
    double *redd = reinterpret_cast<double *>(lds + L.red);  // [2][16]
    int *redi = reinterpret_cast<int *>(redd + 32);           // [2][16]
    int *misc = redi + 32;                                     // [8] published scalars
    uint16_t *nb = reinterpret_cast<uint16_t *>(lds + L.nb);  // [NpS] neighbour stamps
    uint8_t *zos = lds + L.zos;                                // [NpS] zone of site (NONE = none)
    int *selc = reinterpret_cast<int *>(lds + L.selc);         // [nsc][16] per-wave counts
    uint16_t *lst = reinterpret_cast<uint16_t *>(lds + L.lst); // [NpS] compacted members
    // Parameter moves gather from two per-step tables (see delta_param): T[cls][x], cls = zone
    // class * FamC + family class, one neutral row (cls = ncls) for padding positions.
    const int S1 = S + 1, FamC = a.FamC, ncls = (Z + 1) * FamC, row_bytes = S1 * 8;
    const int nent = L.nent;
    double *wtab = reinterpret_cast<double *>(lds + L.wtab);     // [NWV][2][nent] cells old / new
    double *wnw = reinterpret_cast<double *>(lds + L.wnw);       // [NWV][2][4][4] normalised weights
    uint32_t *tdl = reinterpret_cast<uint32_t *>(lds + L.tdl);   // [nent] decomposed entries
    double *gdl = reinterpret_cast<double *>(lds + L.gdl);       // [2][8] grouped moves' deltas
    int *fpr = reinterpret_cast<int *>(lds + L.fpr);             // [FamC][2] positions of each family class
    uint32_t *rowp = reinterpret_cast<uint32_t *>(lds + L.rowp); // [Np] table row (bytes) by position
    uint16_t *ipos = reinterpret_cast<uint16_t *>(lds + L.ipos); // [N] position of each site
    double *plcol = reinterpret_cast<double *>(lds + L.plcol);  // [la][ncol] planned steps' columns
    double *plnw = reinterpret_cast<double *>(lds + L.plnw);    // [la][32] their normalised weights

    uint8_t *gzos = ch.zone_of_site + (size_t)b * N;
    double *w = ch.w + (size_t)b * F * C;
    double *pg = ch.p_global + (size_t)b * F * S;
    double *pz = Z > 0 ? ch.p_zones + (size_t)b * Z * F * S : pg;  // never read when Z == 0
    // without inheritance there is no family table: point at p_global (never read, C == 2)
    double *pf = (C == 3 && Fam > 0) ? ch.p_fam + (size_t)b * Fam * F * S : pg;
    const int max_size = ch.max_size[b];
    const double p_grow = ch.p_grow_connected[b];

    // Block reductions (fixed wave order; every thread gets the same value).  Two slots used
    // alternately: a slot is rewritten only after every wave passed the barrier of the next
    // reduction, so no wave still reads it.
    int rslot = 0;
    // a double sum and an int sum (the range-check flags) in one reduction
    auto block_sum_di = [&](double v, int iv, int &isum) -> double {
        v = wave_sum(v);
        iv = wave_sum_i(iv);
        double *r = redd + rslot * 16;
        int *ri = redi + rslot * 16;
        if (lane == 0) {
            r[wv] = v;
            ri[wv] = iv;
        }
        bsync();
        double t = r[0];
        int ti = ri[0];
#pragma unroll
        for (int i = 1; i < NWV; i++) {
            t = t + r[i];
            ti += ri[i];
        }
        rslot ^= 1;
        isum = uni(ti);
        return uni(t);
    };
    auto block_sum_i = [&](int v) -> int {
        v = wave_sum_i(v);
        int *r = redi + rslot * 16;
        if (lane == 0) r[wv] = v;
        bsync();
        int t = 0;
#pragma unroll
        for (int i = 0; i < NWV; i++) t += r[i];
        rslot ^= 1;
        return uni(t);
    };

    // load the zone assignment; sizes
    for (int z = tid; z < Z; z += NT) zsize[z] = 0;
    for (int s = tid; s < L.NpS; s += NT) nb[s] = 0;
    bsync();
    int occ = 0;
    for (int s = tid; s < L.NpS; s += NT) {
        const int z = s < N ? gzos[s] : NONE;
        zos[s] = (uint8_t)z;
        if (z < Z) {
            atomicAdd(&zsize[z], 1);
            occ++;
        }
    }
    int occupied = block_sum_i(occ);  // (its barrier publishes zos / zsize)
    // positions (family-sorted order of the likelihood context): site of each, its table row
    for (int p = tid; p < a.Np; p += NT) {
        uint32_t r = (uint32_t)(ncls * row_bytes);  // padding: the neutral row
        if (p < N) {
            const int s = a.perm[p];  // < N (built by sbz_open)
            const int z = zos[s];
            ipos[s] = (uint16_t)p;
            r = (uint32_t)((((z < Z) ? z + 1 : 0) * FamC + (C == 3 ? (int)a.famc[p] : 0)) * row_bytes);
        }
        rowp[p] = r;
    }
    bsync();

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
    double prior = ch.prior ? ch.prior[b] : 0.0;  // carried log prior (sbz_set_priors)
    // 'cost_based' geo prior: only the last zone counts (model.py:1110-1139); its current value
    double *geo_key = reinterpret_cast<double *>(lds + L.geo);
    uint16_t *geo_mem = reinterpret_cast<uint16_t *>(geo_key + N);
    int *geo_cnt = reinterpret_cast<int *>(geo_mem + ((N + 7) & ~7));
    double *geo_rd = reinterpret_cast<double *>(geo_cnt + 4);
    int *geo_ri = reinterpret_cast<int *>(geo_rd + 16);
    auto geo_prior = [&](int add, int rm1, int rm2) -> double {
        return geo_zone_prior<NWV>(a.geo_cost, a.geo_scale, N, zos, Z - 1, add, rm1, rm2, geo_key,
                                   geo_mem, geo_cnt, geo_rd, geo_ri);
    };
    double geo_cur = (a.geo_cost && Z > 0) ? geo_prior(-1, -1, -1) : 0.0;
    int err = 0;             // first range-check failure of this thread (MH_IDX)
    long long err_val = 0;
    const long long nFS = (long long)F * S, nZFS = (long long)Z * F * S, nFamFS = (long long)Fam * F * S;
    uint16_t stamp = 0;

    auto is_nb = [&](int s) { return nb[s] == stamp && zos[s] == NONE; };
    // site selections: SEL_NB (neighbours of the marked zone, free), SEL_FREE, SEL_ZONE (members of
    // z), SEL_AVAIL (free or in z: gibbsish_sample_zones' available sites, zone_sampling.py:627)
    enum { SEL_NB = 0, SEL_FREE = 1, SEL_ZONE = 2, SEL_AVAIL = 3 };
    // Scan: every thread builds the bit mask of its selected sites (bit j = site base + j, KT <= 32
    // sites read with a few wide LDS reads) of chunk c; per-wave counts go to selc.
    auto scan_mask = [&](int mode, int z, int c) -> uint32_t {
        const int s0 = c * CH + tid * KT;
        uint32_t m = 0;
#pragma unroll
        for (int g = 0; g < 8; g++) {
            if (4 * g >= KT) break;  // uniform
            const uint32_t zw = *reinterpret_cast<const uint32_t *>(zos + s0 + 4 * g);
            const uint2 nw2 = *reinterpret_cast<const uint2 *>(nb + s0 + 4 * g);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t zs = (zw >> (8 * j)) & 0xffu;
                const uint32_t ns = ((j < 2 ? nw2.x : nw2.y) >> (16 * (j & 1))) & 0xffffu;
                const bool f = mode == SEL_NB     ? (ns == stamp && zs == NONE)
                               : mode == SEL_FREE ? zs == NONE
                               : mode == SEL_ZONE ? zs == (uint32_t)z
                                                  : (zs == NONE || zs == (uint32_t)z);
                m |= (f ? 1u : 0u) << (4 * g + j);
            }
        }
        // padding sites (>= N) hold zone NONE and a stale stamp: never selected
        const int nv = min(max(N - s0, 0), KT);
        return m & (nv >= 32 ? 0xffffffffu : ((1u << nv) - 1u));
    };
    // exclusive prefix of n over the block's threads (thread order) from the per-wave totals in
    // cnt[0..NWV); incl = the inclusive prefix within the wave
    auto wave_incl = [&](int n) -> int { return wave_incl_scan(n); };
    uint32_t msk[4];  // this thread's masks of the last scan (chunks 0..3; more chunks rescan)
    int scan_mode = 0, scan_z = 0;
    // number of selected sites; leaves per-wave counts in selc and the masks in msk
    auto scan_sel = [&](int mode, int z) -> int {
        scan_mode = mode;
        scan_z = z;
        for (int c = 0; c < nsc; c++) {
            const uint32_t m = scan_mask(mode, z, c);
            if (c < 4) msk[c & 3] = m;
            const int wt = uni((int)__builtin_amdgcn_readlane((uint32_t)wave_incl(__popc(m)), 63));
            if (lane == 0) selc[c * 16 + wv] = wt;
        }
        bsync();
        // every wave sums the per-wave counts of every chunk
        int all = 0;
        for (int c = 0; c < nsc; c++)
#pragma unroll
            for (int i = 0; i < NWV; i++) all += selc[c * 16 + i];
        return uni(all);
    };
    // The k-th selected site of the last scan in ascending order (-1 if none).
    auto kth_scan = [&](int k) -> int {
        for (int c = 0; c < nsc; c++) {
            int tot = 0, woff = 0;
#pragma unroll
            for (int i = 0; i < NWV; i++) {
                const int t = selc[c * 16 + i];
                woff += i < wv ? t : 0;
                tot += t;
            }
            tot = uni(tot);
            if (k < tot) {
                const uint32_t m = c < 4 ? msk[c & 3] : scan_mask(scan_mode, scan_z, c);
                const int n = __popc(m);
                const int incl = woff + wave_incl(n);
                const int excl = incl - n;
                int site = -1;
                if (excl <= k && k < incl) {  // exactly one thread
                    uint32_t mm = m;
                    for (int r = k - excl; r > 0; r--) mm &= mm - 1;
                    site = c * CH + tid * KT + (int)__builtin_ctz(mm);
                    misc[0] = site;
                }
                bsync();
                site = uni(misc[0]);
                bsync();  // misc[0] may be rewritten by the next call
                return site;
            }
            k -= tot;
        }
        return -1;
    };
    // the selected sites of (mode, z) compacted into lst[0 .. n) in ascending order; returns n
    auto compact_sel = [&](int mode, int z) -> int {
        const int nsel = scan_sel(mode, z);
        int base = 0;
        for (int c = 0; c < nsc; c++) {
            uint32_t m = c < 4 ? msk[c & 3] : scan_mask(mode, z, c);
            int woff = 0, tot = 0;
#pragma unroll
            for (int i = 0; i < NWV; i++) {
                const int t = selc[c * 16 + i];
                woff += i < wv ? t : 0;
                tot += t;
            }
            const int n = __popc(m);
            int o = base + woff + wave_incl(n) - n;
            while (m) {
                lst[o++] = (uint16_t)(c * CH + tid * KT + (int)__builtin_ctz(m));
                m &= m - 1;
            }
            base += uni(tot);
        }
        bsync();
        return nsel;
    };
    // mark nb[t] = stamp for every site t adjacent to a member of zone z: every thread marks the
    // neighbours of the members among its own sites (a zone's members rarely share a thread's KT
    // sites, so the adjacency loads of all members are in flight at once; marking is idempotent,
    // so no compaction of the members and no barrier before the marks)
    auto mark = [&](int z) {
        stamp++;
        if (stamp == 0) {  // wrapped: clear
            for (int s = tid; s < L.NpS; s += NT) nb[s] = 0;
            bsync();
            stamp = 1;
        }
        for (int c = 0; c < nsc; c++) {
            uint32_t m = scan_mask(SEL_ZONE, z, c);
            while (m) {
                const int s = c * CH + tid * KT + (int)__builtin_ctz(m);
                m &= m - 1;
                const int e0 = a.adj_ptr[s], e1 = a.adj_ptr[s + 1];
                for (int e = e0; e < e1; e += 8) {
                    int t[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) t[k] = a.adj_idx[MH_IDX(min(e + k, e1 - 1), a.nnz, 1)];
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        if (e + k < e1) nb[MH_IDX(t[k], N, 2)] = stamp;
                }
            }
        }
        bsync();
    };

    // delta log-likelihood of moving site s from zone zo to zone zn (NONE = no zone): features
    // split over the block's threads
    auto delta_site = [&](int s, int zo, int zn) {
        const int fc = (C == 3) ? a.fam_site[MH_IDX(s, N, 3)] : 0;
        const bool hf = fc > 0;
        double mn = 1.0, mo = 1.0;
        int en = 0, eo = 0;
        for (int f = tid; f < F; f += NT) {
            const int x = a.obs_sm[MH_IDX((long long)s * F + f, (long long)N * F, 4)];
            const bool na = x == S;
            const int xc = na ? 0 : x;
            // every load is unconditional with an always-valid index (component rows clamped to
            // row 0 when the site lacks the component); the select below discards the value
            const double *wp = w + MH_IDX((long long)f * C, (long long)F * C, 5);
            const double wf[3] = {ldp(wp), ldp(wp + 1), C == 3 ? ldp(wp + C - 1) : 0.0};
            const double l0 = ldp(pg + MH_IDX((long long)f * S + xc, nFS, 6));
            const double l2v = ldp(pf + MH_IDX(((long long)(hf ? fc - 1 : 0) * F + f) * S + xc, C == 3 && Fam > 0 ? nFamFS : nFS, 7));
            const double lzov = ldp(pz + MH_IDX(((long long)(zo < Z ? zo : 0) * F + f) * S + xc, Z > 0 ? nZFS : 1, 8));
            const double lznv = ldp(pz + MH_IDX(((long long)(zn < Z ? zn : 0) * F + f) * S + xc, Z > 0 ? nZFS : 1, 8));
            const double l2 = hf ? l2v : 0.0;
            const double lzo = zo < Z ? lzov : 0.0;
            const double lzn = zn < Z ? lznv : 0.0;
            mo *= cell<C>(wf, zo < Z, hf, na, l0, lzo, l2);
            mn *= cell<C>(wf, zn < Z, hf, na, l0, lzn, l2);
            renorm(mo, eo);
            renorm(mn, en);
        }
        return (flog(mn) - flog(mo)) + (double)(en - eo) * LN2;  // this thread's part (block_sum)
    };

    // gibbsish_sample_zones (zone_sampling.py:644-665): site s's log marginal likelihood with
    // zone z (lw) and without any zone (lwo), sum_f log feature_lh, over the wave's lanes (one
    // wave per site; every lane of the wave gets both)
    auto site_logs = [&](int s, int z, double &lw, double &lwo) {
        const int fc = (C == 3) ? a.fam_site[MH_IDX(s, N, 3)] : 0;
        const bool hf = fc > 0;
        double mw = 1.0, mo = 1.0;
        int ew = 0, eo = 0;
        for (int f = lane; f < F; f += WAVE) {
            const int x = a.obs_sm[MH_IDX((long long)s * F + f, (long long)N * F, 4)];
            const bool na = x == S;
            const int xc = na ? 0 : x;
            const double *wp = w + MH_IDX((long long)f * C, (long long)F * C, 5);
            const double wf[3] = {ldp(wp), ldp(wp + 1), C == 3 ? ldp(wp + C - 1) : 0.0};
            const double l0 = ldp(pg + MH_IDX((long long)f * S + xc, nFS, 6));
            const double l2v = ldp(pf + MH_IDX(((long long)(hf ? fc - 1 : 0) * F + f) * S + xc, C == 3 && Fam > 0 ? nFamFS : nFS, 7));
            const double lz = ldp(pz + MH_IDX(((long long)z * F + f) * S + xc, Z > 0 ? nZFS : 1, 8));
            const double l2 = hf ? l2v : 0.0;
            mw *= cell<C>(wf, true, hf, na, l0, lz, l2);
            mo *= cell<C>(wf, false, hf, na, l0, 0.0, l2);
            renorm(mw, ew);
            renorm(mo, eo);
        }
        lw = wave_sum(flog(mw) + (double)ew * LN2);
        lwo = wave_sum(flog(mo) + (double)eo * LN2);
    };
    double *gib_lw = reinterpret_cast<double *>(lds + L.gib);  // [N] per available site
    double *gib_lwo = gib_lw + N;                               // [N]
    uint8_t *gib_fl = reinterpret_cast<uint8_t *>(gib_lwo + N); // [N] bit 0 new, bit 1 old membership

    // Feature f's parameter column pg | pz[z] | pf[fam] | w: loaded into registers early
    // (col_load, issued before the proposal math so the loads are in flight meanwhile) and
    // written to LDS later (col_store); columns longer than NCV * NT load the rest synchronously.
    constexpr int NCV = 1;
    auto col_src = [&](int f, int i) -> const double * {
        // one unconditional load from a pointer chosen per element (always a valid index)
        const int seg = i / S, r = i - seg * S;
        if (i >= (1 + Z + Fam) * S) return w + MH_IDX((long long)f * C + (i - (1 + Z + Fam) * S), (long long)F * C, 9);
        if (seg == 0) return pg + MH_IDX((long long)f * S + r, nFS, 9);
        if (seg <= Z) return pz + MH_IDX(((long long)(seg - 1) * F + f) * S + r, nZFS, 9);
        return pf + MH_IDX(((long long)(seg - 1 - Z) * F + f) * S + r, nFamFS, 9);
    };
    auto col_load = [&](int f, double (&cv)[NCV]) {
#pragma unroll
        for (int k = 0; k < NCV; k++) cv[k] = ldp(col_src(f, min(tid + NT * k, ncol - 1)));
    };
    auto col_store = [&](int f, const double (&cv)[NCV]) {
#pragma unroll
        for (int k = 0; k < NCV; k++)
            if (tid + NT * k < ncol) col[tid + NT * k] = cv[k];
        for (int i = tid + NT * NCV; i < ncol; i += NT) col[i] = ldp(col_src(f, i));
        bsync();
    };
    // normalize_weights (model.py:436-452) of class h (bit 0: has a zone, bit 1: has a family) for
    // feature weights wc, after the move when nu (weights move: entries ia / ib become va / vb);
    // one division per weight, as the reference
    auto norm_w = [&](const double *wc, int comp, int ia, int ib, double va, double vb, int h, int nu,
                      double *o4) {
        double wv3[3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const double wo = (C == 3 || i < 2) ? wc[i] : 0.0;
            wv3[i] = (nu && comp == 3 && i == ia) ? va : ((nu && comp == 3 && i == ib) ? vb : wo);
        }
        const double w0 = wv3[0] * 1.0, w1 = wv3[1] * ((h & 1) ? 1.0 : 0.0);
        double sum = w0 + w1, w2 = 0.0;
        if (C == 3) {
            w2 = wv3[2] * ((h & 2) ? 1.0 : 0.0);
            sum = sum + w2;
        }
        o4[0] = w0 / sum;
        o4[1] = w1 / sum;
        o4[2] = C == 3 ? w2 / sum : 0.0;
    };
    // table entry e = cls * S1 + x as x | zone class << 8 | family class << 16 | (cls < ncls) << 24
    auto tdecomp = [&](int e) -> uint32_t {
        const int cls = e / S1, x = e - cls * S1;
        const bool real = cls < ncls;
        const int zcl = real ? cls / FamC : 0, fc = real ? cls - (cls / FamC) * FamC : 0;
        return (uint32_t)x | ((uint32_t)zcl << 8) | ((uint32_t)fc << 16) | ((real ? 1u : 0u) << 24);
    };
    for (int e = tid; e < nent; e += NT) tdl[e] = tdecomp(e);
    for (int e = tid; e < a.ntab * nent; e += NT) wtab[(e / nent) * 2 * nent + nent + e % nent] = 1.0;  // sparse
    for (int c = tid; c < 2 * FamC; c += NT) fpr[c] = 0;
    bsync();
    // family class c occupies positions [fpr[2c], fpr[2c + 1]) (sites sorted by class, sbz_open)
    for (int p = tid; p < N; p += NT) {
        const int c = C == 3 ? (int)a.famc[p] : 0;
        if (p == 0 || (C == 3 && (int)a.famc[p - 1] != c)) fpr[2 * c] = p;
        if (p == N - 1 || (C == 3 && (int)a.famc[p + 1] != c)) fpr[2 * c + 1] = p + 1;
    }
    bsync();
    // Delta of a parameter move, computed by ONE wave (the calling wave; every lane of it gets the
    // value).  Parameter moves on different features change disjoint cells, so up to ntab planned
    // moves of a batch get their deltas at once, one per wave (the step loop's grouped path), and
    // an unplanned move is computed the same way by wave 0: the value of a move's delta does not
    // depend on how the steps were grouped or planned.  `cl` is feature f's column in LDS (the
    // staged col, or a planned step's column) and `nwp` its normalised weights before
    // (nwp[0..15]) and after (nwp[16..31]) the move, or null: computed here into the wave's wnw.
    // A cell's value depends only on (zone class, family class, x), so the wave writes one table
    // for feature f in its own LDS slot — new cell / old cell for every (class, x) whose value the
    // move changes (the reference's cells, model.py:436-452, 174-176), 1.0 for every other entry —
    // and each position multiplies the entry of its class row (rowp) and observation byte.  The
    // changed entries are exactly the cells the reference recomputes: every cell for the weights
    // (the slot's dense table, rewritten whole), states ia / ib of the component's rows otherwise
    // (the slot's sparse table, 1.0 everywhere else: only the 2 x rows changed entries are written,
    // and reset to 1.0 after the gathers).  A p_families move reads only its family's position
    // range (families are contiguous in the position order); every other position there, and of
    // the other moves, reads its entry, 1.0 where the move changes nothing.
#ifdef SBZ_MH_STAMP
    double stamp_dp = 0.0;  // phase cycles of the last delta_param (SBZ_MH_STAMP 4 / 5 / 6)
#endif
    constexpr int OBW = 8;  // observation words (chunks of 256 positions) in flight per lane
    const int nch = a.Np / 256;
    const uint32_t *obs32 = reinterpret_cast<const uint32_t *>(a.obs_fm);
    auto delta_param = [&](const double *cl, const double *nwp, int f, int comp, int row, int ia, int ib,
                           double va, double vb) -> double {
#ifdef SBZ_MH_STAMP
        const long long dt_start = clock64();
#endif
        const int wvu = uni(wv);
        const bool dense = comp == 3;
        double *tab = wtab + (size_t)wvu * 2 * nent + (dense ? 0 : nent);
        // positions the move's entries can apply to: [p_lo, p_hi) (a family's range for p_families)
        int p_lo = 0, p_hi = a.Np;
        if (comp == 2) {
            p_lo = uni(fpr[2 * (row + 1)]);
            p_hi = uni(fpr[2 * (row + 1) + 1]);
        }
        const int k_lo = p_lo / 256, k_hi = p_hi > p_lo ? (p_hi + 255) / 256 : k_lo;  // chunks
        // the feature's observation words, all in flight during the table build
        const size_t fo = (size_t)MH_IDX(f, F, 13) * (size_t)(a.Np / 4);
        uint32_t o[OBW];
#pragma unroll
        for (int i = 0; i < OBW; i++) o[i] = obs32[fo + (size_t)min(k_lo + i, nch - 1) * WAVE + lane];
        if (!nwp) {
            double *own = wnw + wvu * 32;
            if (lane < 8) norm_w(cl + (1 + Z + Fam) * S, comp, ia, ib, va, vb, lane & 3, lane >> 2, own + lane * 4);
            wsync();
            nwp = own;
        }
        // the changed entries: dense, every entry e; sparse, entry i of the move's list (state ia /
        // ib of every class row (p_global), of the zone's rows (p_zones), of the family's rows
        // (p_families)); lane takes i = lane + 64 u, two at a time with the LDS reads of both in
        // flight (unconditional, valid indices; selects discard)
        const int n_chg = dense ? nent : (comp == 0 ? 2 * ncls : (comp == 1 ? 2 * FamC : 2 * (Z + 1)));
        auto entry_of = [&](int i) -> int {
            if (dense) return i;
            const int x = (i & 1) ? ib : ia, j = i >> 1;
            const int cls = comp == 0 ? j : (comp == 1 ? (row + 1) * FamC + j : j * FamC + row + 1);
            return cls * S1 + x;
        };
        int wide = 0;
        for (int i0 = lane; i0 < n_chg; i0 += 2 * WAVE) {
            double rt[2];
            int es[2];
            uint32_t dcs[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                es[u] = entry_of(min(i0 + u * WAVE, n_chg - 1));
                dcs[u] = tdl[es[u]];
            }
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t dc = dcs[u];
                const int x = (int)(dc & 0xffu), zcl = (int)((dc >> 8) & 0xffu), fc = (int)((dc >> 16) & 0xffu);
                const bool real = (dc >> 24) != 0;
                const bool na = x == S, hz = zcl > 0, hf = fc > 0;
                const int xc = na ? 0 : x, h = (hz ? 1 : 0) | (hf ? 2 : 0);
                const double l0 = cl[xc];
                const double l1v = cl[zcl * S + xc], l2v = cl[(Z + fc) * S + xc];
                const double l1 = hz ? l1v : 0.0;
                const double l2 = hf ? l2v : 0.0;
                const bool pick = !na && (x == ia || x == ib);
                const bool changed = real && (comp == 3 || (pick && (comp == 0 || (comp == 1 && zcl == row + 1) ||
                                                                     (comp == 2 && fc == row + 1))));
                const double nv = x == ia ? va : vb;
                const double n0 = comp == 0 && pick ? nv : l0;
                const double n1 = comp == 1 && pick ? nv : l1;
                const double n2 = comp == 2 && pick ? nv : l2;
                const double *wo = nwp + h * 4, *wn = nwp + 16 + h * 4;
                const double wold[3] = {wo[0], wo[1], wo[2]}, wnew[3] = {wn[0], wn[1], wn[2]};
                const double vo = cell_nw<C>(wold, hz, hf, na, l0, l1, l2);
                const double vn = cell_nw<C>(wnew, hz, hf, na, n0, n1, n2);
                rt[u] = changed ? vn / vo : 1.0;
                wide |= !(rt[u] >= 0x1p-120 && rt[u] <= 0x1p120) ? 1 : 0;  // (NaN: wide)
            }
#pragma unroll
            for (int u = 0; u < 2; u++)
                if (i0 + u * WAVE < n_chg) tab[es[u]] = rt[u];
        }
        const bool wid = __ballot(wide != 0) != 0;
        wsync();  // the wave's table writes are visible to its gathers
#ifdef SBZ_MH_STAMP
        const long long dt_tb = clock64();
#endif
        // gathers: position p = 256 k + 4 lane + j of chunk k, two chunks (8 positions per lane)
        // at a time, all 8 table reads issued together.  A sparse move's table holds 1.0 wherever
        // the move changes nothing, so every position of its chunk range reads its entry as a dense
        // move does: the product is the same as reading only the changed entries (round 6: no
        // branch per position, 2.97 -> 2.89 us per step of the cfg5 default mix,
        // profiles/r06_mh_sparse_ab.txt).  Safe factors (within 2^+-120): the 8 multiply as a
        // tree, one renormalisation per pair of chunks; otherwise renormalise after every factor.
        double m = 1.0;
        int e = 0;
        const unsigned char *tb = reinterpret_cast<const unsigned char *>(tab);
        const uint32_t xsh = a.xs8 ? 0u : 3u;
        for (int b0 = k_lo; b0 < k_hi; b0 += OBW) {
            if (b0 > k_lo) {
#pragma unroll
                for (int i = 0; i < OBW; i++) o[i] = obs32[fo + (size_t)min(b0 + i, nch - 1) * WAVE + lane];
            }
#pragma unroll
            for (int j = 0; j < OBW; j += 2) {
                const int i0 = b0 + j;
                if (i0 >= k_hi) break;  // uniform
                const bool two = i0 + 1 < k_hi;
                const uint4 ra = *reinterpret_cast<const uint4 *>(rowp + i0 * 256 + 4 * lane);
                const uint4 rb = *reinterpret_cast<const uint4 *>(rowp + (two ? i0 + 1 : i0) * 256 + 4 * lane);
                const uint32_t oa = o[j], ob = o[j + 1];
                const uint32_t r8[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
                double v[8];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const uint32_t xb = ((q < 4 ? oa : ob) >> (8 * (q & 3))) & 0xffu;
                    v[q] = *reinterpret_cast<const double *>(tb + r8[q] + (xb << xsh));
                }
                if (!two) {
#pragma unroll
                    for (int q = 4; q < 8; q++) v[q] = 1.0;
                }
                if (wid) {
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        m *= v[q];
                        renorm(m, e);
                    }
                } else {
                    m *= ((v[0] * v[1]) * (v[2] * v[3])) * ((v[4] * v[5]) * (v[6] * v[7]));
                    renorm(m, e);
                }
            }
        }
        if (!dense) {  // reset the sparse table's entries (this wave's reads of them come first)
            for (int i = lane; i < n_chg; i += WAVE) tab[entry_of(i)] = 1.0;
        }
#ifdef SBZ_MH_STAMP
        const long long dt_ga = clock64();
        const double res = wave_sum(flog_e(m, e));
        const long long dt_lg = clock64();
        if (SBZ_MH_STAMP == 4) stamp_dp = (double)(dt_tb - dt_start);
        if (SBZ_MH_STAMP == 5) stamp_dp = (double)(dt_ga - dt_tb);
        if (SBZ_MH_STAMP == 6) stamp_dp = (double)(dt_lg - dt_ga);
        return res;
#else
        return wave_sum(flog_e(m, e));  // m in [0.5, 1) (1.0 if no pair), 0, or not finite
#endif
    };

    // One MH step per iteration, in four phases with one call site each (keeps the kernel small):
    //   1. draw the operator and its move (zone moves: sites and Hastings terms; parameter moves:
    //      the feature, component and pair of entries);  2. Dirichlet proposal (parameter moves);
    //   3. delta log-likelihood;  4. accept / reject and apply.
    bool broken = false;  // a tape decision with no matching candidate (replay mismatch)
    const bool philox = rng.tape == nullptr;
    const uint64_t ctr0 = rng.ctr;  // Philox: window of step t = ctr0 + WIN t
    // plans (Philox): the steps plan_t0 .. plan_t0 + LAe - 1
    static_assert(NWV <= MAX_NWV && NT >= 10 * LA, "plan stage D needs ten threads per plan");
    const int LAe = min(a.la, LA);
    int plan_t0 = -(1 << 30);
    Plans *pl = reinterpret_cast<Plans *>(lds + L.plans);
    int *okw = pl->ok[wv];  // this wave's validity flags
    // The plans of steps t0 .. t0 + LAe - 1, in thread-parallel stages with the results in LDS:
    // (A) thread k evaluates step t0 + k's draws from its window (the operator, then the same
    // draws in the same order as the sequential code below); (COL) every thread gathers part of
    // the planned features' parameter columns into plcol (all loads in flight at once); (A2) the
    // altered pair read from the column; (B) the two gammas of plan k on threads k and 32 + k, the
    // acceptance uniforms on wave 1; (C) the Dirichlet pair; (D) the ten lgamma / log terms of plan
    // k on threads 10 k .. 10 k + 9 (all waves); (E) the two densities (exp, then log, as
    // util.dirichlet_pdf) on threads k and 32 + k, the 'counts' prior change, and the normalised
    // weights before / after each move on waves 1-3.  A later accepted move patches the columns of
    // the plans it affects (step loop, phase 4), so a step never reloads its column.
    auto make_plans = [&](int t0) {
        bsync();  // every wave is done with the previous batch
        const uint32_t k0 = rng.key0, k1 = rng.key1;
        const uint64_t chain = rng.chain;
        const int la = LAe;
        // precision of component comp (0 global, 1 zone, 2 family, 3 weights) by selects: a
        // lane-varying index into the kernel arguments would copy them to scratch
        const double pr_w = a.prec[0], pr_g = a.prec[1], pr_z = a.prec[2], pr_f = a.prec[3];
        auto prec_of = [&](int comp) {
            const double x = comp == 3 ? pr_w : pr_g;
            const double y = comp == 1 ? pr_z : pr_f;
            return (comp == 3 || comp == 0) ? x : y;
        };
        if (tid < la) {  // (A)
            const int k = tid;
            uint64_t c = ctr0 + (uint64_t)(t0 + k) * WIN;
            int op = -1, comp = -1, row = 0, f = 0, ia = 0, ib = 0;
            if (t0 + k < a.n_steps) {
                const double u = philox_uniform(k0, k1, chain, c++);  // Rng::op
                int n_le = 0;
#pragma unroll
                for (int q = 0; q < SBZ_N_OPS - 1; q++) n_le += (q < a.nops - 1 && !(u < a.op_cdf[q])) ? 1 : 0;
                op = n_le;
                auto below = [&](int n) { return min((int)(philox_uniform(k0, k1, chain, c++) * (double)n), n - 1); };
                if (op >= WEIGHTS && op <= P_FAMILIES && !(op == P_FAMILIES && (C == 2 || Fam == 0)) &&
                    !(op == P_ZONES && Z == 0)) {
                    if (op == WEIGHTS) {
                        f = below(F);
                        comp = 3;
                        if (C == 3) {
                            ia = below(3);
                            ib = below(2);
                            if (ib >= ia) ib++;
                        } else {
                            ia = 0;
                            ib = 1;
                        }
                    } else {
                        if (op == P_ZONES) row = below(Z);
                        if (op == P_FAMILIES) row = below(Fam);
                        f = below(F);
                        const int n = a.app_cnt[f];
                        const int i0 = below(n);
                        int j0 = below(n - 1);
                        if (j0 >= i0) j0++;
                        ia = a.app_list[(size_t)f * S + i0];
                        ib = a.app_list[(size_t)f * S + max(j0, 0)];  // (n < 2: invalid below)
                        comp = op == P_GLOBAL ? 0 : (op == P_ZONES ? 1 : 2);
                    }
                }
            }
            // the sequential path's checks of the move (an invalid one is left to it: it stops
            // the chain with the same status)
            const int lim = comp == 3 ? C : S;
            const bool valid = comp >= 0 && f >= 0 && f < F && ia >= 0 && ib >= 0 && ia != ib && ia < lim &&
                               ib < lim && row >= 0 && !(comp == 1 && row >= Z) && !(comp == 2 && row >= Fam);
            pl->op[k] = op;
            pl->comp[k] = comp;
            pl->row[k] = row;
            pl->f[k] = f;
            pl->ia[k] = ia;
            pl->ib[k] = ib;
            pl->off[k] = comp == 3 ? f * C : (row * F + f) * S;
#pragma unroll
            for (int w = 0; w < NWV; w++) pl->ok[w][k] = valid ? 1 : 0;
            pl->cd[k] = c;
            const int cb = comp == 3 ? (1 + Z + Fam) * S : (comp == 0 ? 0 : (comp == 1 ? (1 + row) * S : (1 + Z + row) * S));
            pl->ci0[k] = cb + ia;
            pl->ci1[k] = cb + ib;
            // later plans of the same feature (compared through the lanes of wave 0)
            uint32_t fmask = 0;
            for (int j = 1; j < la; j++) {
                const int fj = __builtin_amdgcn_readlane(f, j), cj = __builtin_amdgcn_readlane(comp, j);
                fmask |= (j > k && comp >= 0 && cj >= 0 && fj == f) ? (1u << j) : 0u;
            }
            pl->fm[k] = fmask;
        }
        bsync();
        {  // (COL) element e = k * ncol + i: unconditional loads with valid indices, then the stores
            const int tot = la * ncol;
            constexpr int RC = SBZ_MH_COLR;
            for (int e0 = 0; e0 < tot; e0 += RC * NT) {
                double v[RC];
#pragma unroll
                for (int j = 0; j < RC; j++) {
                    const int e = min(e0 + j * NT + tid, tot - 1);
                    const int k = e / ncol;
                    v[j] = ldp(col_src(pl->f[k], e - k * ncol));
                }
#pragma unroll
                for (int j = 0; j < RC; j++)
                    if (e0 + j * NT + tid < tot) plcol[e0 + j * NT + tid] = v[j];
            }
        }
        bsync();
        if (tid < la && pl->comp[tid] >= 0) {  // (A2)
            const int k = tid, comp = pl->comp[k];
            const double c0 = plcol[k * ncol + pl->ci0[k]], c1 = plcol[k * ncol + pl->ci1[k]];
            const double pr = prec_of(comp);
            const bool raw = C == 2 && comp == 3;  // the weight pair as is (zone_sampling.py:440-443)
            const double sum = raw ? 1.0 : c0 + c1;
            const double t0d = raw ? c0 : c0 / sum, t1d = raw ? c1 : c1 / sum;
            pl->c0[k] = c0;
            pl->c1[k] = c1;
            pl->sum[k] = sum;
            pl->t0[k] = t0d;
            pl->t1[k] = t1d;
            pl->a0[k] = 1.0 + pr * t0d;
            pl->a1[k] = 1.0 + pr * t1d;
        }
        wsync();
        {  // (B)
            const int kk = tid & 31, g = tid >> 5;
            if (tid < 64 && kk < la && pl->comp[kk] >= 0) {
                LaneRng lr;
                lr.initk(k0, k1, chain, pl->cd[kk], g);
                pl->g[kk][g] = lr.gamma(g ? pl->a1[kk] : pl->a0[kk]);
            }
            // wave 1: the acceptance uniforms (slot WIN - 1 of each window), as rng.real() draws them
            if (tid >= 64 && tid < 64 + la) {
                const int k = tid - 64;
                pl->lu[k] = log(philox_uniform(k0, k1, chain, ctr0 + (uint64_t)(t0 + k) * WIN + (WIN - 1)));
            }
        }
        wsync();
        if (tid < la && pl->comp[tid] >= 0) {  // (C)
            const int k = tid;
            const double g0 = pl->g[k][0], g1 = pl->g[k][1];
            const double sg = g0 + g1;
            const double n0 = g0 / sg, n1 = g1 / sg;
            const bool raw = C == 2 && pl->comp[k] == 3;
            pl->n0[k] = n0;
            pl->n1[k] = n1;
            pl->nv0[k] = raw ? n0 : n0 * pl->sum[k];
            pl->nv1[k] = raw ? n1 : n1 * pl->sum[k];
        }
        bsync();
        {  // (D) dirichlet_proposal2's terms {a0, a1, a0 + a1, b0, b1, b0 + b1, n0, n1, w0, w1}
            const int k = tid / 10, q = tid - 10 * k;
            if (k < la && pl->comp[k] >= 0) {
                const double pr = prec_of(pl->comp[k]);
                const double a0 = pl->a0[k], a1 = pl->a1[k];
                const double b0 = 1.0 + pr * pl->n0[k], b1 = 1.0 + pr * pl->n1[k];
                double arg = q == 0 ? a0 : q == 1 ? a1 : q == 2 ? a0 + a1 : q == 3 ? b0 : q == 4 ? b1
                           : q == 5 ? b0 + b1 : q == 6 ? pl->n0[k] : q == 7 ? pl->n1[k] : q == 8 ? pl->t0[k] : pl->t1[k];
                pl->v[k][q] = q < 6 ? lgamma(arg) : log(arg);
            }
        }
        bsync();
        {  // (E) -(sum gammaln(a) - gammaln(sum a)) + sum xlogy(a - 1, x); q = exp, log q
            const int kk = tid & 31, g = tid >> 5;
            if (tid < 64 && kk < la && pl->comp[kk] >= 0) {
                const double *v = pl->v[kk];
                const int comp = pl->comp[kk];
                const double pr = prec_of(comp);
                const double x0 = g ? 1.0 + pr * pl->n0[kk] : pl->a0[kk];  // the density's alphas
                const double x1 = g ? 1.0 + pr * pl->n1[kk] : pl->a1[kk];
                const double t0 = (x0 - 1.0) == 0.0 ? 0.0 : (x0 - 1.0) * v[g ? 8 : 6];
                const double t1 = (x1 - 1.0) == 0.0 ? 0.0 : (x1 - 1.0) * v[g ? 9 : 7];
                const double lp = -((v[g ? 3 : 0] + v[g ? 4 : 1]) - v[g ? 5 : 2]) + (t0 + t1);
                const double l = log(exp(lp));
                if (g) pl->lqb[kk] = l;
                else pl->lq[kk] = l;
                if (!g) {
                    double dp = 0.0;
                    if ((comp == 0 && a.alpha_g) || (C == 3 && comp == 2 && a.alpha_f)) {
                        const double *al = comp == 0 ? a.alpha_g : a.alpha_f;
                        const long long off = ((long long)pl->row[kk] * F + pl->f[kk]) * S;
                        const double al0 = al[off + pl->ia[kk]] - 1.0, al1 = al[off + pl->ib[kk]] - 1.0;
                        dp = (xlogy(al0, pl->nv0[kk]) - xlogy(al0, pl->c0[kk])) +
                             (xlogy(al1, pl->nv1[kk]) - xlogy(al1, pl->c1[kk]));
                    }
                    pl->dprior[kk] = dp;
                }
            }
            // waves 1-3: thread 64 + 8 k + 4 nu + h, the normalised weights of plan k (class h,
            // before / after the move)
            if (tid >= 64 && tid < 64 + 8 * la) {
                const int q = tid - 64, k = q >> 3;
                const int comp = pl->comp[k];
                if (comp >= 0)
                    norm_w(plcol + k * ncol + (1 + Z + Fam) * S, comp, pl->ia[k], pl->ib[k], pl->nv0[k],
                           pl->nv1[k], q & 3, (q >> 2) & 1, plnw + k * 32 + (q & 7) * 4);
            }
        }
        bsync();
        plan_t0 = t0;
    };

    // An accepted parameter move's store (thread 0) is not waited for at once: the next load of
    // parameters (or the column store of a prefetched step) first waits for it and publishes it
    // with a barrier (fence_params), by which time it has long completed.
    bool store_pending = false;
    auto fence_params = [&]() {
        if (store_pending) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bsync();
            store_pending = false;
        }
    };
    // per-operator counts: lane op counts operator op's proposals / acceptances (every wave alike)
    int cnt_prop = 0, cnt_acc = 0;
    // An accepted parameter move on feature f: later plans of the batch on this feature (`later`:
    // the plan's mask, made when planned; ~0 for a step that was not planned) take the new values
    // in their columns (wave 0 writes, a barrier publishes them); a plan whose proposal read the
    // altered row (same component and row), or whose weights changed, is stale and recomputed when
    // reached.
    auto patch_later = [&](int pk_, uint32_t later, int comp_, int row_, int f_, int ia_, int ib_, double nv0_,
                           double nv1_) {
        if (later == 0) return;
        const int k = min(lane, LA - 1);
        const bool in = lane < LAe && lane > pk_ && ((later >> k) & 1u) && pl->comp[k] >= 0 && pl->f[k] == f_;
        const int cb = comp_ == 3 ? (1 + Z + Fam) * S : (comp_ == 0 ? 0 : (comp_ == 1 ? (1 + row_) * S : (1 + Z + row_) * S));
        if (wv == 0 && in) {
            plcol[k * ncol + cb + ia_] = nv0_;
            plcol[k * ncol + cb + ib_] = nv1_;
        }
        if (in && (comp_ == 3 || (pl->comp[k] == comp_ && pl->row[k] == row_))) okw[k] = 0;
        if (__ballot(in) != 0) bsync();  // the same ballot in every wave
    };
#ifdef SBZ_MH_STAMP
    // diagnostic builds (tools/build_mh_variant.sh NAME -DSBZ_MH_STAMP=K): the trace's ll column
    // holds shader-clock cycles per step instead (K = 1: the whole step, make_plans included;
    // 2: the grouped path's delta phase; 3: make_plans; a group's cycles are split evenly over its
    // members; 4 / 5 / 6: wave 0's delta_param table build / gathers / log + sum, not split; 7 / 8 /
    // 9: a step of the sequential path (zone moves, unplanned moves): its move draw / proposal and
    // delta / MH test and apply);
    // tools/mh_optime.py --stamps reads them
    long long stamp_t0 = 0, stamp_plan = 0, stamp_d0 = 0, stamp_d1 = 0, stamp_p1 = 0, stamp_p3 = 0;
    double stamp_val = 0.0;
#endif
    auto trace_step = [&](int st, int op_, bool acc) {
        if (ch.trace_op && tid == 0) {
            const size_t t = (size_t)b * a.n_steps + st;
            ch.trace_op[t] = (int8_t)op_;
            ch.trace_accept[t] = acc ? 1 : 0;
#ifdef SBZ_MH_STAMP
            ch.trace_ll[t] = stamp_val;
#else
            ch.trace_ll[t] = ll;
#endif
        }
        if (ch.trace_zos) {
            uint8_t *tz = ch.trace_zos + ((size_t)b * a.n_steps + st) * N;
            for (int s = tid; s < N; s += NT) tz[s] = zos[s];
        }
    };
    int gsl = 0;  // gdl slot of the next group
    for (int step = 0; step < a.n_steps; step++) {
        if (rng.bad || broken) break;
#ifdef SBZ_MH_STAMP
        stamp_t0 = clock64();
        stamp_plan = 0;
#endif
        if (philox) rng.ctr = ctr0 + (uint64_t)step * WIN;
        if (philox && LAe > 1 && step >= plan_t0 + LAe) {
            fence_params();
            make_plans(step);
#ifdef SBZ_MH_STAMP
            stamp_plan = clock64() - stamp_t0;
#endif
        }
        const int pk = step - plan_t0;  // this step's plan (Philox, LAe > 1)
        // the plan's fields, read in one batch (one LDS round trip)
        int p_ok = 0, p_op = 0, p_comp = -1;
        double p_lu = 0.0;
        int nx_ok[MAX_NWV], nx_comp[MAX_NWV];
        uint32_t nx_fm[MAX_NWV];
        if (philox && LAe > 1) {
            p_ok = okw[pk];
            p_op = pl->op[pk];
            p_comp = pl->comp[pk];
            p_lu = pl->lu[pk];
#pragma unroll
            for (int k = 0; k < NWV; k++) {
                const int q = min(pk + k, LA - 1);
                nx_ok[k] = okw[q];
                nx_comp[k] = pl->comp[q];
                nx_fm[k] = pl->fm[q];
            }
        }
        const bool planned = philox && LAe > 1 && uni(p_ok) != 0;
        if (planned && uni(p_comp) >= 0) {
            // ---- grouped planned parameter moves: this step and the next planned, valid parameter
            // moves of the batch whose features differ pairwise (at most NWV).  Each changes only
            // its own feature's cells, so their deltas do not depend on each other's outcome: wave k
            // computes member k's delta, then every wave takes the members' decisions in step order
            // (the trajectory is the one-step-at-a-time trajectory: test_gpu_sampler.py)
            int g = 1;
            uint32_t fmacc = (uint32_t)uni((int)nx_fm[0]);
#pragma unroll
            for (int k = 1; k < NWV; k++) {
                const int q = pk + k;
                const bool more = g == k && k < a.ntab && step + k < a.n_steps && q < LAe && uni(nx_ok[k]) != 0 &&
                                  uni(nx_comp[k]) >= 0 && !((fmacc >> q) & 1u);
                if (more) {
                    fmacc |= (uint32_t)uni((int)nx_fm[k]);
                    g++;
                }
            }
            double *gslot = gdl + gsl * 8;
            gsl ^= 1;  // a slot is rewritten only after every wave passed the next group's barrier
#ifdef SBZ_MH_STAMP
            stamp_d0 = clock64();
#endif
            const int wvu = uni(wv);
            if (wvu < g) {
                const int q = pk + wvu;
                const double d = delta_param(plcol + q * ncol, plnw + q * 32, uni(pl->f[q]), uni(pl->comp[q]),
                                             uni(pl->row[q]), uni(pl->ia[q]), uni(pl->ib[q]), uni(pl->nv0[q]),
                                             uni(pl->nv1[q]));
                if (lane == 0) gslot[wvu] = d;
            }
            bsync();
#ifdef SBZ_MH_STAMP
            stamp_d1 = clock64();
#endif
            for (int k = 0; k < g; k++) {
                const int q = pk + k;
                const int op_k = uni(pl->op[q]), comp_k = uni(pl->comp[q]), row_k = uni(pl->row[q]);
                const int f_k = uni(pl->f[q]), ia_k = uni(pl->ia[q]), ib_k = uni(pl->ib[q]), off_k = uni(pl->off[q]);
                const uint32_t fm_k = (uint32_t)uni((int)pl->fm[q]);
                const double nv0_k = uni(pl->nv0[q]), nv1_k = uni(pl->nv1[q]), lq_k = uni(pl->lq[q]);
                const double lqb_k = uni(pl->lqb[q]), dp_k = uni(pl->dprior[q]), lu_k = uni(pl->lu[q]);
                const double delta_k = uni(gslot[k]);
                // metropolis_hastings_ratio (mcmc_generative.py:331-351), as the sequential path
                bool acc;
                if (lqb_k == -INFINITY) acc = false;
                else if (lq_k == -INFINITY) acc = true;
                else acc = lu_k < (delta_k * 1.0) - (lq_k - lqb_k) + dp_k;
                cnt_prop += lane == op_k ? 1 : 0;
                if (acc) {
                    cnt_acc += lane == op_k ? 1 : 0;
                    ll = ll + delta_k;
                    prior = prior + dp_k;
                    double *bs = (comp_k == 3 ? w : (comp_k == 0 ? pg : (comp_k == 1 ? pz : pf))) + off_k;
                    if (tid == 0) {
                        stp(bs + ia_k, nv0_k);
                        stp(bs + ib_k, nv1_k);
                    }
                    store_pending = true;
                    patch_later(q, fm_k, comp_k, row_k, f_k, ia_k, ib_k, nv0_k, nv1_k);
                }
#ifdef SBZ_MH_STAMP
                {
                    const long long now = clock64();
                    stamp_val = SBZ_MH_STAMP == 1 ? (double)(now - stamp_t0) / g
                              : SBZ_MH_STAMP == 2 ? (double)(stamp_d1 - stamp_d0) / g
                              : SBZ_MH_STAMP == 3 ? (double)stamp_plan / g : uni(stamp_dp);
                }
#endif
                trace_step(step + k, op_k, acc);
            }
            step += g - 1;
            continue;
        }
        const int op = planned ? uni(p_op) : rng.op(a.op_cdf, a.nops);
        if (op < 0 || op > GIBBSISH || (op == P_FAMILIES && (C == 2 || Fam == 0)) ||
            ((op <= SWAP || op == GIBBSISH) && Z == 0) || (op == P_ZONES && Z == 0)) {
            broken = true;
            break;
        }
        double log_q = 0.0, log_q_back = -INFINITY;
        double dprior = 0.0;  // prior_new - prior_prev of the proposal
        // zone move: site sa goes zoa -> zna, site sb (swap) zob -> znb
        int sa = -1, zoa = NONE, zna = NONE, sb = -1;
        // parameter move
        int comp = -1, row = 0, f = 0, ia = 0, ib = 0;
        long long poff = 0;  // offset of the altered row (parameters and prior concentrations)
        double prec = 0.0;
        double *base = nullptr;
        const int n_free = N - occupied;
        // gibbsish_sample_zones: zone gz, its gn available sites in lst, the proposed size, the
        // change of the occupied count and the move's delta ll; gtent: zos holds the proposal
        bool gib = false, gtent = false;
        int gz = 0, gn = 0, gsize = 0, gdocc = 0;
        double gdelta = 0.0;

        // ---- 1. the move
        if (op <= SWAP) {
            const int z = rng.below(Z);
            if (z < 0 || z >= Z) {
                broken = true;
                break;
            }
            const int size = uni(zsize[z]);
            if (op == GROW || op == SWAP) {
                if (op == SWAP || size < max_size) {
                    mark(z);
                    const bool connected = rng.real() < p_grow;
                    const int n_nb = scan_sel(SEL_NB, 0);
                    const int cnt = connected ? n_nb : n_free;
                    if (cnt > 0) {
                        if (!connected) scan_sel(SEL_FREE, 0);
                        const int site = kth_scan(rng.below(cnt));
                        int site_rm = -2;
                        if (op == SWAP) {
                            scan_sel(SEL_ZONE, z);
                            site_rm = kth_scan(rng.below(size));
                        }
                        if (site < 0 || site_rm == -1) {
                            broken = true;
                            break;
                        }
                        double q = (1.0 - p_grow) * (1.0 / (double)n_free);
                        if (is_nb(site)) q += p_grow * (1.0 / (double)n_nb);
                        double q_back;
                        if (op == GROW) {
                            q_back = 1.0 / (double)(size + 1);
                        } else {
                            // back_neighbours = get_neighbours(zone_current, occupied): same set
                            q_back = (1.0 - p_grow) * (1.0 / (double)n_free);
                            if (is_nb(site_rm)) q_back += p_grow * (1.0 / (double)n_nb);
                            sb = site_rm;
                        }
                        log_q = uni(log(q));
                        log_q_back = uni(log(q_back));
                        if (op == GROW) dprior = uni(size_prior_delta(a.size_prior, N, size, size + 1));
                        sa = site;
                        zoa = NONE;
                        zna = z;
                    }
                }
            } else if (size > a.min_size) {  // SHRINK
                scan_sel(SEL_ZONE, z);
                const int site = kth_scan(rng.below(size));
                if (site < 0) {
                    broken = true;
                    break;
                }
                // back step: grow of the shrunk zone (neighbours of the zone without the site)
                if (tid == 0) zos[site] = NONE;
                bsync();
                mark(z);
                const int n_back = scan_sel(SEL_NB, 0);
                double q_back = (1.0 - p_grow) * (1.0 / (double)(n_free + 1));
                if (is_nb(site)) q_back += p_grow * (1.0 / (double)n_back);
                if (a.warmup) q_back = 1.0 / (double)(size + 1);  // zone_sampling.py:1561
                bsync();  // every wave read zos[site] (is_nb) before it is restored
                if (tid == 0) zos[site] = (uint8_t)z;
                bsync();
                log_q = uni(log(1.0 / (double)size));
                log_q_back = uni(log(q_back));
                dprior = uni(size_prior_delta(a.size_prior, N, size, size - 1));
                sa = site;
                zoa = z;
                zna = NONE;
            }
        } else if (op == GIBBSISH) {
            // zone_sampling.py:619-702: zone z's available sites (free or in z; a random subset of
            // about 100 when more), each resampled in / out of z with the posterior
            // exp(lw) / (exp(lw) + exp(lwo)) of its marginal likelihoods; uniforms from the tape
            // in site order (np.random.random(n)) or the per-site Philox streams of slots 2 / 3
            const int z = rng.below(Z);
            if (z < 0 || z >= Z) {
                broken = true;
                break;
            }
            gib = true;
            gz = z;
            fence_params();  // the marginals below read parameters: a pending accepted store first
            const uint64_t slot = ctr0 + (uint64_t)step * WIN;
            auto site_u = [&](int64_t p0, int k, int sl) {
                return rng.tape ? rng.tape[p0 + k] : site_uniform(rng.key0, rng.key1, rng.chain, slot + sl, (uint32_t)k);
            };
            auto take_tape = [&](int n) -> int64_t {  // the next n tape items (wave-uniform)
                const int64_t p0 = rng.pos;
                if (rng.tape) {
                    if (p0 + n > rng.len) rng.bad = 1;
                    rng.pos = uni64(min(p0 + n, rng.len));
                }
                return p0;
            };
            const int size = uni(zsize[z]);
            int n = compact_sel(SEL_AVAIL, z);
            if (n > 100) {  // available[available] &= np.random.random(n) < (100 / n)   (:631-633)
                const double thr = 100.0 / (double)n;
                const int64_t p0 = take_tape(n);
                if (rng.bad) break;
                int kept = 0;
                for (int r0 = 0; r0 < n; r0 += NT) {  // order-preserving compaction in place
                    const int i = r0 + tid;
                    int st = 0;
                    bool keep = false;
                    if (i < n) {
                        st = lst[i];
                        keep = site_u(p0, i, 2) < thr;
                    }
                    const uint64_t bal = __ballot(keep);
                    if (lane == 0) selc[wv] = (int)__popcll(bal);
                    bsync();
                    int woff = 0, tot = 0;
#pragma unroll
                    for (int q = 0; q < NWV; q++) {
                        const int t = selc[q];
                        woff += q < wv ? t : 0;
                        tot += t;
                    }
                    if (keep) lst[kept + woff + (int)__popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)st;
                    kept += uni(tot);
                    bsync();
                }
                n = kept;
            }
            gn = n;
            if (n > 0) {
                for (int k = wv; k < n; k += NWV) {
                    double lw, lwo;
                    site_logs(lst[k], z, lw, lwo);
                    if (lane == 0) {
                        gib_lw[k] = lw;
                        gib_lwo[k] = lwo;
                    }
                }
                bsync();
                const int64_t p1 = take_tape(n);  // new_zone = np.random.random(n) < posterior_zone
                if (rng.bad) break;
                double lq = 0.0, lqb = 0.0, d = 0.0;
                int n_new = 0, n_old = 0, n_zero = 0;
                for (int k = tid; k < n; k += NT) {
                    const double lw = gib_lw[k], lwo = gib_lwo[k];
                    const double mw = exp(lw), mo = exp(lwo);
                    const double post = mw / (mw + mo);
                    const bool nz = site_u(p1, k, 3) < post;
                    const bool oz = zos[lst[k]] == (uint8_t)z;
                    const double fn = nz ? 1.0 : 0.0, fo = oz ? 1.0 : 0.0;
                    const double q = post * fn + (1.0 - post) * (1.0 - fn);
                    const double qb = post * fo + (1.0 - post) * (1.0 - fo);
                    lq += log(q);
                    lqb += log(qb);
                    n_zero += qb == 0.0 ? 1 : 0;
                    n_new += nz ? 1 : 0;
                    n_old += oz ? 1 : 0;
                    if (nz != oz) d += nz ? lw - lwo : lwo - lw;
                    gib_fl[k] = (uint8_t)((nz ? 1 : 0) | (oz ? 2 : 0));
                }
                int nn = 0, no = 0, nzb = 0;
                const double LQ = block_sum_di(lq, n_new, nn);
                const double LQB = block_sum_di(lqb, n_old, no);
                gdelta = block_sum_di(d, n_zero + (err != 0 ? 0x10000 : 0), nzb);
                if (nzb >= 0x10000) {  // a range check failed
                    broken = true;
                    break;
                }
                gsize = size - no + nn;
                gdocc = nn - no;
                // reject: a size outside [min_size, max_size] (:678-681), or a zero back probability
                if (a.min_size <= gsize && gsize <= max_size && nzb == 0) {
                    log_q = LQ;
                    log_q_back = LQB;
                    if (a.size_prior == 1) {  // -log C(N, size) per zone: one site at a time
                        double dp = 0.0;
                        for (int sz = size; sz != gsize; sz += gsize > sz ? 1 : -1)
                            dp += size_prior_delta(1, N, sz, sz + (gsize > sz ? 1 : -1));
                        dprior = uni(dp);
                    } else {
                        dprior = uni(size_prior_delta(a.size_prior, N, size, gsize));
                    }
                    if (a.geo_cost && z == Z - 1) {  // the last zone's MST on the proposed zone
                        for (int k = tid; k < n; k += NT)
                            zos[lst[k]] = (gib_fl[k] & 1) ? (uint8_t)z : (uint8_t)NONE;
                        bsync();
                        gtent = true;
                    }
                }
            }
        } else {
            if (op == WEIGHTS) {
                f = rng.below(F);
                comp = 3;
                if (C == 3) rng.pair(nullptr, 3, ia, ib);
                else {
                    ia = 0;
                    ib = 1;
                }
            } else {
                if (op == P_ZONES) row = rng.below(Z);
                if (op == P_FAMILIES) row = rng.below(Fam);
                f = rng.below(F);
                const size_t fi = MH_IDX(f, F, 14);
                rng.pair(a.app_list + fi * S, a.app_cnt[fi], ia, ib);
                comp = op == P_GLOBAL ? 0 : (op == P_ZONES ? 1 : 2);
            }
            if (f < 0 || f >= F || ia < 0 || ib < 0 || ia == ib || ia >= (comp == 3 ? C : S) ||
                ib >= (comp == 3 ? C : S) || row < 0 || (comp == 1 && row >= Z) ||
                (comp == 2 && row >= Fam)) {
                broken = true;
                break;
            }
            double *arr = comp == 3 ? w : (comp == 0 ? pg : (comp == 1 ? pz : pf));
            const long long lim = comp == 3 ? (long long)F * C : (comp == 0 ? nFS : (comp == 1 ? nZFS : nFamFS));
            const long long off = comp == 3 ? (long long)f * C : ((long long)row * F + f) * S;
            prec = a.prec[comp == 3 ? 0 : comp + 1];
            // uniform indices: every thread of every wave takes the same branch
            if (!(off + ia >= 0 && off + ia < lim && off + ib >= 0 && off + ib < lim)) {
                MH_IDX(off + ia, lim, 15);
                MH_IDX(off + ib, lim, 15);
                broken = true;
                break;
            }
            base = arr + off;
            poff = off;
        }

#ifdef SBZ_MH_STAMP
        stamp_p1 = clock64();
#endif
        // ---- 2. Dirichlet proposal of the pair (zone_sampling.py:421-438, :537-569)
        fence_params();  // (planned parameter moves took the grouped path above)
        double nv0 = 0.0, nv1 = 0.0;
        double cv[NCV];
        if (comp >= 0) {
            const double c0 = uni(ldp(base + ia)), c1 = uni(ldp(base + ib));
            // the move's column: in flight during the proposal math
            col_load(f, cv);
            // without inheritance the weight pair is used as is (zone_sampling.py:440-443)
            const bool raw = C == 2 && comp == 3;
            const double sum = raw ? 1.0 : c0 + c1;
            const double t0 = raw ? c0 : c0 / sum, t1 = raw ? c1 : c1 / sum;
            double u0 = t0, u1 = t1;
            dirichlet_proposal2(rng, t0, t1, prec, u0, u1, log_q, log_q_back);
            nv0 = raw ? u0 : u0 * sum;
            nv1 = raw ? u1 : u1 * sum;
            // 'counts' priors: dirichlet_logpdf(p[f, states], alpha) changes only in the two
            // altered states' xlogy(alpha - 1, p) terms (prior_p_global_dirichlet
            // model.py:1142-1170, prior_p_families_dirichlet :1173-1219)
            if ((comp == 0 && a.alpha_g) || (C == 3 && comp == 2 && a.alpha_f)) {
                // the concentrations sit at the same offset as the altered pair (off + ia / ib)
                const double *al = comp == 0 ? a.alpha_g : a.alpha_f;
                const double a0 = uni(al[poff + ia]) - 1.0;
                const double a1 = uni(al[poff + ib]) - 1.0;
                dprior = uni((xlogy(a0, nv0) - xlogy(a0, c0)) + (xlogy(a1, nv1) - xlogy(a1, c1)));
            }
        }

        // ---- 3. delta log-likelihood (one block reduction; it also makes a range-check failure
        // of any thread known to every wave)
        double delta = 0.0;
        if (sa >= 0 || comp >= 0) {
            double part = 0.0;
            if (sa >= 0) {
                part = delta_site(sa, zoa, zna);
                if (sb >= 0) part = part + delta_site(sb, zna, NONE);
            } else if (comp >= 0) {
                // the column staged here; wave 0 computes the delta as a grouped move's wave would,
                // and the block sum below adds zeros to it (exact)
                col_store(f, cv);
                if (uni(wv) == 0) {
                    const double d = delta_param(col, nullptr, f, comp, row, ia, ib, nv0, nv1);
                    part = lane == 0 ? d : 0.0;
                }
            }
            int n_err = 0;
            delta = block_sum_di(part, err != 0 ? 1 : 0, n_err);
            if (n_err != 0) {  // a range check failed: stop before using the move
                broken = true;
                break;
            }
        }

        if (gib) delta = gdelta;
        // the geo prior of the last zone, when the move changes it
        double geo_new = geo_cur;
        if (gtent) {
            geo_new = geo_prior(-1, -1, -1);
            dprior = uni(dprior + (geo_new - geo_cur));
        }
        if (a.geo_cost && sa >= 0 && (zna == Z - 1 || zoa == Z - 1)) {
            geo_new = geo_prior(zna == Z - 1 ? sa : -1, zoa == Z - 1 ? sa : -1,
                                (sb >= 0 && zna == Z - 1) ? sb : -1);
            dprior = uni(dprior + (geo_new - geo_cur));
        }

#ifdef SBZ_MH_STAMP
        stamp_p3 = clock64();
#endif
        // ---- 4. metropolis_hastings_ratio (mcmc_generative.py:331-351, uniform priors)
        bool accept = false;
        if (log_q_back == -INFINITY) {
            accept = false;
        } else if (log_q == -INFINITY) {
            accept = true;
        } else {
            const double mh = (delta * 1.0) - (log_q - log_q_back) + dprior;
            if (philox && LAe > 1) {
                accept = uni(p_lu) < mh;
            } else {
                if (philox) rng.ctr = ctr0 + (uint64_t)step * WIN + (WIN - 1);
                accept = log(rng.real()) < mh;
            }
        }
        cnt_prop += lane == op ? 1 : 0;
        if (accept) {
            cnt_acc += lane == op ? 1 : 0;
            ll = ll + delta;
            prior = prior + dprior;
            geo_cur = geo_new;
            if (gib) {
                for (int k = tid; k < gn; k += NT) {
                    const int st = lst[k];
                    const bool nz = gib_fl[k] & 1;
                    const int fcs = C == 3 ? (int)a.fam_site[st] : 0;
                    zos[st] = nz ? (uint8_t)gz : (uint8_t)NONE;
                    rowp[ipos[st]] = (uint32_t)(((nz ? gz + 1 : 0) * FamC + fcs) * row_bytes);
                }
                if (tid == 0) zsize[gz] = gsize;
                occupied += gdocc;
                bsync();
            } else if (sa >= 0) {
                if (tid == 0) {
                    const int fca = C == 3 ? (int)a.fam_site[sa] : 0;
                    rowp[ipos[sa]] = (uint32_t)(((zna < Z ? zna + 1 : 0) * FamC + fca) * row_bytes);
                    if (sb >= 0) rowp[ipos[sb]] = (uint32_t)((C == 3 ? (int)a.fam_site[sb] : 0) * row_bytes);
                    zos[sa] = (uint8_t)zna;
                    if (zoa < Z) zsize[zoa]--;
                    if (zna < Z) zsize[zna]++;
                    if (sb >= 0) {
                        zos[sb] = NONE;
                        zsize[zna]--;
                    }
                }
                occupied += (zna < Z ? 1 : -1) + (sb >= 0 ? -1 : 0);
                bsync();
            } else {
                if (tid == 0) {
                    stp(base + ia, nv0);
                    stp(base + ib, nv1);
                }
                store_pending = true;
                // (a step that was not planned compares every later plan)
                patch_later(pk, !philox || LAe <= 1 ? 0u : ~0u, comp, row, f, ia, ib, nv0, nv1);
            }
        }
        if (gtent && !accept) {  // restore the assignment the proposal overwrote
            for (int k = tid; k < gn; k += NT)
                zos[lst[k]] = (gib_fl[k] & 2) ? (uint8_t)gz : (uint8_t)NONE;
            bsync();
        }
#ifdef SBZ_MH_STAMP
        {
            const long long now = clock64();
            stamp_val = SBZ_MH_STAMP == 1 ? (double)(now - stamp_t0)
                      : SBZ_MH_STAMP == 3 ? (double)stamp_plan
                      : SBZ_MH_STAMP == 7 ? (double)(stamp_p1 - stamp_t0)
                      : SBZ_MH_STAMP == 8 ? (double)(stamp_p3 - stamp_p1)
                      : SBZ_MH_STAMP == 9 ? (double)(now - stamp_p3) : 0.0;
        }
#endif
        trace_step(step, op, accept);
    }

    bsync();
    for (int s = tid; s < N; s += NT) gzos[s] = zos[s];
    if (tid == 0) {
        ch.ll[b] = ll;
        if (ch.prior) ch.prior[b] = prior;
        if (ch.tape_pos) ch.tape_pos[b] = rng.pos;
        if (ch.counter) ch.counter[b] = philox ? ctr0 + (uint64_t)a.n_steps * WIN : rng.ctr;
        if (ch.status) ch.status[b] = broken ? 2 : (rng.bad ? 1 : 0);
    }
    if (tid < SBZ_N_OPS) {  // per-operator counters, one thread each
        if (ch.accepted) ch.accepted[(size_t)b * SBZ_N_OPS + tid] += cnt_acc;
        if (ch.proposed) ch.proposed[(size_t)b * SBZ_N_OPS + tid] += cnt_prop;
    }
    // the first range-check failure (lowest thread): status 16 + code
    {
        const uint64_t bad = __ballot(err != 0);
        if (lane == 0) redi[wv] = bad ? __shfl(err, (int)__builtin_ctzll(bad), 64) : 0;
        bsync();
        if (tid == 0) {
            int code = 0;
            for (int i = 0; i < NWV && !code; i++) code = redi[i];
            if (code && ch.status) ch.status[b] = 16 + code;
        }
    }
}

// Waves per chain (one workgroup per chain): 8 since round 6, two per SIMD at <= 256 registers
// per lane (2 spilled); with move groups of 8 the cfg5 default mix runs 2.99 us per step against
// 3.23 for 4 waves with groups of 4 (tools/ab_mh_waves_r06.sh, profiles/r06_mh_ab.txt).  A/B builds:
// tools/build_mh_variant.sh NAME -DSBZ_MH_WAVES=4.
#ifndef SBZ_MH_WAVES
#define SBZ_MH_WAVES 8
#endif
constexpr int MH_WAVES = SBZ_MH_WAVES;  // waves per chain (one workgroup per chain)

}  // namespace

size_t mh_lds_bytes(const sbz_dims &d, int C, bool geo, bool gib) {
    const int FamC = C == 3 ? d.n_families + 1 : 1;
    return MhLayout(d.n_sites, np_of(d.n_sites), d.n_states, d.n_zones, d.n_families, C, FamC,
                    MH_WAVES * WAVE, geo, 1, gib).total;
}

namespace {
// sbz_draw_gamma: draw i from LaneRng stream (key = seed, chain = i / 64, lane i % 64, counter 0)
__global__ __launch_bounds__(256) void draw_gamma_kernel(int n, const double *alpha, uint64_t seed, double *out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    LaneRng lr;
    lr.initk((uint32_t)seed, (uint32_t)(seed >> 32), (uint64_t)(i / 64), 0, i % 64);
    out[i] = lr.gamma(alpha[i]);
}
}  // namespace

int launch_draw_gamma(sbz_ctx *ctx, int n, const double *alpha, uint64_t seed, double *out) {
    draw_gamma_kernel<<<(n + 255) / 256, 256, 0, ctx->stream>>>(n, alpha, seed, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "draw_gamma_kernel launch");
}

int launch_mh(sbz_ctx *ctx, int B, int n_steps, const sbz_mh_config *cfg, const sbz_chains *chains) {
    const sbz_dims &d = ctx->d;
    if (!ctx->d_adj_ptr) return fail(ctx, SBZ_ESTATE, "sbz_set_network must be called before sbz_mh_run_device");
    if (B <= 0 || n_steps <= 0) return SBZ_OK;
    // Philox blocks carry the global chain id in one 32-bit word (LaneRng, sbz_mh_common.h)
    if (chains->chain_id0 > 0xffffffffull - (uint64_t)B)
        return fail(ctx, SBZ_EINVAL, "global chain ids must stay below 2^32");
    const bool src = cfg->sample_source != 0;
    MhArgs a{};
    a.N = d.n_sites;
    a.F = d.n_features;
    a.S = d.n_states;
    a.Z = d.n_zones;
    a.Fam = d.n_families;
    a.C = ctx->C;
    a.FamC = ctx->FamC;
    a.Np = ctx->Np;
    a.xs8 = ctx->xs8;
    a.n_steps = n_steps;
    a.min_size = cfg->min_size;
    a.warmup = cfg->warmup;
    // operators of the mode: zone moves + alter_* (mixture) or + Gibbs operators (source mode)
    bool allowed[SBZ_N_OPS] = {};
    allowed[SHRINK] = allowed[GROW] = allowed[SWAP] = allowed[GIBBSISH] = true;
    if (src) {
        for (int i = G_SOURCES; i <= G_P_FAMILIES; i++) allowed[i] = true;
    } else {
        for (int i = WEIGHTS; i <= P_FAMILIES; i++) allowed[i] = true;
    }
    double tot = 0.0;
    int last = -1;
    for (int i = 0; i < SBZ_N_OPS; i++) {
        const double p = cfg->op_prob[i];
        if (p < 0.0 || std::isnan(p)) return fail(ctx, SBZ_EINVAL, "negative operator probability");
        if (p > 0.0 && !allowed[i])
            return fail(ctx, SBZ_EINVAL, std::string("operator ") + std::to_string(i) +
                                             " is not available in this mode (sample_source)");
        if (p > 0.0) last = i;
        tot += p;
    }
    if (!(tot > 0.0)) return fail(ctx, SBZ_EINVAL, "operator probabilities sum to 0");
    const double zone_ops = cfg->op_prob[SHRINK] + cfg->op_prob[GROW] + cfg->op_prob[SWAP] +
                            cfg->op_prob[GIBBSISH] + cfg->op_prob[P_ZONES] + cfg->op_prob[G_P_ZONES];
    if (d.n_zones == 0 && zone_ops > 0) return fail(ctx, SBZ_EINVAL, "zone operators need n_zones > 0");
    if ((ctx->C == 2 || d.n_families == 0) && (cfg->op_prob[P_FAMILIES] + cfg->op_prob[G_P_FAMILIES]) > 0)
        return fail(ctx, SBZ_EINVAL, "family operators need inheritance with families");
    double acc = 0.0;
    a.nops = last + 1;
    for (int i = 0; i < a.nops; i++) {
        acc += cfg->op_prob[i] / tot;
        a.op_cdf[i] = acc;
    }
    a.op_cdf[a.nops - 1] = 1.0;
    for (int i = 0; i < 4; i++) a.prec[i] = cfg->precision[i];
    a.gib = cfg->op_prob[GIBBSISH] > 0.0 ? 1 : 0;
    a.obs_fm = ctx->d_obs_fm;
    a.famc = ctx->d_famc;
    a.perm = ctx->d_perm;
    a.obs_sm = ctx->d_obs_sm;
    a.fam_site = ctx->d_fam_site;
    a.adj_ptr = ctx->d_adj_ptr;
    a.adj_idx = ctx->d_adj_idx;
    a.nnz = ctx->adj_nnz;
    a.app_list = ctx->d_app_list;
    a.app_cnt = ctx->d_app_cnt;
    a.alpha_g = ctx->d_alpha_g;
    a.alpha_f = ctx->C == 3 ? ctx->d_alpha_f : nullptr;
    a.size_prior = ctx->size_prior;
    a.gc_g = ctx->d_gc_g;
    a.gc_f = ctx->C == 3 ? ctx->d_gc_f : nullptr;
    a.geo_cost = d.n_zones > 0 ? ctx->d_geo_cost : nullptr;
    a.geo_scale = ctx->geo_scale;
    a.ch = *chains;
    if (!a.ch.zone_of_site || !a.ch.w || !a.ch.p_global || !a.ch.ll || !a.ch.max_size ||
        !a.ch.p_grow_connected || (d.n_zones > 0 && !a.ch.p_zones) ||
        (ctx->C == 3 && d.n_families > 0 && !a.ch.p_fam) || (src && !a.ch.source))
        return fail(ctx, SBZ_EINVAL, "null chain-state pointer");
    if (a.ch.alias_pending &&
        (!src || !a.ch.alias_p_global || (d.n_zones > 0 && !a.ch.alias_p_zones) ||
         (ctx->C == 3 && d.n_families > 0 && !a.ch.alias_p_fam)))
        return fail(ctx, SBZ_EINVAL, "alias_pending needs sample_source and the alias_p_* buffers");
    if (a.ch.tape && (!a.ch.tape_pos || !a.ch.tape_len))
        return fail(ctx, SBZ_EINVAL, "tape mode needs tape_pos and tape_len");
    if (src) return launch_mh_source(ctx, B, a);
    if (d.n_sites > 65535) return fail(ctx, SBZ_EINVAL, "sampler supports at most 65535 sites");
    const bool geo = a.geo_cost != nullptr;
    if (mh_lds_bytes(d, ctx->C, geo, a.gib != 0) > 160 * 1024)
        return fail(ctx, SBZ_EINVAL, "sampler state exceeds the 160 KiB of LDS (too many sites)");
    // planned steps per batch (Philox only): as many as SBZ_MH_LA asks whose columns fit the LDS,
    // and table slots for grouped parameter moves (one per wave): the most slots that leave room
    // for min(8, asked) planned steps, then the most planned steps beside them
    auto lds_of = [&](int la, int nt) {
        return MhLayout(d.n_sites, np_of(d.n_sites), d.n_states, d.n_zones, d.n_families, ctx->C, ctx->FamC,
                        MH_WAVES * WAVE, geo, la, a.gib != 0, nt).total;
    };
    constexpr size_t LDS_MAX = 160 * 1024;
    const int la_ask = a.ch.tape ? 1 : std::min(ctx->mh_la, LA);
    int ntab = la_ask > 1 ? std::min(MH_WAVES, ctx->mh_group) : 1;  // groups need plans
    while (ntab > 1 && lds_of(std::min(la_ask, 8), ntab) > LDS_MAX) ntab--;
    int la = la_ask;
    while (la > 1 && lds_of(la, ntab) > LDS_MAX) la--;
    a.la = la;
    a.ntab = ntab;
    const size_t lds = lds_of(la, ntab);
    auto fn = ctx->C == 3 ? mh_kernel<3, MH_WAVES> : mh_kernel<2, MH_WAVES>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
    }
    fn<<<B, MH_WAVES * WAVE, lds, ctx->stream>>>(a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "sampler launch");
    return SBZ_OK;
}

}  // namespace sbz
