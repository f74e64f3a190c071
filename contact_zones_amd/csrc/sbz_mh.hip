// sbz_mh.hip — batched Metropolis-Hastings for the sBayes zone model on CDNA4 (gfx950).
//
// One wave (64 lanes) runs one chain for n_steps without leaving the kernel:
// MCMCGenerative.step (sbayes/sampling/mcmc_generative.py:282-351) with the operators of
// ZoneMCMC / ZoneMCMCWarmup (sbayes/sampling/zone_sampling.py) for SAMPLE_SOURCE = false; priors
// zero, 'counts' on p_global / p_families and 'uniform' / 'quadratic' zone size (sbz_set_priors):
//   shrink_zone :866-933 (warm-up :1498-1574)   grow_zone :788-864 (:1418-1496)
//   swap_zone :704-786 (:1328-1416)             alter_weights :408-452
//   alter_p_global :454-493   alter_p_zones :495-535   alter_p_families :571-612
//   dirichlet_proposal :537-569 (q = exp(scipy dirichlet._logpdf) then log)
// Every decision is wave-uniform: all lanes draw the same values and take the same branches;
// lanes share the per-site / per-feature work.
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



namespace {

template <int C>
__global__ __launch_bounds__(WAVE) void mh_kernel(MhArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x;
    const int b = blockIdx.x;
    const int N = a.N, F = a.F, S = a.S, Z = a.Z, Fam = (C == 3) ? a.Fam : 0;
    const sbz_chains &ch = a.ch;

    // LDS carve-up
    double *col = reinterpret_cast<double *>(lds);                  // (1+Z+Fam)*S + C doubles
    const int ncol = (1 + Z + Fam) * S + C;
    int *zsize = reinterpret_cast<int *>(col + ((ncol + 1) & ~1));  // [Z]
    uint16_t *nb = reinterpret_cast<uint16_t *>(zsize + ((Z + 1) & ~1));  // [N]
    uint8_t *zos = reinterpret_cast<uint8_t *>(nb + ((N + 1) & ~1));      // [N]
    int *stat = reinterpret_cast<int *>(zos + ((N + 3) & ~3));  // [MH_STAT_INTS] proposed | accepted

    uint8_t *gzos = ch.zone_of_site + (size_t)b * N;
    double *w = ch.w + (size_t)b * F * C;
    double *pg = ch.p_global + (size_t)b * F * S;
    double *pz = Z > 0 ? ch.p_zones + (size_t)b * Z * F * S : pg;  // never read when Z == 0
    // without inheritance there is no family table: point at p_global (never read, C == 2)
    double *pf = (C == 3 && Fam > 0) ? ch.p_fam + (size_t)b * Fam * F * S : pg;
    const int max_size = ch.max_size[b];
    const double p_grow = ch.p_grow_connected[b];

    // load the zone assignment; sizes
    for (int z = lane; z < Z; z += WAVE) zsize[z] = 0;
    if (lane < MH_STAT_INTS) stat[lane] = 0;
    for (int s = lane; s < N; s += WAVE) nb[s] = 0;
    wsync();
    int occ = 0;
    for (int s = lane; s < N; s += WAVE) {
        const int z = gzos[s];
        zos[s] = (uint8_t)z;
        if (z < Z) {
            atomicAdd(&zsize[z], 1);
            occ++;
        }
    }
    int occupied = uni(wave_sum_i(occ));
    wsync();

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
    int err = 0;             // first range-check failure (MH_IDX)
    long long err_val = 0;
    const long long nFS = (long long)F * S, nZFS = (long long)Z * F * S, nFamFS = (long long)Fam * F * S;
    uint16_t stamp = 0;
    // per-operator counters, kept in LDS by lane 0 (no dynamically indexed private array)

    // mark nb[t] = stamp for every site t adjacent to a member of zone z
    auto mark = [&](int z) {
        stamp++;
        if (stamp == 0) {  // wrapped: clear
            for (int s = lane; s < N; s += WAVE) nb[s] = 0;
            wsync();
            stamp = 1;
        }
        for (int s = lane; s < N; s += WAVE)
            if (zos[s] == z)
                for (int e = a.adj_ptr[s]; e < a.adj_ptr[s + 1]; e++)
                    nb[MH_IDX(a.adj_idx[MH_IDX(e, a.nnz, 1)], N, 2)] = stamp;
        wsync();
    };
    auto is_nb = [&](int s) { return nb[s] == stamp && zos[s] == NONE; };
    // site selections: SEL_NB (neighbours of the marked zone, free), SEL_FREE, SEL_ZONE (members of z)
    enum { SEL_NB = 0, SEL_FREE = 1, SEL_ZONE = 2 };
    auto sel = [&](int mode, int z, int s) -> bool {
        const int zs = zos[s];
        return mode == SEL_NB ? (nb[s] == stamp && zs == NONE) : (mode == SEL_FREE ? zs == NONE : zs == z);
    };
    // number of selected sites; the k-th selected site in ascending order (-1 if none)
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

    // delta log-likelihood of moving site s from zone zo to zone zn (NONE = no zone)
    auto delta_site = [&](int s, int zo, int zn) {
        const int fc = (C == 3) ? a.fam_site[MH_IDX(s, N, 3)] : 0;
        const bool hf = fc > 0;
        double mn = 1.0, mo = 1.0;
        int en = 0, eo = 0;
        for (int f = lane; f < F; f += WAVE) {
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
        const double d = (log(mn) - log(mo)) + (double)(en - eo) * LN2;
        return uni(wave_sum(d));
    };

    // stage feature f's parameter column into LDS: pg | pz[z] | pf[fam] | w
    auto stage_col = [&](int f) {
        for (int i = lane; i < ncol; i += WAVE) {
            // one unconditional load from a pointer chosen per element (always a valid index)
            const int seg = i / S, r = i - seg * S;
            const double *src;
            long long idx, lim;
            if (i >= (1 + Z + Fam) * S) {
                src = w;
                idx = (long long)f * C + (i - (1 + Z + Fam) * S);
                lim = (long long)F * C;
            } else if (seg == 0) {
                src = pg;
                idx = (long long)f * S + r;
                lim = nFS;
            } else if (seg <= Z) {
                src = pz;
                idx = ((long long)(seg - 1) * F + f) * S + r;
                lim = nZFS;
            } else {
                src = pf;
                idx = ((long long)(seg - 1 - Z) * F + f) * S + r;
                lim = nFamFS;
            }
            col[i] = ldp(src + MH_IDX(idx, lim, 9));
        }
        wsync();
    };
    // delta of a parameter move on feature f: component comp (0 global, 1 zone, 2 family,
    // 3 weights), row (zone / family), the two altered entries ia, ib with new values va, vb
    auto delta_param = [&](int f, int comp, int row, int ia, int ib, double va, double vb) {
        const double *wc = col + (1 + Z + Fam) * S;
        double wold[3], wnew[3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            wold[i] = (C == 3 || i < 2) ? wc[i] : 0.0;
            wnew[i] = (comp == 3 && i == ia) ? va : ((comp == 3 && i == ib) ? vb : wold[i]);
        }
        const uint8_t *ob = a.obs_fm + MH_IDX((long long)f * a.Np, (long long)F * a.Np, 13);
        double mn = 1.0, mo = 1.0;
        int en = 0, eo = 0;
        for (int p = lane; p < N; p += WAVE) {
            const int s = a.perm[p];
            const int zc = zos[s];
            const int fc = (C == 3) ? a.famc[p] : 0;
            const int x = a.xs8 ? (ob[p] >> 3) : ob[p];
            const bool na = x == S;
            bool hit;
            if (comp == 3) hit = true;
            else if (comp == 0) hit = !na && (x == ia || x == ib);
            else if (comp == 1) hit = zc == row && !na && (x == ia || x == ib);
            else hit = fc == row + 1 && !na && (x == ia || x == ib);
            if (!hit) continue;
            const int xc = na ? 0 : x;
            const bool hz = zc < Z, hf = fc > 0;
            const double l0 = col[xc];
            const double l1 = hz ? col[(1 + zc) * S + xc] : 0.0;
            const double l2 = hf ? col[(1 + Z + fc - 1) * S + xc] : 0.0;
            double n0 = l0, n1 = l1, n2 = l2;
            if (comp == 0) n0 = x == ia ? va : vb;
            else if (comp == 1) n1 = x == ia ? va : vb;
            else if (comp == 2) n2 = x == ia ? va : vb;
            mo *= cell<C>(wold, hz, hf, na, l0, l1, l2);
            mn *= cell<C>(comp == 3 ? wnew : wold, hz, hf, na, n0, n1, n2);
            renorm(mo, eo);
            renorm(mn, en);
        }
        const double d = (log(mn) - log(mo)) + (double)(en - eo) * LN2;
        return uni(wave_sum(d));
    };

    // One MH step per iteration, in four phases with one call site each (keeps the kernel small):
    //   1. draw the operator and its move (zone moves: sites and Hastings terms; parameter moves:
    //      the feature, component and pair of entries);  2. Dirichlet proposal (parameter moves);
    //   3. delta log-likelihood;  4. accept / reject and apply.
    bool broken = false;  // a tape decision with no matching candidate (replay mismatch)
    for (int step = 0; step < a.n_steps; step++) {
        if (rng.bad || broken) break;
        const int op = rng.op(a.op_cdf, a.nops);
        if (op < 0 || op > P_FAMILIES || (op == P_FAMILIES && (C == 2 || Fam == 0)) ||
            (op <= SWAP && Z == 0) || (op == P_ZONES && Z == 0)) {
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
                    const int n_nb = count_sel(SEL_NB, 0);
                    const int cnt = connected ? n_nb : n_free;
                    if (cnt > 0) {
                        const int site = kth_sel(connected ? SEL_NB : SEL_FREE, 0, rng.below(cnt));
                        int site_rm = -2;
                        if (op == SWAP) site_rm = kth_sel(SEL_ZONE, z, rng.below(size));
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
                const int site = kth_sel(SEL_ZONE, z, rng.below(size));
                if (site < 0) {
                    broken = true;
                    break;
                }
                // back step: grow of the shrunk zone (neighbours of the zone without the site)
                wsync();
                if (lane == 0) zos[site] = NONE;
                wsync();
                mark(z);
                const int n_back = count_sel(SEL_NB, 0);
                double q_back = (1.0 - p_grow) * (1.0 / (double)(n_free + 1));
                if (is_nb(site)) q_back += p_grow * (1.0 / (double)n_back);
                if (a.warmup) q_back = 1.0 / (double)(size + 1);  // zone_sampling.py:1561
                wsync();
                if (lane == 0) zos[site] = (uint8_t)z;
                wsync();
                log_q = uni(log(1.0 / (double)size));
                log_q_back = uni(log(q_back));
                dprior = uni(size_prior_delta(a.size_prior, N, size, size - 1));
                sa = site;
                zoa = z;
                zna = NONE;
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
            MH_IDX(off + ia, lim, 15);
            MH_IDX(off + ib, lim, 15);
            if (__ballot(err != 0)) {
                broken = true;
                break;
            }
            base = arr + off;
            poff = off;
        }

        // ---- 2. Dirichlet proposal of the pair (zone_sampling.py:421-438, :537-569)
        double nv0 = 0.0, nv1 = 0.0;
        if (comp >= 0) {
            const double c0 = uni(ldp(base + ia)), c1 = uni(ldp(base + ib));
            // without inheritance the weight pair is used as is (zone_sampling.py:440-443)
            const bool raw = C == 2 && comp == 3;
            const double sum = raw ? 1.0 : c0 + c1;
            const double t0 = raw ? c0 : c0 / sum, t1 = raw ? c1 : c1 / sum;
            double u0, u1;
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

        // ---- 3. delta log-likelihood
        double delta = 0.0;
        if (sa >= 0) {
            delta = delta_site(sa, zoa, zna);
            if (sb >= 0) delta = delta + delta_site(sb, zna, NONE);
        } else if (comp >= 0) {
            stage_col(f);
            delta = delta_param(f, comp, row, ia, ib, nv0, nv1);
        }
        if (__ballot(err != 0)) {  // a range check failed: stop before using the move
            broken = true;
            break;
        }

        // ---- 4. metropolis_hastings_ratio (mcmc_generative.py:331-351, uniform priors)
        bool accept = false;
        if (log_q_back == -INFINITY) {
            accept = false;
        } else if (log_q == -INFINITY) {
            accept = true;
        } else {
            const double mh = (delta * 1.0) - (log_q - log_q_back) + dprior;
            accept = log(rng.real()) < mh;
        }
        if (lane == 0) stat[op]++;
        if (accept) {
            if (lane == 0) stat[SBZ_N_OPS + op]++;
            ll = ll + delta;
            prior = prior + dprior;
            wsync();
            if (sa >= 0) {
                if (lane == 0) {
                    zos[sa] = (uint8_t)zna;
                    if (zoa < Z) zsize[zoa]--;
                    if (zna < Z) zsize[zna]++;
                    if (sb >= 0) {
                        zos[sb] = NONE;
                        zsize[zna]--;
                    }
                }
                occupied += (zna < Z ? 1 : -1) + (sb >= 0 ? -1 : 0);
            } else if (lane == 0) {
                stp(base + ia, nv0);
                stp(base + ib, nv1);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            wsync();
        }
        if (ch.trace_op && lane == 0) {
            const size_t t = (size_t)b * a.n_steps + step;
            ch.trace_op[t] = (int8_t)op;
            ch.trace_accept[t] = accept ? 1 : 0;
            ch.trace_ll[t] = ll;
        }
        if (ch.trace_zos) {
            uint8_t *tz = ch.trace_zos + ((size_t)b * a.n_steps + step) * N;
            for (int s = lane; s < N; s += WAVE) tz[s] = zos[s];
        }
    }

    for (int s = lane; s < N; s += WAVE) gzos[s] = zos[s];
    if (lane == 0) {
        ch.ll[b] = ll;
        if (ch.prior) ch.prior[b] = prior;
        if (ch.tape_pos) ch.tape_pos[b] = rng.pos;
        if (ch.counter) ch.counter[b] = rng.ctr;
        if (ch.status) ch.status[b] = broken ? 2 : (rng.bad ? 1 : 0);
    }
    if (lane < SBZ_N_OPS) {  // per-operator counters, one lane each
        if (ch.accepted) ch.accepted[(size_t)b * SBZ_N_OPS + lane] += stat[SBZ_N_OPS + lane];
        if (ch.proposed) ch.proposed[(size_t)b * SBZ_N_OPS + lane] += stat[lane];
    }
    {
        const uint64_t bad = __ballot(err != 0);
        if (bad) {
            const int code = __shfl(err, (int)__builtin_ctzll(bad), 64);
            if (lane == 0 && ch.status) ch.status[b] = 16 + code;
        }
    }
}

}  // namespace

size_t mh_lds_bytes(const sbz_dims &d, int C) {
    const size_t Fam = C == 3 ? (size_t)d.n_families : 0;
    const size_t ncol = (1 + (size_t)d.n_zones + Fam) * d.n_states + C;
    return ((ncol + 1) & ~(size_t)1) * 8 + (((size_t)d.n_zones + 1) & ~(size_t)1) * 4 +
           (((size_t)d.n_sites + 1) & ~(size_t)1) * 2 + (((size_t)d.n_sites + 3) & ~(size_t)3) +
           MH_STAT_INTS * 4;
}

int launch_mh(sbz_ctx *ctx, int B, int n_steps, const sbz_mh_config *cfg, const sbz_chains *chains) {
    const sbz_dims &d = ctx->d;
    if (!ctx->d_adj_ptr) return fail(ctx, SBZ_ESTATE, "sbz_set_network must be called before sbz_mh_run_device");
    if (B <= 0 || n_steps <= 0) return SBZ_OK;
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
    allowed[SHRINK] = allowed[GROW] = allowed[SWAP] = true;
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
                                             (i == 7 ? " (gibbsish_sample_zones) is not supported"
                                                     : " is not available in this mode (sample_source)"));
        if (p > 0.0) last = i;
        tot += p;
    }
    if (!(tot > 0.0)) return fail(ctx, SBZ_EINVAL, "operator probabilities sum to 0");
    const double zone_ops = cfg->op_prob[SHRINK] + cfg->op_prob[GROW] + cfg->op_prob[SWAP] +
                            cfg->op_prob[P_ZONES] + cfg->op_prob[G_P_ZONES];
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
    const size_t lds = mh_lds_bytes(d, ctx->C);
    if (lds > 64 * 1024) return fail(ctx, SBZ_EINVAL, "sampler state exceeds 64 KiB of LDS (too many sites)");
    if (ctx->C == 3) mh_kernel<3><<<B, WAVE, lds, ctx->stream>>>(a);
    else mh_kernel<2><<<B, WAVE, lds, ctx->stream>>>(a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "sampler launch");
    return SBZ_OK;
}

}  // namespace sbz
