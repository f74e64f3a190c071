// sbz_internal.h — shared definitions for the HIP implementation of include/sbz.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/sbz.h"

namespace sbz {

// Device buffer that grows on demand (kept for the context's lifetime).
struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
};

struct LikArgs {
    int N, F, S, Z, Fam, C, FamC;
    int Np;          // sites padded to a multiple of 64 * sites-per-lane
    int W, fpw;      // tasks (single-wave workgroups) per chain, features per task
    int xs8;         // obs bytes hold x*8 (S + 1 <= 32) instead of x
    int B;
    // Sites are stored in a family-sorted order (position p holds site perm[p]) so that
    // neighbouring lanes mostly read the same table row (LDS bank-conflict free).
    const uint8_t *obs_fm;  // [F][Np]  x (or x*8) by position, x = S for NA; padding holds 0
    const uint8_t *famc;    // [Np]     by position: 0 = no family (or no inheritance), fam + 1
    const int *perm;        // [Np]     site of each position (padding: 0)
    const uint8_t *zone;    // [B][N]   zone index, 255 = none
    const double *w;        // [B][F][C]
    const double *pg;       // [B][F][S]
    const double *pz;       // [B][Z][F][S]
    const double *pf;       // [B][Fam][F][S] (C == 3 only)
    const uint8_t *src_pm;  // [B][F][Np] component per cell by position (position-major), or nullptr
    const uint8_t *src_rm;  // [B][N][F]  the caller's sources by site (lik_source_generic_kernel)
    int pk_row;             // src_pm holds 2-bit planes (source_to_pk_kernel): bytes per feature row
    double *partial;        // [B][W]     task partial sums
    unsigned *ticket;       // [B]        finished tasks per chain (0 between launches)
    unsigned *zflag;        // [B]        source branch: a task saw a zero selected weight (0
                            //            between launches), or nullptr (mixture)
    double *out;            // [B]        log-likelihood per chain
};

}  // namespace sbz

struct sbz_ctx {
    int device = 0;
    sbz_dims d{};
    int C = 2, FamC = 1;
    int Np = 0, spl = 4, xs8 = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    uint8_t *d_obs_fm = nullptr;
    uint8_t *d_famc = nullptr;
    int *d_perm = nullptr;  // [Np] site index of each position (family-sorted order)
    // sampler data (sbz_open / sbz_set_network)
    uint8_t *d_obs_sm = nullptr;    // [N][F] x by site (S = NA)
    uint8_t *d_fam_site = nullptr;  // [N] family class by site
    int *d_adj_ptr = nullptr, *d_adj_idx = nullptr;  // CSR network
    int adj_nnz = 0;
    int *d_app_list = nullptr, *d_app_cnt = nullptr; // [F][S] applicable states, [F] counts
    double *d_alpha_g = nullptr;  // [F][S] 'counts' prior on p_global (sbz_set_priors) or null
    double *d_alpha_f = nullptr;  // [Fam][F][S] 'counts' prior on p_families or null
    int size_prior = 0;           // 0 none, 1 uniform, 2 quadratic
    double *d_geo_cost = nullptr; // [N][N] 'cost_based' geo prior costs (sbz_set_geo_prior) or null
    double geo_scale = 0.0;
    double *d_gc_g = nullptr;     // [F][S] Gibbs prior counts of p_global (sbz_set_gibbs_counts)
    double *d_gc_f = nullptr;     // [Fam][F][S] of p_families
    std::vector<int> h_perm;  // [Np] host copy of d_perm, -1 at the padding positions
    // options (sbz_set_option; defaults are the production choices)
    int lik_banked = 1;    // SBZ_OPT_LIK_BANKED 0: dense kernel with the packed [class][x] table
    int src_rc = 1;        // SBZ_OPT_SRC_TABLE 0: source branch on the generic per-cell kernel
    int src_stage = 1;     // SBZ_OPT_SRC_STAGE 0: source-mode sampler passes read parameters from L2
    const void *mix_occ_fn = nullptr;  // the kernel mix_occ was queried for
    int tasks_per_cu = 0;  // SBZ_OPT_LIK_TASKS_PER_CU: single-wave tasks per CU per launch (0: by shape)
    int mix_occ = 0;       // resident mixture-kernel waves per CU (queried at first launch)
    int n_cu = 256;        // compute units of the device
    int src_waves = 0;     // SBZ_OPT_SRC_WAVES: waves per chain of the source-mode sampler (0: 8)
    int mh_la = 24;        // SBZ_OPT_MH_LOOKAHEAD: sampler proposals planned ahead per batch (1..24)
    int mh_group = 8;      // SBZ_OPT_MH_GROUP: grouped planned parameter moves (1..8; at most the waves)
    int src_pack = 1;      // SBZ_OPT_SRC_PACK 0: by-site likelihood sources reordered into bytes, not bit planes
    int src_hbm = 0;       // SBZ_OPT_SRC_HBM 1: source-mode sampler keeps sources in HBM even when they fit LDS
    int src_pass_tables = 1;  // SBZ_OPT_SRC_PASS_TABLES 0: HBM-source sampler passes per cell, no count tables
    std::string last_kernels;  // sbz_last_kernels
    sbz::DevBuf mh_stage;      // host-form sampler staging (sbz_mh_run)
    sbz::DevBuf partial, ticket, zflag, src_t, stage, out, src_cand, flags;
    sbz::DevBuf src_ctab;      // source-mode sampler count tables (current / candidate per chain)
    std::string err;
};

namespace sbz {

// Ensure `buf` holds at least `bytes` (contents not preserved).
int ensure(sbz_ctx *ctx, DevBuf &buf, size_t bytes);
int fail(sbz_ctx *ctx, int code, const std::string &msg);
int hip_fail(sbz_ctx *ctx, hipError_t e, const char *what);

size_t lik_lds_bytes(const sbz_dims &d, bool source_mode);
// Raise the dynamic-LDS limit of the likelihood kernels (gfx950: 160 KiB per workgroup).
int lik_configure(sbz_ctx *ctx);
// Sites per lane of the likelihood kernels for n_sites (4, 8, 16 or 32).
int sites_per_lane(int n_sites);
// Positions of the likelihood context: n_sites padded to a multiple of 64 * sites_per_lane.
inline int np_of(int n_sites) {
    const int chunk = 64 * sites_per_lane(n_sites);
    return (n_sites + chunk - 1) / chunk * chunk;
}

// Sampler (sbz_mh.hip)
size_t mh_lds_bytes(const sbz_dims &d, int C, bool geo = false, bool gib = false);
int launch_mh(sbz_ctx *ctx, int B, int n_steps, const sbz_mh_config *cfg, const sbz_chains *chains);
// sbz_draw_gamma: n gamma draws of the samplers' generator (device arrays)
int launch_draw_gamma(sbz_ctx *ctx, int n, const double *alpha, uint64_t seed, double *out);

// Launch the likelihood kernels for B chains (all pointers device); out_ll device [B].
// source_pm: `source` is [B][F][Np] by position (else [B][N][F] by site).
int launch_loglik(sbz_ctx *ctx, int B, const uint8_t *zone, const double *w, const double *pg,
                  const double *pz, const double *pf, const uint8_t *source, bool source_pm,
                  double *out_ll);
// [B][N][F] by site <-> [B][F][Np] by position (to_pm), device arrays, on ctx's stream.
int launch_source_transpose(sbz_ctx *ctx, int B, const uint8_t *src, uint8_t *dst, bool to_pm);

}  // namespace sbz
