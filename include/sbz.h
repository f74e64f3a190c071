/*
 * sbz.h — C-ABI of the MI355X-native sBayes likelihood + sampler core.
 *
 * The reference (sBayes, Python) has no native boundary: its hot path is called
 * in-process.  The entry points below are exactly what a ctypes binding on the
 * reference side would bind to replace that path (INTEGRATION.md shows the stub):
 *
 *   sbz_loglik_batch / sbz_loglik_batch_device
 *       replaces  Likelihood.__call__(sample, caching=False)      sbayes/model.py:145-171
 *       (incl.    update_component_likelihoods :230-249, update_weights :257-294,
 *                 normalize_weights :436-452, combine_lh :173-184)  — B chains per call
 *   sbz_set_network / sbz_mh_run (host arrays) / sbz_mh_run_device
 *       replaces  MCMCGenerative.step (the generate_samples hot loops) sbayes/sampling/mcmc_generative.py:149-351
 *       with the  operators of ZoneMCMC / ZoneMCMCWarmup           sbayes/sampling/zone_sampling.py:408-933,1272-1577
 *
 * Conventions
 *   - Return 0 (SBZ_OK) on success, a negative SBZ_E* code otherwise; the message is
 *     available from sbz_last_error(ctx).  No exceptions cross the ABI.  A log-likelihood
 *     of -inf is a value, not an error (combine_lh source branch, sbayes/model.py:181-182).
 *   - Host arrays are borrowed for the duration of the call, C-contiguous, in the layouts
 *     documented per argument.  Device arrays (the *_device entry points) must be device
 *     pointers valid on ctx's device; those calls are asynchronous on ctx's stream.
 *   - One context per GPU per process; calls on one context must be serialised.
 *
 * Layouts (B = chains in the call, N sites, F features, S states, Z zones, Fam families,
 * C = 3 with inheritance else 2):
 *   obs          int8   [N][F]        state index 0..S-1, -1 = NA         (one-hot features, util.py:289-336)
 *   fam_of_site  uint8  [N]           family index, 255 = no family       (families (Fam,N), disjoint)
 *   zone_of_site uint8  [B][N]        zone index, 255 = no zone           (zones (Z,N), disjoint)
 *   w            double [B][F][C]     unnormalised mixture weights         (Sample.weights)
 *   p_global     double [B][F][S]                                          (Sample.p_global[0])
 *   p_zones      double [B][Z][F][S]                                       (Sample.p_zones)
 *   p_fam        double [B][Fam][F][S] or NULL without inheritance         (Sample.p_families)
 *   source       uint8  [B][N][F]     component index per cell, or NULL   (Sample.source one-hot -> index)
 *   source_pm    uint8  [B][F][Np]    the same by POSITION: row f = feature f, column p = site
 *                                     positions[p] of the context's site order (sbz_site_positions;
 *                                     Np >= N, columns p >= N are padding and never read).  The
 *                                     layout the kernels read in place; the sampler keeps it.
 */
#ifndef SBZ_H
#define SBZ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBZ_NONE 255

enum sbz_status {
    SBZ_OK = 0,
    SBZ_EINVAL = -1,   /* bad argument / shape */
    SBZ_EHIP = -2,     /* HIP runtime error */
    SBZ_ENOMEM = -3,   /* device allocation failed */
    SBZ_ESTATE = -4,   /* call out of order (e.g. no chains resident) */
};

enum sbz_flags {
    SBZ_INHERITANCE = 1, /* model families: C = 3 components (Model.inheritance, model.py:45) */
};

enum sbz_source_layout {
    SBZ_SOURCE_BY_SITE = 0,     /* [B][N][F], the reference's Sample.source order */
    SBZ_SOURCE_BY_POSITION = 1, /* [B][F][Np] in the context's site order (source_pm above) */
};

typedef struct sbz_dims {
    int32_t n_sites;
    int32_t n_features;
    int32_t n_states;   /* max states over features (S), <= 127 */
    int32_t n_zones;    /* Z, 0..254 */
    int32_t n_families; /* Fam, 0..254 (ignored without SBZ_INHERITANCE) */
    int32_t flags;      /* SBZ_INHERITANCE */
} sbz_dims;

typedef struct sbz_ctx sbz_ctx;

/* Library version string. */
const char *sbz_version(void);

/* Number of visible HIP devices (0 if none); never fails. */
int sbz_device_count(void);

/*
 * Open a context on `device`, uploading the shared data once (obs, fam_of_site).
 * Replaces the per-chain Model copies' shared Likelihood state
 * (Likelihood.__init__, sbayes/model.py:105-131; mcmc_generative.py:80).
 */
int sbz_open(int device, const sbz_dims *dims, const int8_t *obs, const uint8_t *fam_of_site,
             sbz_ctx **out);
void sbz_close(sbz_ctx *ctx);
const char *sbz_last_error(const sbz_ctx *ctx);

/* Use `hip_stream` (a hipStream_t, e.g. torch.cuda.current_stream().cuda_stream) verbatim for
 * every subsequent launch; NULL is the device's legacy null stream.  A new context launches on
 * a non-blocking stream of its own. */
int sbz_set_stream(sbz_ctx *ctx, void *hip_stream);
int sbz_synchronize(sbz_ctx *ctx);

/* Tuning options of a context.  Every default is the production choice; nothing is read from the
 * environment.  No reference counterpart (the reference has no device code).
 *   SBZ_OPT_LIK_TASKS_PER_CU  likelihood single-wave tasks per CU and launch; 0 (default) = by
 *                             shape: 4 when N <= 256, else the kernel's occupancy
 *   SBZ_OPT_LIK_BANKED        1 (default): the banked table layout of the dense mixture kernel where
 *                             it applies (S + 1 <= 16); 0: the packed [class][x] layout
 *   SBZ_OPT_SRC_TABLE         1 (default): source branch on the table kernel where it applies;
 *                             0: the per-cell kernel
 *   SBZ_OPT_SRC_WAVES         source-mode sampler waves per chain: 0 (default) = 8, or 1, 4, 8
 *   SBZ_OPT_SRC_HBM           1: the source-mode sampler keeps the sources in HBM even when they
 *                             fit LDS (default 0: LDS when they fit)
 *   SBZ_OPT_SRC_STAGE         1 (default): the source-mode sampler stages parameters in LDS where
 *                             they fit; 0: its passes read them from L2
 *   SBZ_OPT_MH_LOOKAHEAD      sampler with Philox draws: parameter proposals planned ahead per
 *                             batch, 1..24 (default 24; 1 = none; trajectories do not depend on it)
 *   SBZ_OPT_SRC_PASS_TABLES   1 (default): the source-mode sampler with its sources in HBM runs its
 *                             passes over the observations on per-feature tables and keeps per-chain
 *                             source counts, so the Gibbs parameter operators need no pass (where the
 *                             tables fit: 4 or 8 waves, Np <= 2048, table lines and count-table
 *                             columns <= 192, and the LDS holds them); 0: per-cell passes
 *   SBZ_OPT_MH_GROUP          mixture sampler with Philox draws: planned parameter moves on pairwise
 *                             different features whose deltas are computed at once, one per wave,
 *                             1..8 (default 8; at most the sampler's waves per chain, fewer when the
 *                             per-wave cell tables do not fit the LDS; trajectories do not depend on it)
 *   SBZ_OPT_SRC_PACK          1 (default): sbz_loglik_batch / sbz_loglik_batch_device with by-site
 *                             sources on the table kernel, N > 512 and F a multiple of 4 (F >= 16),
 *                             reorder the sources into 2-bit component planes by position before the
 *                             launch; 0: into one byte per cell (the by-position layout).  Results do
 *                             not depend on it.
 * SBZ_EINVAL for an unknown option or a value out of range. */
enum sbz_option {
    SBZ_OPT_LIK_TASKS_PER_CU = 1,
    SBZ_OPT_LIK_BANKED = 2,
    SBZ_OPT_SRC_TABLE = 3,
    SBZ_OPT_SRC_WAVES = 4,
    SBZ_OPT_SRC_HBM = 5,
    SBZ_OPT_SRC_STAGE = 6,
    SBZ_OPT_MH_LOOKAHEAD = 7,
    SBZ_OPT_SRC_PASS_TABLES = 8,
    SBZ_OPT_MH_GROUP = 9,
    SBZ_OPT_SRC_PACK = 10,
};
int sbz_set_option(sbz_ctx *ctx, int32_t option, int64_t value);
int sbz_get_option(const sbz_ctx *ctx, int32_t option, int64_t *value);

/* The context's site order: positions[p] = site at position p for p < N, -1 for the padding
 * positions N <= p < Np (sites sorted stably by family, so that neighbouring lanes read the same
 * table rows).  Returns Np (> 0), or a negative code; `positions` (int32[Np]) may be NULL. */
int sbz_site_positions(const sbz_ctx *ctx, int32_t *positions);

/*
 * Full log-likelihood of B chains, host buffers (PCIe copies included; blocks until done).
 * source == NULL: mixture branch  sum_{s,f} log sum_c w_norm*lh      (model.py:174-176)
 * source != NULL: source branch   sum_{s,f} log (w_norm*lh)[source]  (model.py:177-184)
 * out_ll: double[B] (host).
 */
int sbz_loglik_batch(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w,
                     const double *p_global, const double *p_zones, const double *p_fam,
                     const uint8_t *source, double *out_ll);

/* Same, with the (host) sources by position (source_pm [B][F][Np], see Layouts; padding columns
 * are not read): the copy is the likelihood's input as is, with no by-site -> by-position
 * transpose on the device.  Replaces the same model.py:177-184 call as sbz_loglik_batch. */
int sbz_loglik_batch_pm(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w,
                        const double *p_global, const double *p_zones, const double *p_fam,
                        const uint8_t *source_pm, double *out_ll);

/* Same, all pointers on the device (out_ll: double[B] device); asynchronous on ctx's stream.
 * The device entry points (this one and sbz_mh_run_device) TRUST their index bytes: they do
 * not re-check zone_of_site < n_zones (or SBZ_NONE) and source < C, which sbz_loglik_batch
 * checks on the host.  A caller holding device buffers of unknown origin calls
 * sbz_check_indices_device first. */
int sbz_loglik_batch_device(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w,
                            const double *p_global, const double *p_zones, const double *p_fam,
                            const uint8_t *source, double *out_ll);

/* Same, with the sources by position (source_pm [B][F][Np], see Layouts): read in place, as the
 * source-mode sampler keeps them (sbz_chains.source_layout = SBZ_SOURCE_BY_POSITION).  The
 * reference's combine_lh source branch (model.py:177-184) on the sampler's own state. */
int sbz_loglik_batch_device_pm(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w,
                               const double *p_global, const double *p_zones, const double *p_fam,
                               const uint8_t *source_pm, double *out_ll);

/* Convert B chains' sources between the layouts (device arrays, asynchronous on ctx's stream):
 * to_positions = 1: src [B][N][F] -> dst [B][F][Np] (padding columns 0); 0: the reverse. */
int sbz_source_layout_device(sbz_ctx *ctx, int B, const uint8_t *src, uint8_t *dst,
                             int32_t to_positions);

/* Validate device index arrays (zone_of_site [B][N]: < n_zones or SBZ_NONE; source
 * [B][N][F] or NULL: < C) with one kernel pass; synchronises ctx's stream.  SBZ_EINVAL with
 * a message naming the first offending array, SBZ_OK otherwise.  No reference counterpart:
 * the reference's arrays are host numpy arrays whose shapes/values it builds itself. */
int sbz_check_indices_device(sbz_ctx *ctx, int B, const uint8_t *zone_of_site,
                             const uint8_t *source);
/* Same for sources by position (source_pm [B][F][Np]; padding columns are not checked). */
int sbz_check_indices_device_pm(sbz_ctx *ctx, int B, const uint8_t *zone_of_site,
                                const uint8_t *source_pm);

/* Device memory helpers (so a host without torch can stage device buffers). */
int sbz_device_alloc(sbz_ctx *ctx, uint64_t bytes, void **out);
int sbz_device_free(sbz_ctx *ctx, void *ptr);
int sbz_memcpy_h2d(sbz_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int sbz_memcpy_d2h(sbz_ctx *ctx, void *dst, const void *src, uint64_t bytes);

/* Bytes of LDS the likelihood kernel needs per workgroup for these dims (0 if unsupported). */
uint64_t sbz_lik_lds_bytes(const sbz_dims *dims, int source_mode);

/* Diagnostics: the kernels the context's last launch ran, space-separated (a likelihood launch,
 * e.g. "lik_mixture_kernel" or "lik_source_rc_kernel"; a source-mode sampler launch,
 * "mh_src_kernel<lds>", "mh_src_kernel<hbm>" or "mh_src_kernel<hbm, tables>"), "" before the
 * first. */
const char *sbz_last_kernels(const sbz_ctx *ctx);

/* Diagnostics: n draws of the samplers' gamma generator (LaneRng::gamma, Marsaglia-Tsang on
 * Philox4x32-10 uniforms; the Dirichlet draws of alter_* / gibbs_sample_* in Philox mode), draw i
 * with shape alpha[i] from its own stream (key = seed, chain = i / 64, lane i % 64).  Host
 * arrays [n]; for distribution tests.  Returns 0 or a negative code. */
int sbz_draw_gamma(sbz_ctx *ctx, int32_t n, const double *alpha, uint64_t seed, double *out);

/* ------------------------------------------------------------------------------------------
 * Metropolis-Hastings sampler  (MCMCGenerative.step, sbayes/sampling/mcmc_generative.py:282-351,
 * operators of ZoneMCMC / ZoneMCMCWarmup, sbayes/sampling/zone_sampling.py:408-933, 1272-1577;
 * SAMPLE_SOURCE = false (sbz_mh.hip) and true (sbz_mh_src.hip); zero, 'counts', zone-size and
 * 'cost_based' geo priors).  One workgroup (4 waves; SAMPLE_SOURCE = true: 8) runs one chain
 * for n_steps in one launch.
 * ------------------------------------------------------------------------------------------ */

/* Canonical operator order of sbz_mh_config.op_prob. */
enum sbz_op {
    SBZ_OP_SHRINK_ZONE = 0, SBZ_OP_GROW_ZONE = 1, SBZ_OP_SWAP_ZONE = 2, SBZ_OP_ALTER_WEIGHTS = 3,
    SBZ_OP_ALTER_P_GLOBAL = 4, SBZ_OP_ALTER_P_ZONES = 5, SBZ_OP_ALTER_P_FAMILIES = 6,
    SBZ_OP_GIBBSISH_SAMPLE_ZONES = 7, /* zone_sampling.py:619-702; weight 0 in the reference's table (mcmc_setup.py:77) */
    /* SAMPLE_SOURCE = true operators (mcmc_setup.py:80-87, zone_sampling.py:180-406) */
    SBZ_OP_GIBBS_SAMPLE_SOURCES = 8, SBZ_OP_GIBBS_SAMPLE_WEIGHTS = 9,
    SBZ_OP_GIBBS_SAMPLE_P_GLOBAL = 10, SBZ_OP_GIBBS_SAMPLE_P_ZONES = 11,
    SBZ_OP_GIBBS_SAMPLE_P_FAMILIES = 12,
    SBZ_N_OPS = 16 /* width of op_prob and of the per-chain counters */
};

typedef struct sbz_mh_config {
    double op_prob[16];   /* operator weights, SBZ_OP_* order (normalised here) (mcmc_setup.py:70-95) */
    double precision[4];  /* PROPOSAL_PRECISION: weights, universal, contact, inheritance */
    int32_t min_size;     /* MIN_M (model.py:43) */
    int32_t warmup;       /* 1: ZoneMCMCWarmup semantics (shrink back-probability 1/(size+1)) */
    int32_t sample_source;/* 1: SAMPLE_SOURCE = true (sbz_chains.source; Gibbs operators 8-12) */
    int32_t reserved;
} sbz_mh_config;

/* Chain state and I/O of a run; every pointer is a device pointer, chain-major (B chains). */
typedef struct sbz_chains {
    uint8_t *zone_of_site;            /* [B][N] in/out (255 = no zone) */
    double *w, *p_global, *p_zones, *p_fam;  /* in/out, layouts as sbz_loglik_batch */
    double *ll;                       /* [B] in/out: the chain's current log-likelihood */
    const int32_t *max_size;          /* [B] MAX_M per chain (warm-up: get_max_size_list) */
    const double *p_grow_connected;   /* [B] per chain (warm-up: 0.95 or the configured value) */
    /* draws: a replay tape of the reference's decisions (tests/golden/make_golden_mh.py) ... */
    const double *tape;               /* [B][tape_stride] or NULL for Philox */
    int64_t tape_stride;
    const int64_t *tape_len;          /* [B] */
    int64_t *tape_pos;                /* [B] in/out cursor */
    /* ... or Philox4x32-10 keyed by seed, counter (ctr, global chain id) */
    uint64_t seed;
    uint64_t chain_id0;               /* global id of chain 0 (rank offset) */
    uint64_t *counter;                /* [B] in/out, or NULL (start at 0) */
    int64_t *accepted, *proposed;     /* [B][SBZ_N_OPS] accumulated per operator, or NULL */
    int32_t *status;                  /* [B] 1 = tape exhausted, or NULL */
    int8_t *trace_op;                 /* [B][n_steps] or NULL */
    uint8_t *trace_accept;            /* [B][n_steps] (with trace_op) */
    double *trace_ll;                 /* [B][n_steps] (with trace_op) */
    uint8_t *trace_zos;               /* [B][n_steps][N] or NULL (tests) */
    double *prior;                    /* [B] in/out: the chain's log prior (sbz_set_priors), or NULL
                                         when every prior term is 0 */
    uint8_t *source;                  /* in/out (sample_source): component of each observation,
                                         0 global, 1 zone, 2 family (Sample.source), in the layout
                                         source_layout names.  By position, the padding columns
                                         (p >= N) may be rewritten with 0 (the HBM-sources kernel
                                         with pass tables copies whole rows back); never read. */
    /* sample_source only: the reference's Gibbs operators on p_global / p_zones / p_families
     * change the chain's Sample in place (zone_sampling.py:333-400), so the parameter arrays of a
     * logged sample (mcmc_generative.py:353-367 keeps references) go on changing until an
     * accepted operator replaces the Sample (Sample.copy, :100-115: the zone moves and
     * gibbs_sample_weights).  With alias_pending[b] = 1 the first such accept copies the chain's
     * p_* into alias_* and clears the flag. */
    int32_t *alias_pending;           /* [B] in/out, or NULL */
    double *alias_p_global, *alias_p_zones, *alias_p_fam;  /* [B][...] as p_global / p_zones / p_fam */
    int32_t source_layout;            /* sbz_source_layout of `source`: SBZ_SOURCE_BY_SITE [B][N][F]
                                         (0) or SBZ_SOURCE_BY_POSITION [B][F][Np] (the layout the
                                         likelihood reads in place, sbz_loglik_batch_device_pm) */
} sbz_chains;

/* Sampler-only data: applicable states (uint8 [F][S], data.states) and the site network as CSR
 * (data.network['adj_mat'], sbayes/util.py:139-155; rows sorted).  Call once after sbz_open. */
int sbz_set_network(sbz_ctx *ctx, const uint8_t *applicable, int32_t nnz, const int32_t *adj_indptr,
                    const int32_t *adj_indices);

/* Priors of the MH ratio (Prior.__call__, sbayes/model.py:484-505).  Default: all zero (the
 * uniform priors of config/default_config.json:33-40).
 *   alpha_global  double [F][S] or NULL: 'counts' prior on p_global — the Dirichlet
 *                 concentration of each applicable state (PGlobalPrior.dirichlet,
 *                 model.py:571-597, util.counts_to_dirichlet); other entries ignored.
 *   alpha_fam     double [Fam][F][S] or NULL: 'counts' prior on p_families (PFamiliesPrior,
 *                 model.py:631-672, util.inheritance_counts_to_dirichlet).
 *   size_prior    0 'none', 1 'uniform' (-sum log C(N, size)), 2 'quadratic' (-sum log size^2)
 *                 (ZoneSizePrior, model.py:893-976).
 * The kernel adds the prior difference of each proposal (dirichlet_logpdf terms of the two
 * altered states, or the changed zone size) to the MH ratio and carries sbz_chains.prior. */
int sbz_set_priors(sbz_ctx *ctx, const double *alpha_global, const double *alpha_fam,
                   int32_t size_prior);

/* 'cost_based' geo prior (GeoPrior, sbayes/model.py:979-1139; experiments/simulation/sim_exp2):
 *   cost   double [N][N] row-major cost matrix between sites (load_data.py:106-121: a cost file,
 *          or the distance matrix), or NULL to switch the geo prior off (uniform, 0);
 *   scale  > 0, the exponential's scale.
 * The geo prior is the mean exp(scale) log density over the edges of the minimum spanning tree
 * of the LAST zone's cost submatrix (geo_prior_distance, model.py:1096-1139, overwrites its value
 * in the zone loop, so zone n_zones - 1 alone counts; zero-cost edges are not counted, as in
 * scipy's sparse tree).  Zone moves that change that zone add the difference to the MH ratio. */
int sbz_set_geo_prior(sbz_ctx *ctx, const double *cost, double scale);

/* Prior pseudo-counts of the source-mode Gibbs operators (SAMPLE_SOURCE = true): p_global is
 * redrawn from Dirichlet(counts_global[f] + source counts) (gibbs_sample_p_global,
 * zone_sampling.py:334-357; PGlobalPrior.counts, model.py:576-586), p_families from
 * Dirichlet(counts_fam[fam][f] + ...) (:381-406; PFamiliesPrior.counts).  double [F][S] and
 * [Fam][F][S]; NULL = 1 everywhere (the 'uniform' priors' counts). */
int sbz_set_gibbs_counts(sbz_ctx *ctx, const double *counts_global, const double *counts_fam);

/* Run n_steps MH steps on B device-resident chains; asynchronous on ctx's stream.
 * With sample_source the chain's Gibbs scratch (F x max(S, 2) doubles of redraws, 8F bytes of
 * scans, the count tables) lives in the 160 KiB of LDS, the sources too when N*F fits (else HBM):
 * a shape beyond that (e.g. F*S above ~18k) is refused with SBZ_EINVAL and a message naming the
 * LDS budget before anything runs. */
int sbz_mh_run_device(sbz_ctx *ctx, int B, int n_steps, const sbz_mh_config *cfg,
                      const sbz_chains *chains);

/* ---- Host-form sampler (SURVEY.md §8b's sbz_mh_run): the same run on HOST arrays, for a
 * reference-side binding without a device allocator (ctypes + numpy only).  The state is staged
 * to the device, each chain's log-likelihood is evaluated from it (the reference's initial
 * _ll[c] = likelihood(sample), mcmc_generative.py:159-170), the chains run n_steps steps, and the
 * state, counters and traces are copied back.  Blocks until done. ---- */
typedef struct sbz_state {
    uint8_t *zone_of_site;            /* [B][N] in/out */
    double *w, *p_global, *p_zones, *p_fam;  /* in/out, layouts as sbz_loglik_batch */
    uint8_t *source;                  /* [B][N][F] in/out with cfg->sample_source, else NULL */
    double *ll;                       /* [B] out: each chain's log-likelihood after the run */
    double *prior;                    /* [B] in/out log prior (sbz_set_priors), or NULL when every
                                         prior term is 0 */
    const int32_t *max_size;          /* [B] MAX_M per chain */
    const double *p_grow_connected;   /* [B] */
    uint64_t chain_id0;               /* global id of chain 0 (Philox key) */
    uint64_t *counter;                /* [B] in/out Philox counters, or NULL (start at 0) */
    int64_t *accepted, *proposed;     /* [B][SBZ_N_OPS] accumulated, or NULL */
    int32_t *status;                  /* [B] out (1 = tape exhausted), or NULL */
} sbz_state;

typedef struct sbz_tape {             /* replay of the reference's recorded decisions */
    const double *values;             /* [B][stride] (tests/golden/make_golden_mh.py) */
    int64_t stride;
    const int64_t *len;               /* [B] */
    int64_t *pos;                     /* [B] in/out cursor, or NULL (start at 0) */
} sbz_tape;

typedef struct sbz_trace {            /* per-step trace, [B][n_steps] each, or NULL members */
    int8_t *op;                       /* operator (sbz_op) */
    uint8_t *accept;
    double *ll;                       /* log-likelihood after the step */
} sbz_trace;

/* tape == NULL: Philox4x32-10 draws keyed by (seed, chain_id0 + b, counter[b]). */
int sbz_mh_run(sbz_ctx *ctx, int B, int n_steps, const sbz_mh_config *cfg, uint64_t seed,
               const sbz_tape *tape, sbz_state *io_state, sbz_trace *out_trace);

/* Bytes of LDS the SAMPLE_SOURCE = false sampler needs per chain for these dims (0 if above the
 * 160 KiB of a CU), for an operator table without gibbsish_sample_zones: a non-zero weight on it
 * adds 17 * n_sites bytes of scratch, which sbz_mh_run_device checks (SBZ_EINVAL beyond the 160 KiB). */
uint64_t sbz_mh_lds_bytes(const sbz_dims *dims);

#ifdef __cplusplus
}
#endif

#endif /* SBZ_H */
