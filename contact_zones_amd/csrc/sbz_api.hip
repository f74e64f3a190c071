// sbz_api.hip — C-ABI entry points of include/sbz.h (context, memory, likelihood).
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "sbz_internal.h"

#define SBZ_VERSION "sbz 0.1.0 (gfx950)"

namespace sbz {

int fail(sbz_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int hip_fail(sbz_ctx *ctx, hipError_t e, const char *what) {
    return fail(ctx, SBZ_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(sbz_ctx *ctx, DevBuf &buf, size_t bytes) {
    if (buf.bytes >= bytes && buf.ptr) return SBZ_OK;
    if (buf.ptr) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(buf.ptr);
        buf.ptr = nullptr;
        buf.bytes = 0;
    }
    const size_t want = std::max<size_t>(bytes, 256);
    hipError_t e = hipMalloc(&buf.ptr, want);
    if (e != hipSuccess) {
        buf.ptr = nullptr;
        return fail(ctx, SBZ_ENOMEM, std::string("hipMalloc(") + std::to_string(want) +
                                         "): " + hipGetErrorString(e));
    }
    buf.bytes = want;
    return SBZ_OK;
}

static void free_buf(DevBuf &b) {
    if (b.ptr) (void)hipFree(b.ptr);
    b.ptr = nullptr;
    b.bytes = 0;
}

static int check_dims(sbz_ctx *ctx, const sbz_dims *d) {
    if (!d) return fail(ctx, SBZ_EINVAL, "dims is NULL");
    if (d->n_sites <= 0 || d->n_features <= 0)
        return fail(ctx, SBZ_EINVAL, "n_sites and n_features must be positive");
    if (d->n_states < 1 || d->n_states > 127)
        return fail(ctx, SBZ_EINVAL, "n_states must be in 1..127");
    if ((size_t)d->n_sites * d->n_features > (size_t)1 << 31)
        return fail(ctx, SBZ_EINVAL, "n_sites * n_features must be < 2^31");
    if (d->n_zones < 0 || d->n_zones > 254) return fail(ctx, SBZ_EINVAL, "n_zones must be in 0..254");
    if (d->n_families < 0 || d->n_families > 254)
        return fail(ctx, SBZ_EINVAL, "n_families must be in 0..254");
    return SBZ_OK;
}

}  // namespace sbz

using namespace sbz;

extern "C" {

const char *sbz_version(void) { return SBZ_VERSION; }

int sbz_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *sbz_last_error(const sbz_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int sbz_open(int device, const sbz_dims *dims, const int8_t *obs, const uint8_t *fam_of_site,
             sbz_ctx **out) {
    if (!out) return SBZ_EINVAL;
    *out = nullptr;
    sbz_ctx *ctx = new (std::nothrow) sbz_ctx();
    if (!ctx) return SBZ_ENOMEM;
    int rc = check_dims(ctx, dims);
    if (rc) {
        delete ctx;
        return rc;
    }
    if (!obs) {
        delete ctx;
        return SBZ_EINVAL;
    }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete ctx;
        return SBZ_EHIP;
    }
    ctx->device = device;
    ctx->d = *dims;
    if (hipDeviceGetAttribute(&ctx->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        ctx->n_cu <= 0)
        ctx->n_cu = 256;
    const bool inh = (dims->flags & SBZ_INHERITANCE) != 0;
    ctx->C = inh ? 3 : 2;
    ctx->FamC = inh ? dims->n_families + 1 : 1;
    ctx->spl = sites_per_lane(dims->n_sites);
    {
        const int chunk = 64 * ctx->spl;
        ctx->Np = (dims->n_sites + chunk - 1) / chunk * chunk;
    }
    ctx->xs8 = (dims->n_states + 1) * 8 <= 256 ? 1 : 0;
    e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return SBZ_EHIP;
    }
    ctx->stream = ctx->own_stream;

    const int N = dims->n_sites, F = dims->n_features, S = dims->n_states, Np = ctx->Np;
    // family class of each site; validate the families
    std::vector<uint8_t> famc_site(N, 0);
    if (inh && fam_of_site) {
        for (int s = 0; s < N; s++) {
            const int fam = fam_of_site[s];
            if (fam != SBZ_NONE && fam >= dims->n_families) {
                sbz_close(ctx);
                return SBZ_EINVAL;
            }
            famc_site[s] = fam == SBZ_NONE ? 0 : (uint8_t)(fam + 1);
        }
    }
    // family-sorted site order (stable): position p holds site perm[p]
    std::vector<int> perm(Np, 0);
    for (int s = 0; s < N; s++) perm[s] = s;
    std::stable_sort(perm.begin(), perm.begin() + N,
                     [&](int x, int y) { return famc_site[x] < famc_site[y]; });
    std::vector<uint8_t> famc(Np, 0);
    for (int p = 0; p < N; p++) famc[p] = famc_site[perm[p]];
    // obs -> feature-major [F][Np] by position, x in 0..S (S = NA) stored as x*8 when it fits a
    // byte; padded positions hold 0.  Validate the states.
    std::vector<uint8_t> obs_fm((size_t)F * Np, 0);
    const int scale = ctx->xs8 ? 8 : 1;
    for (int p = 0; p < N; p++) {
        const int s = perm[p];
        for (int f = 0; f < F; f++) {
            const int x = obs[(size_t)s * F + f];
            if (x >= S) {
                sbz_close(ctx);
                return SBZ_EINVAL;
            }
            obs_fm[(size_t)f * Np + p] = (uint8_t)((x < 0 ? S : x) * scale);
        }
    }
    ctx->h_perm.assign(perm.begin(), perm.end());
    for (int p = N; p < Np; p++) ctx->h_perm[p] = -1;
    // site-major observations and family classes for the sampler's per-site deltas
    {
        std::vector<uint8_t> obs_sm((size_t)N * F);
        for (size_t i = 0; i < obs_sm.size(); i++) obs_sm[i] = (uint8_t)(obs[i] < 0 ? S : obs[i]);
        if (hipMalloc(&ctx->d_obs_sm, obs_sm.size()) != hipSuccess ||
            hipMalloc(&ctx->d_fam_site, (size_t)N) != hipSuccess ||
            hipMemcpy(ctx->d_obs_sm, obs_sm.data(), obs_sm.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(ctx->d_fam_site, famc_site.data(), (size_t)N, hipMemcpyHostToDevice) != hipSuccess) {
            sbz_close(ctx);
            return SBZ_ENOMEM;
        }
    }
    if (hipMalloc(&ctx->d_obs_fm, obs_fm.size()) != hipSuccess ||
        hipMalloc(&ctx->d_famc, famc.size()) != hipSuccess ||
        hipMalloc(&ctx->d_perm, perm.size() * sizeof(int)) != hipSuccess) {
        sbz_close(ctx);
        return SBZ_ENOMEM;
    }
    if (hipMemcpy(ctx->d_obs_fm, obs_fm.data(), obs_fm.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ctx->d_famc, famc.data(), famc.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ctx->d_perm, perm.data(), perm.size() * sizeof(int), hipMemcpyHostToDevice) !=
            hipSuccess) {
        sbz_close(ctx);
        return SBZ_EHIP;
    }
    // Allow the likelihood kernels their full dynamic LDS table.
    rc = lik_configure(ctx);
    if (rc) {
        sbz_close(ctx);
        return rc;
    }
    *out = ctx;
    return SBZ_OK;
}

void sbz_close(sbz_ctx *ctx) {
    if (!ctx) return;
    if (ctx->own_stream) (void)hipStreamSynchronize(ctx->own_stream);
    if (ctx->stream != ctx->own_stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->d_obs_fm) (void)hipFree(ctx->d_obs_fm);
    if (ctx->d_famc) (void)hipFree(ctx->d_famc);
    if (ctx->d_perm) (void)hipFree(ctx->d_perm);
    for (void *p : {(void *)ctx->d_obs_sm, (void *)ctx->d_fam_site, (void *)ctx->d_adj_ptr,
                    (void *)ctx->d_adj_idx, (void *)ctx->d_app_list, (void *)ctx->d_app_cnt,
                    (void *)ctx->d_alpha_g, (void *)ctx->d_alpha_f, (void *)ctx->d_gc_g,
                    (void *)ctx->d_gc_f, (void *)ctx->d_geo_cost})
        if (p) (void)hipFree(p);
    free_buf(ctx->partial);
    free_buf(ctx->zflag);
    free_buf(ctx->mh_stage);
    free_buf(ctx->src_t);
    free_buf(ctx->src_cand);
    free_buf(ctx->src_ctab);
    free_buf(ctx->ticket);
    free_buf(ctx->stage);
    free_buf(ctx->out);
    free_buf(ctx->flags);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
}

int sbz_set_stream(sbz_ctx *ctx, void *hip_stream) {
    if (!ctx) return SBZ_EINVAL;
    ctx->stream = static_cast<hipStream_t>(hip_stream);
    return SBZ_OK;
}

int sbz_synchronize(sbz_ctx *ctx) {
    if (!ctx) return SBZ_EINVAL;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "hipStreamSynchronize");
}

uint64_t sbz_lik_lds_bytes(const sbz_dims *dims, int source_mode) {
    if (!dims) return 0;
    const size_t b = lik_lds_bytes(*dims, source_mode != 0);
    return b > 160 * 1024 ? 0 : b;
}

int sbz_loglik_batch_device(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w,
                            const double *p_global, const double *p_zones, const double *p_fam,
                            const uint8_t *source, double *out_ll) {
    if (!ctx) return SBZ_EINVAL;
    if (B < 0 || !zone_of_site || !w || !p_global || !out_ll ||
        (ctx->d.n_zones > 0 && !p_zones))
        return fail(ctx, SBZ_EINVAL, "null argument or negative B");
    (void)hipSetDevice(ctx->device);
    return launch_loglik(ctx, B, zone_of_site, w, p_global, p_zones, p_fam, source, false, out_ll);
}

int sbz_loglik_batch_device_pm(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w,
                               const double *p_global, const double *p_zones, const double *p_fam,
                               const uint8_t *source_pm, double *out_ll) {
    if (!ctx) return SBZ_EINVAL;
    if (B < 0 || !zone_of_site || !w || !p_global || !out_ll || !source_pm ||
        (ctx->d.n_zones > 0 && !p_zones))
        return fail(ctx, SBZ_EINVAL, "null argument or negative B");
    (void)hipSetDevice(ctx->device);
    return launch_loglik(ctx, B, zone_of_site, w, p_global, p_zones, p_fam, source_pm, true, out_ll);
}

int sbz_source_layout_device(sbz_ctx *ctx, int B, const uint8_t *src, uint8_t *dst, int32_t to_positions) {
    if (!ctx) return SBZ_EINVAL;
    if (B < 0 || (B > 0 && (!src || !dst)) || src == dst)
        return fail(ctx, SBZ_EINVAL, "sbz_source_layout_device: bad arguments (src and dst must differ)");
    (void)hipSetDevice(ctx->device);
    return launch_source_transpose(ctx, B, src, dst, to_positions != 0);
}

int sbz_site_positions(const sbz_ctx *ctx, int32_t *positions) {
    if (!ctx) return SBZ_EINVAL;
    if (positions)
        for (int p = 0; p < ctx->Np; p++) positions[p] = ctx->h_perm[p];
    return ctx->Np;
}

int sbz_set_option(sbz_ctx *ctx, int32_t option, int64_t value) {
    if (!ctx) return SBZ_EINVAL;
    auto flag = [&](int &dst) -> int {
        if (value != 0 && value != 1) return fail(ctx, SBZ_EINVAL, "option value must be 0 or 1");
        dst = (int)value;
        return SBZ_OK;
    };
    switch (option) {
        case SBZ_OPT_LIK_TASKS_PER_CU:
            if (value < 0 || value > 64) return fail(ctx, SBZ_EINVAL, "tasks per CU must be in 0..64");
            ctx->tasks_per_cu = (int)value;
            return SBZ_OK;
        case SBZ_OPT_LIK_BANKED: return flag(ctx->lik_banked);
        case SBZ_OPT_SRC_TABLE: return flag(ctx->src_rc);
        case SBZ_OPT_SRC_HBM: return flag(ctx->src_hbm);
        case SBZ_OPT_SRC_STAGE: return flag(ctx->src_stage);
        case SBZ_OPT_SRC_PASS_TABLES: return flag(ctx->src_pass_tables);
        case SBZ_OPT_SRC_WAVES:
            if (value != 0 && value != 1 && value != 4 && value != 8)
                return fail(ctx, SBZ_EINVAL, "source-mode sampler waves must be 0, 1, 4 or 8");
            ctx->src_waves = (int)value;
            return SBZ_OK;
        case SBZ_OPT_MH_LOOKAHEAD:
            if (value < 1 || value > 24) return fail(ctx, SBZ_EINVAL, "sampler lookahead must be in 1..24");
            ctx->mh_la = (int)value;
            return SBZ_OK;
        case SBZ_OPT_MH_GROUP:
            if (value < 1 || value > 8) return fail(ctx, SBZ_EINVAL, "sampler move groups must be in 1..8");
            ctx->mh_group = (int)value;
            return SBZ_OK;
        case SBZ_OPT_SRC_PACK: return flag(ctx->src_pack);
        default: return fail(ctx, SBZ_EINVAL, "unknown option " + std::to_string(option));
    }
}

int sbz_get_option(const sbz_ctx *ctx, int32_t option, int64_t *value) {
    if (!ctx || !value) return SBZ_EINVAL;
    switch (option) {
        case SBZ_OPT_LIK_TASKS_PER_CU: *value = ctx->tasks_per_cu; return SBZ_OK;
        case SBZ_OPT_LIK_BANKED: *value = ctx->lik_banked; return SBZ_OK;
        case SBZ_OPT_SRC_TABLE: *value = ctx->src_rc; return SBZ_OK;
        case SBZ_OPT_SRC_HBM: *value = ctx->src_hbm; return SBZ_OK;
        case SBZ_OPT_SRC_STAGE: *value = ctx->src_stage; return SBZ_OK;
        case SBZ_OPT_SRC_WAVES: *value = ctx->src_waves; return SBZ_OK;
        case SBZ_OPT_MH_LOOKAHEAD: *value = ctx->mh_la; return SBZ_OK;
        case SBZ_OPT_SRC_PASS_TABLES: *value = ctx->src_pass_tables; return SBZ_OK;
        case SBZ_OPT_MH_GROUP: *value = ctx->mh_group; return SBZ_OK;
        case SBZ_OPT_SRC_PACK: *value = ctx->src_pack; return SBZ_OK;
        default: return SBZ_EINVAL;
    }
}

namespace {
// bit 0: a zone byte >= n_zones (and != SBZ_NONE); bit 1: a source byte >= C
// (sources by position: rows of Np bytes whose columns >= N are padding, not checked)
__global__ void check_indices_kernel(size_t nz, const uint8_t *zone, int Z, size_t ns,
                                     const uint8_t *src, int C, int N, int row, unsigned *flags) {
    unsigned bad = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nz; i += stride) {
        const unsigned z = zone[i];
        bad |= (z != SBZ_NONE && z >= (unsigned)Z) ? 1u : 0u;
    }
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride)
        bad |= (src[i] >= (unsigned)C && (int)(i % (size_t)row) < N) ? 2u : 0u;
    if (__any(bad != 0)) {
        const unsigned m = bad;
        atomicOr(flags, m);
    }
}
}  // namespace

static int check_indices(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const uint8_t *source,
                         bool pm) {
    if (!ctx) return SBZ_EINVAL;
    if (B < 0 || (B > 0 && !zone_of_site)) return fail(ctx, SBZ_EINVAL, "null argument or negative B");
    if (B == 0) return SBZ_OK;
    (void)hipSetDevice(ctx->device);
    int rc = ensure(ctx, ctx->flags, sizeof(unsigned));
    if (rc) return rc;
    unsigned *flags = static_cast<unsigned *>(ctx->flags.ptr);
    hipError_t e = hipMemsetAsync(flags, 0, sizeof(unsigned), ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipMemsetAsync(flags)");
    const size_t nz = (size_t)B * ctx->d.n_sites;
    const size_t ns = source ? (size_t)B * ctx->d.n_features * (pm ? ctx->Np : ctx->d.n_sites) : 0;
    const size_t work = std::max(nz, ns);
    const int grid = (int)std::min<size_t>(2048, (work + 255) / 256);
    // site-major rows hold F components, all checked (row = N = F would do; use N >= any column)
    const int N = pm ? ctx->d.n_sites : ctx->d.n_features, row = pm ? ctx->Np : ctx->d.n_features;
    check_indices_kernel<<<grid, 256, 0, ctx->stream>>>(nz, zone_of_site, ctx->d.n_zones, ns, source,
                                                        ctx->C, N, row, flags);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "check_indices_kernel launch");
    unsigned h = 0;
    e = hipMemcpyAsync(&h, flags, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "check_indices (read flags)");
    if (h & 1u) return fail(ctx, SBZ_EINVAL, "zone_of_site holds an index >= n_zones");
    if (h & 2u) return fail(ctx, SBZ_EINVAL, "source holds a component index >= C");
    return SBZ_OK;
}

int sbz_check_indices_device(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const uint8_t *source) {
    return check_indices(ctx, B, zone_of_site, source, false);
}

int sbz_check_indices_device_pm(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const uint8_t *source_pm) {
    return check_indices(ctx, B, zone_of_site, source_pm, true);
}

namespace {
int loglik_host(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w, const double *p_global,
                const double *p_zones, const double *p_fam, const uint8_t *source, bool source_pm,
                double *out_ll) {
    if (!ctx) return SBZ_EINVAL;
    if (B < 0 || !zone_of_site || !w || !p_global || !out_ll ||
        (ctx->d.n_zones > 0 && !p_zones))
        return fail(ctx, SBZ_EINVAL, "null argument or negative B");
    if (B == 0) return SBZ_OK;
    (void)hipSetDevice(ctx->device);
    const sbz_dims &d = ctx->d;
    const size_t N = d.n_sites, F = d.n_features, S = d.n_states, Z = d.n_zones,
                 Fam = d.n_families, C = ctx->C;
    const bool inh = C == 3;
    if (inh && Fam > 0 && !p_fam) return fail(ctx, SBZ_EINVAL, "p_fam is required with inheritance");
    // host-side validation of the indices the kernels trust
    for (size_t i = 0; i < (size_t)B * N; i++)
        if (zone_of_site[i] != SBZ_NONE && zone_of_site[i] >= Z)
            return fail(ctx, SBZ_EINVAL, "zone_of_site holds an index >= n_zones");
    const size_t Np = ctx->Np;
    if (source && !source_pm)
        for (size_t i = 0; i < (size_t)B * N * F; i++)
            if (source[i] >= C) return fail(ctx, SBZ_EINVAL, "source holds a component index >= C");
    if (source && source_pm)  // rows of Np bytes; columns >= N are padding, not checked
        for (size_t r = 0; r < (size_t)B * F; r++)
            for (size_t p = 0; p < N; p++)
                if (source[r * Np + p] >= C) return fail(ctx, SBZ_EINVAL, "source holds a component index >= C");

    const size_t bz = B * N, bw = B * F * C * 8, bg = B * F * S * 8, bpz = B * Z * F * S * 8,
                 bpf = inh ? B * Fam * F * S * 8 : 0, bs = source ? B * F * (source_pm ? Np : N) : 0;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_w = 0, o_g = o_w + al(bw), o_z = o_g + al(bg), o_f = o_z + al(bpz),
                 o_zone = o_f + al(bpf), o_src = o_zone + al(bz), total = o_src + al(bs);
    int rc = ensure(ctx, ctx->stage, total);
    if (rc) return rc;
    rc = ensure(ctx, ctx->out, (size_t)B * 8);
    if (rc) return rc;
    char *base = static_cast<char *>(ctx->stage.ptr);
    hipStream_t st = ctx->stream;
    hipError_t e = hipMemcpyAsync(base + o_w, w, bw, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(base + o_g, p_global, bg, hipMemcpyHostToDevice, st);
    if (e == hipSuccess && bpz) e = hipMemcpyAsync(base + o_z, p_zones, bpz, hipMemcpyHostToDevice, st);
    if (e == hipSuccess && bpf) e = hipMemcpyAsync(base + o_f, p_fam, bpf, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(base + o_zone, zone_of_site, bz, hipMemcpyHostToDevice, st);
    if (e == hipSuccess && bs) e = hipMemcpyAsync(base + o_src, source, bs, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipMemcpyAsync H2D");
    rc = launch_loglik(ctx, B, reinterpret_cast<uint8_t *>(base + o_zone),
                       reinterpret_cast<double *>(base + o_w), reinterpret_cast<double *>(base + o_g),
                       reinterpret_cast<double *>(base + o_z),
                       inh ? reinterpret_cast<double *>(base + o_f) : nullptr,
                       source ? reinterpret_cast<uint8_t *>(base + o_src) : nullptr, source_pm,
                       static_cast<double *>(ctx->out.ptr));
    if (rc) return rc;
    e = hipMemcpyAsync(out_ll, ctx->out.ptr, (size_t)B * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(ctx, e, "likelihood D2H");
    return SBZ_OK;
}
}  // namespace

int sbz_loglik_batch(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w,
                     const double *p_global, const double *p_zones, const double *p_fam,
                     const uint8_t *source, double *out_ll) {
    return loglik_host(ctx, B, zone_of_site, w, p_global, p_zones, p_fam, source, false, out_ll);
}

int sbz_loglik_batch_pm(sbz_ctx *ctx, int B, const uint8_t *zone_of_site, const double *w,
                        const double *p_global, const double *p_zones, const double *p_fam,
                        const uint8_t *source_pm, double *out_ll) {
    if (ctx && !source_pm) return fail(ctx, SBZ_EINVAL, "source_pm is required");
    return loglik_host(ctx, B, zone_of_site, w, p_global, p_zones, p_fam, source_pm, true, out_ll);
}

int sbz_set_network(sbz_ctx *ctx, const uint8_t *applicable, int32_t nnz, const int32_t *adj_indptr,
                    const int32_t *adj_indices) {
    if (!ctx) return SBZ_EINVAL;
    const int N = ctx->d.n_sites, F = ctx->d.n_features, S = ctx->d.n_states;
    if (!applicable || !adj_indptr || (nnz > 0 && !adj_indices) || nnz < 0)
        return fail(ctx, SBZ_EINVAL, "null network argument");
    if (adj_indptr[0] != 0 || adj_indptr[N] != nnz)
        return fail(ctx, SBZ_EINVAL, "adj_indptr must start at 0 and end at nnz");
    for (int s = 0; s < N; s++)
        if (adj_indptr[s + 1] < adj_indptr[s]) return fail(ctx, SBZ_EINVAL, "adj_indptr not monotone");
    for (int i = 0; i < nnz; i++)
        if (adj_indices[i] < 0 || adj_indices[i] >= N)
            return fail(ctx, SBZ_EINVAL, "adjacency index out of range");
    std::vector<int> list((size_t)F * S, 0), cnt(F, 0);
    for (int f = 0; f < F; f++)
        for (int x = 0; x < S; x++)
            if (applicable[(size_t)f * S + x]) list[(size_t)f * S + cnt[f]++] = x;
    (void)hipSetDevice(ctx->device);
    for (void *p : {(void *)ctx->d_adj_ptr, (void *)ctx->d_adj_idx, (void *)ctx->d_app_list,
                    (void *)ctx->d_app_cnt})
        if (p) (void)hipFree(p);
    ctx->d_adj_ptr = ctx->d_adj_idx = ctx->d_app_list = ctx->d_app_cnt = nullptr;
    const size_t bp = (size_t)(N + 1) * 4, bi = (size_t)std::max(nnz, 1) * 4;
    if (hipMalloc(&ctx->d_adj_ptr, bp) != hipSuccess || hipMalloc(&ctx->d_adj_idx, bi) != hipSuccess ||
        hipMalloc(&ctx->d_app_list, list.size() * 4) != hipSuccess ||
        hipMalloc(&ctx->d_app_cnt, cnt.size() * 4) != hipSuccess)
        return fail(ctx, SBZ_ENOMEM, "network allocation failed");
    hipError_t e = hipMemcpy(ctx->d_adj_ptr, adj_indptr, bp, hipMemcpyHostToDevice);
    if (e == hipSuccess && nnz > 0)
        e = hipMemcpy(ctx->d_adj_idx, adj_indices, (size_t)nnz * 4, hipMemcpyHostToDevice);
    ctx->adj_nnz = nnz;
    if (e == hipSuccess) e = hipMemcpy(ctx->d_app_list, list.data(), list.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(ctx->d_app_cnt, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice);
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "network upload");
}

int sbz_set_priors(sbz_ctx *ctx, const double *alpha_global, const double *alpha_fam,
                   int32_t size_prior) {
    if (!ctx) return SBZ_EINVAL;
    if (size_prior < 0 || size_prior > 2) return fail(ctx, SBZ_EINVAL, "size_prior must be 0, 1 or 2");
    if (alpha_fam && (ctx->C != 3 || ctx->d.n_families == 0))
        return fail(ctx, SBZ_EINVAL, "alpha_fam needs inheritance with families");
    const size_t fs = (size_t)ctx->d.n_features * ctx->d.n_states;
    (void)hipSetDevice(ctx->device);
    for (double **pp : {&ctx->d_alpha_g, &ctx->d_alpha_f}) {
        if (*pp) (void)hipFree(*pp);
        *pp = nullptr;
    }
    auto upload = [&](const double *src, size_t n, double **dst) -> int {
        if (!src) return SBZ_OK;
        for (size_t i = 0; i < n; i++)
            if (!(src[i] >= 0.0) || std::isinf(src[i]))
                return fail(ctx, SBZ_EINVAL, "prior concentrations must be finite and >= 0");
        if (hipMalloc(dst, n * sizeof(double)) != hipSuccess)
            return fail(ctx, SBZ_ENOMEM, "prior allocation failed");
        hipError_t e = hipMemcpy(*dst, src, n * sizeof(double), hipMemcpyHostToDevice);
        return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "prior upload");
    };
    int rc = upload(alpha_global, fs, &ctx->d_alpha_g);
    if (rc == SBZ_OK) rc = upload(alpha_fam, (size_t)ctx->d.n_families * fs, &ctx->d_alpha_f);
    if (rc == SBZ_OK) ctx->size_prior = size_prior;
    return rc;
}

int sbz_set_geo_prior(sbz_ctx *ctx, const double *cost, double scale) {
    if (!ctx) return SBZ_EINVAL;
    (void)hipSetDevice(ctx->device);
    if (ctx->d_geo_cost) (void)hipFree(ctx->d_geo_cost);
    ctx->d_geo_cost = nullptr;
    ctx->geo_scale = 0.0;
    if (!cost) return SBZ_OK;
    if (!(scale > 0.0) || std::isinf(scale)) return fail(ctx, SBZ_EINVAL, "geo prior scale must be finite and > 0");
    const size_t n = (size_t)ctx->d.n_sites * ctx->d.n_sites;
    for (size_t i = 0; i < n; i++)
        if (!(cost[i] >= 0.0) || std::isnan(cost[i]))
            return fail(ctx, SBZ_EINVAL, "geo prior costs must be >= 0 (inf: no edge)");
    if (hipMalloc(&ctx->d_geo_cost, n * sizeof(double)) != hipSuccess)
        return fail(ctx, SBZ_ENOMEM, "geo prior allocation failed");
    hipError_t e = hipMemcpy(ctx->d_geo_cost, cost, n * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(ctx, e, "geo prior upload");
    ctx->geo_scale = scale;
    return SBZ_OK;
}

int sbz_set_gibbs_counts(sbz_ctx *ctx, const double *counts_global, const double *counts_fam) {
    if (!ctx) return SBZ_EINVAL;
    if (counts_fam && (ctx->C != 3 || ctx->d.n_families == 0))
        return fail(ctx, SBZ_EINVAL, "counts_fam needs inheritance with families");
    const size_t fs = (size_t)ctx->d.n_features * ctx->d.n_states;
    (void)hipSetDevice(ctx->device);
    for (double **pp : {&ctx->d_gc_g, &ctx->d_gc_f}) {
        if (*pp) (void)hipFree(*pp);
        *pp = nullptr;
    }
    auto upload = [&](const double *src, size_t n, double **dst) -> int {
        if (!src) return SBZ_OK;
        for (size_t i = 0; i < n; i++)
            if (!(src[i] >= 0.0) || std::isinf(src[i]))
                return fail(ctx, SBZ_EINVAL, "Gibbs prior counts must be finite and >= 0");
        if (hipMalloc(dst, n * sizeof(double)) != hipSuccess)
            return fail(ctx, SBZ_ENOMEM, "Gibbs counts allocation failed");
        hipError_t e = hipMemcpy(*dst, src, n * sizeof(double), hipMemcpyHostToDevice);
        return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "Gibbs counts upload");
    };
    int rc = upload(counts_global, fs, &ctx->d_gc_g);
    if (rc == SBZ_OK) rc = upload(counts_fam, (size_t)ctx->d.n_families * fs, &ctx->d_gc_f);
    return rc;
}

int sbz_mh_run_device(sbz_ctx *ctx, int B, int n_steps, const sbz_mh_config *cfg,
                      const sbz_chains *chains) {
    if (!ctx) return SBZ_EINVAL;
    if (!cfg || !chains || B < 0 || n_steps < 0) return fail(ctx, SBZ_EINVAL, "bad sampler arguments");
    (void)hipSetDevice(ctx->device);
    return launch_mh(ctx, B, n_steps, cfg, chains);
}

const char *sbz_last_kernels(const sbz_ctx *ctx) { return ctx ? ctx->last_kernels.c_str() : ""; }

int sbz_mh_run(sbz_ctx *ctx, int B, int n_steps, const sbz_mh_config *cfg, uint64_t seed,
               const sbz_tape *tape, sbz_state *st, sbz_trace *tr) {
    if (!ctx) return SBZ_EINVAL;
    if (!cfg || !st || B < 0 || n_steps < 0) return fail(ctx, SBZ_EINVAL, "bad sampler arguments");
    if (B == 0) return SBZ_OK;
    const sbz_dims &d = ctx->d;
    const size_t N = d.n_sites, F = d.n_features, S = d.n_states, Z = d.n_zones, Fam = d.n_families;
    const bool inh = ctx->C == 3, src = cfg->sample_source != 0;
    if (!st->zone_of_site || !st->w || !st->p_global || (Z > 0 && !st->p_zones) || !st->ll ||
        !st->max_size || !st->p_grow_connected || (inh && Fam > 0 && !st->p_fam) || (src && !st->source))
        return fail(ctx, SBZ_EINVAL, "sbz_state: a required array is NULL");
    if (tape && (!tape->values || !tape->len || tape->stride <= 0))
        return fail(ctx, SBZ_EINVAL, "sbz_tape: values, len and stride > 0 are required");
    if (tape)
        for (int b = 0; b < B; b++) {
            const int64_t len = tape->len[b], pos = tape->pos ? tape->pos[b] : 0;
            if (len < 0 || len > tape->stride || pos < 0 || pos > len)
                return fail(ctx, SBZ_EINVAL, "sbz_tape: need 0 <= pos[b] <= len[b] <= stride");
        }
    for (size_t i = 0; i < (size_t)B * N; i++)
        if (st->zone_of_site[i] != SBZ_NONE && st->zone_of_site[i] >= Z)
            return fail(ctx, SBZ_EINVAL, "zone_of_site holds an index >= n_zones");
    if (src)
        for (size_t i = 0; i < (size_t)B * N * F; i++)
            if (st->source[i] >= (unsigned)ctx->C) return fail(ctx, SBZ_EINVAL, "source holds a component index >= C");
    (void)hipSetDevice(ctx->device);
    // one staging buffer: every array at a 256-B aligned offset
    const size_t K = SBZ_N_OPS, T = (size_t)n_steps;
    struct Part { const void *host; size_t bytes; bool in; void *out; size_t off; };
    std::vector<Part> parts;
    auto part = [&](const void *h, size_t bytes, bool in, void *out) {
        parts.push_back({h, bytes, in, out, 0});
        return parts.size() - 1;
    };
    const size_t izos = part(st->zone_of_site, (size_t)B * N, true, st->zone_of_site);
    const size_t iw = part(st->w, (size_t)B * F * ctx->C * 8, true, st->w);
    const size_t ig = part(st->p_global, (size_t)B * F * S * 8, true, st->p_global);
    const size_t iz = part(st->p_zones, (size_t)B * Z * F * S * 8, true, st->p_zones);
    const size_t ifm = part(st->p_fam, inh ? (size_t)B * Fam * F * S * 8 : 0, true, st->p_fam);
    const size_t isrc = part(st->source, src ? (size_t)B * N * F : 0, true, st->source);
    const size_t ill = part(nullptr, (size_t)B * 8, false, st->ll);
    const size_t ipr = part(st->prior, st->prior ? (size_t)B * 8 : 0, true, st->prior);
    const size_t ims = part(st->max_size, (size_t)B * 4, true, nullptr);
    const size_t ipg = part(st->p_grow_connected, (size_t)B * 8, true, nullptr);
    const size_t ictr = part(st->counter, (size_t)B * 8, st->counter != nullptr, st->counter);
    const size_t iacc = part(st->accepted, (size_t)B * K * 8, st->accepted != nullptr, st->accepted);
    const size_t iprp = part(st->proposed, (size_t)B * K * 8, st->proposed != nullptr, st->proposed);
    const size_t ista = part(nullptr, (size_t)B * 4, false, st->status);
    const size_t itv = part(tape ? tape->values : nullptr, tape ? (size_t)B * tape->stride * 8 : 0, true, nullptr);
    const size_t itl = part(tape ? tape->len : nullptr, tape ? (size_t)B * 8 : 0, true, nullptr);
    const size_t itp = part(tape ? tape->pos : nullptr, tape ? (size_t)B * 8 : 0, tape && tape->pos, tape ? tape->pos : nullptr);
    const bool trace = tr && tr->op && tr->accept && tr->ll;
    const size_t iop = part(nullptr, trace ? (size_t)B * T : 0, false, trace ? tr->op : nullptr);
    const size_t iac = part(nullptr, trace ? (size_t)B * T : 0, false, trace ? tr->accept : nullptr);
    const size_t itll = part(nullptr, trace ? (size_t)B * T * 8 : 0, false, trace ? tr->ll : nullptr);
    size_t total = 0;
    for (Part &p : parts) {
        p.off = total;
        total += (p.bytes + 255) & ~(size_t)255;
    }
    int rc = ensure(ctx, ctx->mh_stage, total);
    if (rc) return rc;
    char *base = static_cast<char *>(ctx->mh_stage.ptr);
    hipStream_t s = ctx->stream;
    hipError_t e = hipMemsetAsync(base, 0, total, s);  // counters / cursors / outputs start at 0
    for (const Part &p : parts)
        if (e == hipSuccess && p.in && p.host && p.bytes)
            e = hipMemcpyAsync(base + p.off, p.host, p.bytes, hipMemcpyHostToDevice, s);
    // from here on the H2D copies from the caller's (pageable) arrays may be in flight: an error
    // return first waits for them, so the caller may free its arrays
    auto bail = [&](int code) {
        (void)hipStreamSynchronize(s);
        return code;
    };
    if (e != hipSuccess) return bail(hip_fail(ctx, e, "sbz_mh_run: H2D"));
    auto dp = [&](size_t i) -> void * { return parts[i].bytes ? base + parts[i].off : nullptr; };
    // the chains' log-likelihood from the staged state
    rc = launch_loglik(ctx, B, static_cast<uint8_t *>(dp(izos)), static_cast<double *>(dp(iw)),
                       static_cast<double *>(dp(ig)), static_cast<double *>(dp(iz)),
                       static_cast<double *>(dp(ifm)), src ? static_cast<uint8_t *>(dp(isrc)) : nullptr, false,
                       static_cast<double *>(dp(ill)));
    if (rc) return bail(rc);
    sbz_chains ch{};
    ch.zone_of_site = static_cast<uint8_t *>(dp(izos));
    ch.w = static_cast<double *>(dp(iw));
    ch.p_global = static_cast<double *>(dp(ig));
    ch.p_zones = static_cast<double *>(dp(iz));
    ch.p_fam = static_cast<double *>(dp(ifm));
    ch.source = src ? static_cast<uint8_t *>(dp(isrc)) : nullptr;
    ch.ll = static_cast<double *>(dp(ill));
    ch.prior = static_cast<double *>(dp(ipr));
    ch.max_size = static_cast<const int32_t *>(dp(ims));
    ch.p_grow_connected = static_cast<const double *>(dp(ipg));
    ch.seed = seed;
    ch.chain_id0 = st->chain_id0;
    ch.counter = static_cast<uint64_t *>(dp(ictr));
    ch.accepted = static_cast<int64_t *>(dp(iacc));
    ch.proposed = static_cast<int64_t *>(dp(iprp));
    ch.status = static_cast<int32_t *>(dp(ista));
    if (tape) {
        ch.tape = static_cast<const double *>(dp(itv));
        ch.tape_stride = tape->stride;
        ch.tape_len = static_cast<const int64_t *>(dp(itl));
        ch.tape_pos = static_cast<int64_t *>(dp(itp));
    }
    if (trace) {
        ch.trace_op = static_cast<int8_t *>(dp(iop));
        ch.trace_accept = static_cast<uint8_t *>(dp(iac));
        ch.trace_ll = static_cast<double *>(dp(itll));
    }
    rc = launch_mh(ctx, B, n_steps, cfg, &ch);
    if (rc) return bail(rc);
    for (const Part &p : parts)
        if (e == hipSuccess && p.out && p.bytes)
            e = hipMemcpyAsync(p.out, base + p.off, p.bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "sbz_mh_run: D2H");
}

int sbz_draw_gamma(sbz_ctx *ctx, int32_t n, const double *alpha, uint64_t seed, double *out) {
    if (!ctx) return SBZ_EINVAL;
    if (n < 0 || (n > 0 && (!alpha || !out))) return fail(ctx, SBZ_EINVAL, "sbz_draw_gamma: bad arguments");
    for (int i = 0; i < n; i++)
        if (!(alpha[i] > 0.0) || !std::isfinite(alpha[i])) return fail(ctx, SBZ_EINVAL, "sbz_draw_gamma: alpha must be finite and > 0");
    if (n == 0) return SBZ_OK;
    (void)hipSetDevice(ctx->device);
    const size_t bytes = (size_t)n * sizeof(double);
    int rc = ensure(ctx, ctx->mh_stage, 2 * bytes);
    if (rc) return rc;
    double *d_alpha = static_cast<double *>(ctx->mh_stage.ptr), *d_out = d_alpha + n;
    hipError_t e = hipMemcpyAsync(d_alpha, alpha, bytes, hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "sbz_draw_gamma: H2D");
    rc = launch_draw_gamma(ctx, n, d_alpha, seed, d_out);
    if (rc) return rc;
    e = hipMemcpyAsync(out, d_out, bytes, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "sbz_draw_gamma: D2H");
}

uint64_t sbz_mh_lds_bytes(const sbz_dims *dims) {
    if (!dims) return 0;
    const size_t b = mh_lds_bytes(*dims, (dims->flags & SBZ_INHERITANCE) ? 3 : 2);
    return b > 160 * 1024 ? 0 : b;
}

int sbz_device_alloc(sbz_ctx *ctx, uint64_t bytes, void **out) {
    if (!ctx || !out) return SBZ_EINVAL;
    (void)hipSetDevice(ctx->device);
    hipError_t e = hipMalloc(out, std::max<uint64_t>(bytes, 1));
    return e == hipSuccess ? SBZ_OK : fail(ctx, SBZ_ENOMEM, hipGetErrorString(e));
}

int sbz_device_free(sbz_ctx *ctx, void *ptr) {
    if (!ctx) return SBZ_EINVAL;
    hipError_t e = hipFree(ptr);
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "hipFree");
}

int sbz_memcpy_h2d(sbz_ctx *ctx, void *dst, const void *src, uint64_t bytes) {
    if (!ctx) return SBZ_EINVAL;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "h2d");
}

int sbz_memcpy_d2h(sbz_ctx *ctx, void *dst, const void *src, uint64_t bytes) {
    if (!ctx) return SBZ_EINVAL;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? SBZ_OK : hip_fail(ctx, e, "d2h");
}

}  // extern "C"
