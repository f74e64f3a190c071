// sbz_lik.hip — batched full log-likelihood kernels for CDNA4 (gfx950).
//
// Computes, for each of B chains, the reference Likelihood.__call__(sample, caching=False)
// (sbayes/model.py:145-171):
//   mixture : sum_{s,f} log( (w0*l0 + w1*l1) + w2*l2 )          combine_lh  model.py:174-176
//   source  : sum_{s,f} log( w_src * l_src ), -inf on w_src == 0  combine_lh  model.py:177-184
// with l_c the one-hot gathers of p_global / p_zones / p_families (model.py:297-433), NA -> 1
// (model.py:247) and w_c = w[f,c]*has[s,c] / ((w0*h0 + w1*h1) + w2*h2) (model.py:436-452).
//
// Design (memory-bound gather-reduce; no MFMA):
//   * grid = (feature tile t, chain b); one 256-thread workgroup per (b, t), FT = 16 features.
//   * Every cell value depends only on (site class, f, x), class = (zone or none) x (family or
//     none).  The workgroup stages the chain's parameters for its tile into an LDS table
//     T[class][f][x] (x = S is the NA column, padded features hold 1.0), computed with the
//     reference's operation order (no FMA contraction: built with -ffp-contract=off), so each
//     table entry is bit-identical to the reference's per-cell value.
//   * Sites stream through: one coalesced 16-byte load of the site's packed observations per
//     tile, 16 LDS gathers.  Instead of one fp64 log per cell the lanes multiply the cells
//     into a mantissa/exponent accumulator (v_frexp every 4 factors) and take ONE log per lane:
//     sum log(c_i) = log(prod c_i) within ~1e-16 relative.  A table entry outside
//     [2^-240, 2^240] (or negative / NaN) flips the workgroup to a per-cell log path, so
//     the product can never under/overflow.
//   * One fp64 partial per (b, t); a second tiny kernel sums the T partials of each chain in
//     fixed order (deterministic).
#include <cmath>

#include "sbz_internal.h"

namespace sbz {

namespace {

constexpr double LN2 = 0.69314718055994530941723212145818;

__device__ __forceinline__ bool safe_factor(double v) {
    return v == 0.0 || (v >= 0x1p-240 && v <= 0x1p240);
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

// LDS carve (bytes): [0,16) flag, [16, 16+8*8) wave partials, then nw[4][FT][4], then tables.
constexpr int LDS_FLAG = 0;
constexpr int LDS_RED = 16;
constexpr int LDS_NW = 16 + 8 * 8;
constexpr int LDS_TAB = LDS_NW + 4 * FT * 4 * 8;

// Normalised weights for the 4 (has_zone, has_family) classes of every feature in the tile.
// normalize_weights (model.py:451-452): w*has / sum_c(w*has), sum in component order.
template <int C>
__device__ __forceinline__ void build_nw(const LikArgs &a, int b, int f0, double *nw) {
    const int tid = threadIdx.x;
    if (tid < 4 * FT) {
        const int h = tid / FT, f = tid % FT, gf = f0 + f;
        const double hz = (h & 1) ? 1.0 : 0.0;
        const double hf = (h & 2) ? 1.0 : 0.0;
        double n0 = 0.0, n1 = 0.0, n2 = 0.0;
        if (gf < a.F) {
            const double *wr = a.w + ((size_t)b * a.F + gf) * C;
            const double w0 = wr[0] * 1.0;
            const double w1 = wr[1] * hz;
            double s = w0 + w1;
            double w2 = 0.0;
            if (C == 3) {
                w2 = wr[2] * hf;
                s = s + w2;
            }
            n0 = w0 / s;
            n1 = w1 / s;
            if (C == 3) n2 = w2 / s;
        }
        double *o = nw + (h * FT + f) * 4;
        o[0] = n0;
        o[1] = n1;
        o[2] = n2;
        o[3] = 0.0;
    }
}

__device__ __forceinline__ double block_reduce_store(double v, double *red, double *dst) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
        for (int i = 0; i < LIK_BLOCK / 64; i++) r += red[i];
        *dst = r;
    }
    return r;
}

// ---------------------------------------------------------------------------------------
// Mixture branch.
// Table T[cls][f][x], cls = zc * FamC + fc, zc = 0 (no zone) | z+1, fc = 0 (no family) | fam+1.
// ---------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(LIK_BLOCK) void lik_mixture_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    int *flag = reinterpret_cast<int *>(lds + LDS_FLAG);
    double *red = reinterpret_cast<double *>(lds + LDS_RED);
    double *nw = reinterpret_cast<double *>(lds + LDS_NW);
    double *tab = reinterpret_cast<double *>(lds + LDS_TAB);

    const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int f0 = t * FT;
    const int S = a.S, S1 = a.S + 1;
    const int per_cls = FT * S1;

    if (tid == 0) *flag = 0;
    build_nw<C>(a, b, f0, nw);
    __syncthreads();

    const double *pgb = a.pg + (size_t)b * a.F * S;
    const double *pzb = a.pz + (size_t)b * a.Z * a.F * S;
    const double *pfb = (C == 3) ? a.pf + (size_t)b * a.Fam * a.F * S : nullptr;

    // Build the table: one (class, feature) row per thread iteration, x innermost.
    const int ncls = (a.Z + 1) * a.FamC;
    int bad = 0;
    for (int p = tid; p < ncls * FT; p += LIK_BLOCK) {
        const int cls = p / FT, f = p % FT, gf = f0 + f;
        double *row = tab + (size_t)cls * per_cls + f * S1;
        if (gf >= a.F) {
            for (int x = 0; x < S1; x++) row[x] = 1.0;
            continue;
        }
        const int zc = cls / a.FamC, fc = cls - zc * a.FamC;
        const int h = (zc > 0 ? 1 : 0) | (fc > 0 ? 2 : 0);
        const double n0 = nw[(h * FT + f) * 4 + 0];
        const double n1 = nw[(h * FT + f) * 4 + 1];
        const double n2 = nw[(h * FT + f) * 4 + 2];
        const double *g = pgb + (size_t)gf * S;
        const double *zr = zc > 0 ? pzb + ((size_t)(zc - 1) * a.F + gf) * S : nullptr;
        const double *fr = (C == 3 && fc > 0) ? pfb + ((size_t)(fc - 1) * a.F + gf) * S : nullptr;
        for (int x = 0; x <= S; x++) {
            const bool na = (x == S);
            const double l0 = na ? 1.0 : g[x];
            const double l1 = na ? 1.0 : (zr ? zr[x] : 0.0);
            double v = n0 * l0 + n1 * l1;
            if (C == 3) {
                const double l2 = na ? 1.0 : (fr ? fr[x] : 0.0);
                v = v + n2 * l2;
            }
            bad |= !safe_factor(v);
            row[x] = v;
        }
    }
    if (bad) atomicOr(flag, 1);
    __syncthreads();
    const bool slow = *flag != 0;

    const uint8_t *zb = a.zone + (size_t)b * a.N;
    const uint4 *ob = reinterpret_cast<const uint4 *>(a.obs_t + (size_t)t * a.N * FT);
    double m = 1.0, lsum = 0.0;
    int e = 0;
    for (int s = tid; s < a.N; s += LIK_BLOCK) {
        const int z = zb[s];
        const int zc = (z < a.Z) ? z + 1 : 0;
        const double *tb = tab + (size_t)(zc * a.FamC + a.famc[s]) * per_cls;
        const uint4 o = ob[s];
        const uint32_t wd[4] = {o.x, o.y, o.z, o.w};
        if (!slow) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int x = (wd[q] >> (8 * k)) & 0xff;
                    m *= tb[(q * 4 + k) * S1 + x];
                }
                renorm(m, e);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int x = (wd[q] >> (8 * k)) & 0xff;
                    lsum += log(tb[(q * 4 + k) * S1 + x]);
                }
        }
    }
    const double v = slow ? lsum : (log(m) + (double)e * LN2);
    block_reduce_store(v, red, a.partial + (size_t)b * a.T + t);
}

// ---------------------------------------------------------------------------------------
// Source branch: cell = w_norm[src] * l_src.  Per-component tables:
//   T0[h][f][x]          h = hz | hf<<1                   w_norm[h][f][0] * l0
//   T1[z][hf][f][x]      (has_zone = 1)                   w_norm[1|hf<<1][f][1] * l1
//   T2[fam][hz][f][x]    (has_family = 1)                 w_norm[hz|2][f][2] * l2
//   Z0[f][x]             a selected component the site lacks: weight 0 -> cell 0 -> -inf
// ---------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(LIK_BLOCK) void lik_source_kernel(LikArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    int *flag = reinterpret_cast<int *>(lds + LDS_FLAG);
    double *red = reinterpret_cast<double *>(lds + LDS_RED);
    double *nw = reinterpret_cast<double *>(lds + LDS_NW);
    double *tab = reinterpret_cast<double *>(lds + LDS_TAB);

    const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int f0 = t * FT;
    const int S = a.S, S1 = a.S + 1;
    const int per = FT * S1;
    const int Famx = (C == 3) ? a.Fam : 0;
    const int off1 = 4, off2 = 4 + 2 * a.Z, offz = 4 + 2 * a.Z + 2 * Famx;
    const int nrows = offz + 1;

    if (tid == 0) *flag = 0;
    build_nw<C>(a, b, f0, nw);
    __syncthreads();

    const double *pgb = a.pg + (size_t)b * a.F * S;
    const double *pzb = a.pz + (size_t)b * a.Z * a.F * S;
    const double *pfb = (C == 3) ? a.pf + (size_t)b * a.Fam * a.F * S : nullptr;

    int bad = 0;
    for (int p = tid; p < nrows * FT; p += LIK_BLOCK) {
        const int k = p / FT, f = p % FT, gf = f0 + f;
        double *row = tab + (size_t)k * per + f * S1;
        if (gf >= a.F) {
            for (int x = 0; x < S1; x++) row[x] = 1.0;
            continue;
        }
        double n;
        const double *pr;
        if (k < off1) {
            n = nw[(k * FT + f) * 4 + 0];
            pr = pgb + (size_t)gf * S;
        } else if (k < off2) {
            const int j = k - off1, z = j >> 1, hf = j & 1;
            n = nw[(((1 | (hf << 1))) * FT + f) * 4 + 1];
            pr = pzb + ((size_t)z * a.F + gf) * S;
        } else if (k < offz) {
            const int j = k - off2, fam = j >> 1, hz = j & 1;
            n = nw[((hz | 2) * FT + f) * 4 + 2];
            pr = pfb + ((size_t)fam * a.F + gf) * S;
        } else {
            for (int x = 0; x < S1; x++) row[x] = 0.0;
            continue;
        }
        for (int x = 0; x <= S; x++) {
            const double l = (x == S) ? 1.0 : pr[x];
            const double v = n * l;
            bad |= !safe_factor(v);
            row[x] = v;
        }
    }
    if (bad) atomicOr(flag, 1);
    __syncthreads();
    const bool slow = *flag != 0;

    const uint8_t *zb = a.zone + (size_t)b * a.N;
    const uint4 *ob = reinterpret_cast<const uint4 *>(a.obs_t + (size_t)t * a.N * FT);
    const uint4 *sb = reinterpret_cast<const uint4 *>(a.src_t + ((size_t)b * a.T + t) * a.N * FT);
    double m = 1.0, lsum = 0.0;
    int e = 0;
    for (int s = tid; s < a.N; s += LIK_BLOCK) {
        const int z = zb[s];
        const bool hz = z < a.Z;
        const int fc = a.famc[s];
        const bool hf = fc > 0;
        const int h = (hz ? 1 : 0) | (hf ? 2 : 0);
        const int o0 = h * per;
        const int o1 = hz ? (off1 + 2 * z + (hf ? 1 : 0)) * per : offz * per;
        const int o2 = hf ? (off2 + 2 * (fc - 1) + (hz ? 1 : 0)) * per : offz * per;
        const int oz = offz * per;
        const uint4 o = ob[s];
        const uint4 c4 = sb[s];
        const uint32_t wd[4] = {o.x, o.y, o.z, o.w};
        const uint32_t cd[4] = {c4.x, c4.y, c4.z, c4.w};
        auto cell = [&](int q, int k) -> double {
            const int x = (wd[q] >> (8 * k)) & 0xff;
            const int c = (cd[q] >> (8 * k)) & 0xff;
            const int base = (c == 0) ? o0 : (c == 1 ? o1 : ((C == 3 && c == 2) ? o2 : oz));
            return tab[base + (q * 4 + k) * S1 + x];
        };
        if (!slow) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
#pragma unroll
                for (int k = 0; k < 4; k++) m *= cell(q, k);
                renorm(m, e);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int k = 0; k < 4; k++) lsum += log(cell(q, k));
        }
    }
    const double v = slow ? lsum : (log(m) + (double)e * LN2);
    block_reduce_store(v, red, a.partial + (size_t)b * a.T + t);
}

// Sum the T tile partials of each chain in tile order (deterministic).
__global__ void lik_reduce_kernel(int B, int T, const double *partial, double *out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double s = 0.0;
    for (int t = 0; t < T; t++) s += partial[(size_t)b * T + t];
    out[b] = s;
}

// Row-major source [B][N][F] -> tiled [B][T][N][FT] (padded features -> component 0).
__global__ void repack_source_kernel(int B, int N, int F, int T, const uint8_t *src,
                                     uint8_t *dst) {
    const size_t total = (size_t)B * T * N * FT;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int f = (int)(i % FT);
        size_t r = i / FT;
        const int s = (int)(r % N);
        r /= N;
        const int t = (int)(r % T);
        const int b = (int)(r / T);
        const int gf = t * FT + f;
        dst[i] = gf < F ? src[((size_t)b * N + s) * F + gf] : 0;
    }
}

}  // namespace

size_t lik_lds_bytes(const sbz_dims &d, bool source_mode) {
    const bool inh = (d.flags & SBZ_INHERITANCE) != 0;
    const size_t S1 = (size_t)d.n_states + 1;
    size_t rows;
    if (!source_mode) {
        rows = (size_t)(d.n_zones + 1) * (inh ? (size_t)d.n_families + 1 : 1);
    } else {
        rows = 4 + 2 * (size_t)d.n_zones + (inh ? 2 * (size_t)d.n_families : 0) + 1;
    }
    return LDS_TAB + rows * FT * S1 * sizeof(double);
}

int lik_configure(sbz_ctx *ctx) {
    const int lim = 160 * 1024;
    const void *fns[] = {
        reinterpret_cast<const void *>(&lik_mixture_kernel<2>),
        reinterpret_cast<const void *>(&lik_mixture_kernel<3>),
        reinterpret_cast<const void *>(&lik_source_kernel<2>),
        reinterpret_cast<const void *>(&lik_source_kernel<3>),
    };
    for (const void *fn : fns) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
    }
    return SBZ_OK;
}

int launch_loglik(sbz_ctx *ctx, int B, const uint8_t *zone, const double *w, const double *pg,
                  const double *pz, const double *pf, const uint8_t *source, double *out_ll) {
    const sbz_dims &d = ctx->d;
    const bool src_mode = source != nullptr;
    const size_t lds = lik_lds_bytes(d, src_mode);
    if (lds > 160 * 1024)
        return fail(ctx, SBZ_EINVAL, "likelihood table needs " + std::to_string(lds) +
                                         " B of LDS (> 160 KiB): too many zones x families x states");
    if (ctx->C == 3 && d.n_families > 0 && pf == nullptr)
        return fail(ctx, SBZ_EINVAL, "p_fam is required with inheritance");
    if (B <= 0) return SBZ_OK;

    int rc = ensure(ctx, ctx->partial, (size_t)B * ctx->T * sizeof(double));
    if (rc) return rc;

    LikArgs a{};
    a.N = d.n_sites;
    a.F = d.n_features;
    a.S = d.n_states;
    a.Z = d.n_zones;
    a.Fam = d.n_families;
    a.C = ctx->C;
    a.FamC = ctx->FamC;
    a.T = ctx->T;
    a.B = B;
    a.obs_t = ctx->d_obs_t;
    a.famc = ctx->d_famc;
    a.zone = zone;
    a.w = w;
    a.pg = pg;
    a.pz = pz;
    a.pf = pf;
    a.partial = static_cast<double *>(ctx->partial.ptr);

    if (src_mode) {
        rc = ensure(ctx, ctx->src_t, (size_t)B * ctx->T * d.n_sites * FT);
        if (rc) return rc;
        const size_t total = (size_t)B * ctx->T * d.n_sites * FT;
        const int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
        repack_source_kernel<<<blocks, 256, 0, ctx->stream>>>(B, d.n_sites, d.n_features, ctx->T,
                                                             source,
                                                             static_cast<uint8_t *>(ctx->src_t.ptr));
        a.src_t = static_cast<const uint8_t *>(ctx->src_t.ptr);
    }

    dim3 grid(ctx->T, B);
    if (!src_mode) {
        if (ctx->C == 3)
            lik_mixture_kernel<3><<<grid, LIK_BLOCK, lds, ctx->stream>>>(a);
        else
            lik_mixture_kernel<2><<<grid, LIK_BLOCK, lds, ctx->stream>>>(a);
    } else {
        if (ctx->C == 3)
            lik_source_kernel<3><<<grid, LIK_BLOCK, lds, ctx->stream>>>(a);
        else
            lik_source_kernel<2><<<grid, LIK_BLOCK, lds, ctx->stream>>>(a);
    }
    lik_reduce_kernel<<<(B + 63) / 64, 64, 0, ctx->stream>>>(B, ctx->T, a.partial, out_ll);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "likelihood launch");
    return SBZ_OK;
}

}  // namespace sbz
