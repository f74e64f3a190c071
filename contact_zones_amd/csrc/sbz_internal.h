// sbz_internal.h — shared definitions for the HIP implementation of include/sbz.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/sbz.h"

namespace sbz {

// Features per likelihood tile: one 16-byte observation row per site per tile.
constexpr int FT = 16;
// Threads per likelihood workgroup (4 waves).
constexpr int LIK_BLOCK = 256;

// Device buffer that grows on demand (kept for the context's lifetime).
struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
};

struct LikArgs {
    int N, F, S, Z, Fam, C, FamC, T;  // T = ceil(F / FT) feature tiles
    int B;
    const uint8_t *obs_t;   // [T][N][FT]  x in 0..S (S = NA); padded features hold 0
    const uint8_t *famc;    // [N]  0 = no family (or no inheritance), fam + 1 otherwise
    const uint8_t *zone;    // [B][N]  zone index, 255 = none
    const double *w;        // [B][F][C]
    const double *pg;       // [B][F][S]
    const double *pz;       // [B][Z][F][S]
    const double *pf;       // [B][Fam][F][S] (C == 3 only)
    const uint8_t *src_t;   // [B][T][N][FT] component index per cell, or nullptr (mixture)
    double *partial;        // [B][T]
};

}  // namespace sbz

struct sbz_ctx {
    int device = 0;
    sbz_dims d{};
    int C = 2, FamC = 1, T = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    uint8_t *d_obs_t = nullptr;
    uint8_t *d_famc = nullptr;
    sbz::DevBuf partial, src_t, stage, out;
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

// Launch the likelihood kernels for B chains (all pointers device); out_ll device [B].
int launch_loglik(sbz_ctx *ctx, int B, const uint8_t *zone, const double *w, const double *pg,
                  const double *pz, const double *pf, const uint8_t *source_rowmajor,
                  double *out_ll);

}  // namespace sbz
