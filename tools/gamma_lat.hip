// Latency of the samplers' random-number pieces on gfx950 (diagnostic, not part of libsbz):
// shader cycles per dependent repetition of a Philox block, the f64 log / sqrt / cospi /
// division, the short log flog(), one Box-Muller normal and one Marsaglia-Tsang gamma (LaneRng, sbz_mh_common.h),
// measured with s_memtime around a dependent chain in every thread of a workgroup.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off tools/gamma_lat.hip -o tools/gamma_lat
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../contact_zones_amd/csrc/sbz_mh_common.h"

using namespace sbz;

// prototype: two Marsaglia-Tsang candidates per round (the Box-Muller pair's two normals, two
// acceptance uniforms); a lane takes the first candidate that passes
__device__ __forceinline__ bool mt_accept(double x, double w, double d, double c, double &v) {
    v = 1.0 + c * x;
    const bool pos = v > 0.0;
    v = v * v * v;
    bool ok = w < 1.0 - 0.0331 * (x * x) * (x * x);
    if (!ok && pos) ok = flog(w) < 0.5 * x * x + d * (1.0 - v + flog(v));
    return ok && pos;
}
__device__ double gamma2(LaneRng &lr, double alpha) {
    const double boost = alpha < 1.0 ? pow(lr.u(), 1.0 / alpha) : 1.0;
    const double a = alpha < 1.0 ? alpha + 1.0 : alpha;
    const double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
    double r = d;
    for (int it = 0; it < 32; it++) {
        const double u1 = 1.0 - lr.u(), u2 = lr.u();
        const double w0 = lr.u(), w1 = lr.u();
        const double rad = sqrt(-2.0 * flog(u1));
        double sn, cs;
        sincospi(2.0 * u2, &sn, &cs);
        double v0, v1;
        const bool ok0 = mt_accept(rad * cs, w0, d, c, v0);
        const bool ok1 = mt_accept(rad * sn, w1, d, c, v1);
        if (ok0 || ok1) {
            r = d * (ok0 ? v0 : v1);
            break;
        }
    }
    return r * boost;
}

__global__ void lat_kernel(int which, int reps, double alpha, double *cyc, double *sink) {
    const int tid = threadIdx.x;
    double x = 0.5 + tid * 1e-3;
    uint32_t c[4] = {(uint32_t)tid, 1u, (uint32_t)blockIdx.x, 3u};
    double a = alpha;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; r++) {
        switch (which) {
            case 0: philox4x32_10(c, 11u, 13u); break;
            case 1: x = log(x + 2.0); break;
            case 2: x = sqrt(x + 2.0); break;
            case 3: x = cospi(x); break;
            case 4: x = 1.0 / (x + 1.0); break;
            case 5: {
                LaneRng lr;
                lr.initk(11u, 13u, blockIdx.x, (uint64_t)r + (x > 1e300 ? 1 : 0), tid);
                x = lr.normal();
            } break;
            case 6: {
                LaneRng lr;
                lr.initk(11u, 13u, blockIdx.x, (uint64_t)r, tid);
                const double g = lr.gamma(a);
                a = alpha + (g > 1e300 ? 1.0 : 0.0);
                x += g;
            } break;
            case 8: x = flog(x + 2.0); break;
            case 9: x = fdiv_pos(1.0, x + 1.0); break;
            case 11: {
                LaneRng lr;
                lr.initk(11u, 13u, blockIdx.x, (uint64_t)r, tid);
                const double g = gamma2(lr, a);
                a = alpha + (g > 1e300 ? 1.0 : 0.0);
                x += g;
            } break;
            case 10: x = __builtin_amdgcn_sqrt(x + 2.0); break;
            case 7: {  // the u() uniform alone (one Philox block per two)
                LaneRng lr;
                lr.initk(11u, 13u, blockIdx.x, (uint64_t)r + (x > 1e300 ? 1 : 0), tid);
                x += lr.u();
            } break;
            default: break;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    cyc[blockIdx.x * blockDim.x + tid] = (double)(t1 - t0) / reps;
    sink[blockIdx.x * blockDim.x + tid] = x + c[0] + c[1] + c[2] + c[3];
}

// flog() on the device against a long-double log on the host: max and mean ulp error
__global__ void flog_kernel(int n, const double *x, double *y, double *q, double *r) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        y[i] = flog(x[i]);
        q[i] = fdiv_pos(0.5 + 0.5 * x[(i * 7) % n] / (1.0 + x[(i * 7) % n]), 0.5 + 0.5 * x[i] / (1.0 + x[i]));
        r[i] = __builtin_amdgcn_sqrt(x[i]);
    }
}

static void flog_accuracy() {
    const int n = 1 << 22;
    std::vector<double> hx(n), hy(n);
    uint64_t st = 88172645463325252ull;
    auto next = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    for (int i = 0; i < n; i++) {
        const double u = (double)(next() >> 11) * 0x1p-53;
        const int k = i & 3;
        hx[i] = k == 0 ? u : k == 1 ? 0.5 + u : k == 2 ? 1.0 + 1e-6 * (u - 0.5) : ldexp(1.0 + u, (int)(next() % 2100) - 1074);
    }
    double *dx, *dy, *dq, *dr;
    if (hipMalloc(&dx, n * 8) != hipSuccess || hipMalloc(&dy, n * 8) != hipSuccess || hipMalloc(&dq, n * 8) != hipSuccess ||
        hipMalloc(&dr, n * 8) != hipSuccess)
        return;
    (void)hipMemcpy(dx, hx.data(), n * 8, hipMemcpyHostToDevice);
    flog_kernel<<<(n + 255) / 256, 256>>>(n, dx, dy, dq, dr);
    std::vector<double> hq(n), hr(n);
    (void)hipMemcpy(hy.data(), dy, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hq.data(), dq, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hr.data(), dr, n * 8, hipMemcpyDeviceToHost);
    // fdiv_pos on [0.5, 1) operands (the delta's mantissas) and v_sqrt_f64, against the
    // correctly rounded host results: max ulp
    double wq = 0, wr = 0;
    for (int i = 0; i < n; i++) {
        if (!std::isfinite(hx[i]) || hx[i] <= 0.0) continue;
        const double a = 0.5 + 0.5 * hx[(i * 7) % n] / (1.0 + hx[(i * 7) % n]), b = 0.5 + 0.5 * hx[i] / (1.0 + hx[i]);
        const double eq = fabs(hq[i] - a / b) / (nextafter(a / b, INFINITY) - a / b);
        const double sr = sqrt(hx[i]);
        const double er = fabs(hr[i] - sr) / (nextafter(sr, INFINITY) - sr);
        if (eq > wq) wq = eq;
        if (er > wr && std::isnormal(hx[i])) wr = er;
    }
    printf("{\"fdiv_pos_max_ulp\": %.3f, \"v_sqrt_f64_max_ulp\": %.3f}\n", wq, wr);
    double worst = 0, sum = 0, wx = 0;
    long cnt = 0;
    for (int i = 0; i < n; i++) {
        if (hx[i] == 1.0 || hx[i] <= 0.0 || !std::isfinite(hx[i])) continue;
        const long double ref = logl((long double)hx[i]);
        const double r = (double)ref;
        const double ulp = nextafter(fabs(r), INFINITY) - fabs(r);
        const double e = (double)fabsl((long double)hy[i] - ref) / ulp;
        sum += e;
        cnt++;
        if (e > worst) { worst = e; wx = hx[i]; }
    }
    int special = (hy[0] == hy[0]);
    printf("{\"flog_max_ulp\": %.3f, \"at\": %.17g, \"mean_ulp\": %.4f, \"n\": %ld}\n", worst, wx, sum / cnt, cnt);
    (void)special;
    (void)hipFree(dx);
    (void)hipFree(dy);
    (void)hipFree(dq);
    (void)hipFree(dr);
}

// gamma2 sample moments (mean alpha, variance alpha) as a sanity check of the prototype
__global__ void gamma2_kernel(int n, double alpha, double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    LaneRng lr;
    lr.initk(7u, 9u, (uint64_t)(i / 64), 0, i % 64);
    out[i] = gamma2(lr, alpha);
}
static void gamma2_moments() {
    const int n = 1 << 22;
    double *d;
    if (hipMalloc(&d, n * 8) != hipSuccess) return;
    std::vector<double> h(n);
    for (double alpha : {0.3, 1.0, 1.5, 4.0, 30.0}) {
        gamma2_kernel<<<n / 256, 256>>>(n, alpha, d);
        (void)hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
        double m = 0, v = 0;
        for (double x : h) m += x;
        m /= n;
        for (double x : h) v += (x - m) * (x - m);
        v /= n - 1;
        printf("{\"gamma2_alpha\": %.1f, \"mean\": %.5f, \"var\": %.5f, \"z_mean\": %.2f}\n", alpha, m, v,
               (m - alpha) / sqrt(alpha / n));
    }
    (void)hipFree(d);
}

int main() {
    flog_accuracy();
    gamma2_moments();
    const char *names[] = {"philox4x32_10", "log", "sqrt", "cospi", "div", "normal", "gamma", "u", "flog", "fdiv_pos", "v_sqrt_f64", "gamma2"};
    const int reps = 64;
    for (int threads : {64, 256, 512}) {
        const int blocks = 256;
        const int n = blocks * threads;
        double *cyc, *sink;
        if (hipMalloc(&cyc, n * 8) != hipSuccess || hipMalloc(&sink, n * 8) != hipSuccess) return 1;
        std::vector<double> h(n);
        for (int which = 0; which < 12; which++) {
            for (double alpha : {1.5, 30.0}) {
                if (which != 6 && which != 11 && alpha != 1.5) continue;
                lat_kernel<<<blocks, threads>>>(which, reps, alpha, cyc, sink);
                if (hipDeviceSynchronize() != hipSuccess) return 2;
                if (hipMemcpy(h.data(), cyc, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
                double s = 0;
                for (double v : h) s += v;
                printf("{\"threads\": %d, \"op\": \"%s\", \"alpha\": %.1f, \"cycles_per_rep\": %.1f}\n", threads,
                       names[which], alpha, s / n);
            }
        }
        (void)hipFree(cyc);
        (void)hipFree(sink);
    }
    return 0;
}
