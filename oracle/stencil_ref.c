/*
 * stencil_ref.c — ORACLE (test infrastructure only): the BASELINE.json workloads as the plain C
 * loop nests pystencils' CPU backend emits for the reference (generate_c(dialect='c'),
 * framework_integration/printer.py:73-75; kernels built by _autodiff.py:479-492,510-525 with
 * ghost_layers=0 and every relative read wrapped in ConditionalFieldAccess, transformations.py:26-30).
 * Cells are visited in C order (coordinate 0 outermost); each neighbour read is
 * `out_of_bounds ? 0 : u[...]`. With -fopenmp the outermost loop is split across threads, which is
 * what the reference does when cpu_openmp=True is forwarded to create_kernel (_autodiff.py:487-489).
 *
 * Used by tests (cross-check of oracle/stencils.py) and as bench.py's cpu_baseline (kind "port").
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef long long i64;

#define IN(c, n) ((c) >= 0 && (c) < (n))

/* out = u + alpha*(sum_6 u[nb] - 6u), zero-padded; float32 storage and arithmetic. The TF-MAD adjoint
 * of this symmetric stencil is the same stencil applied to diffout, so one routine serves both sweeps. */
void oracle_diffusion7_f32(const float* restrict u, float* restrict out, i64 Z, i64 Y, i64 X, float alpha) {
    const float c0 = 1.0f - 6.0f * alpha;
#pragma omp parallel for schedule(static)
    for (i64 z = 0; z < Z; ++z)
        for (i64 y = 0; y < Y; ++y)
            for (i64 x = 0; x < X; ++x) {
                const i64 i = (z * Y + y) * X + x;
                const float ub = IN(z - 1, Z) ? u[i - Y * X] : 0.0f;
                const float ut = IN(z + 1, Z) ? u[i + Y * X] : 0.0f;
                const float us = IN(y - 1, Y) ? u[i - X] : 0.0f;
                const float un = IN(y + 1, Y) ? u[i + X] : 0.0f;
                const float uw = IN(x - 1, X) ? u[i - 1] : 0.0f;
                const float ue = IN(x + 1, X) ? u[i + 1] : 0.0f;
                out[i] = alpha * ub + c0 * u[i] + alpha * ue + alpha * un + alpha * us + alpha * ut + alpha * uw;
            }
}

/* Generic linear stencil out[c] = sum_k w_k u[c + o_k] over a 3-D box (2-D fields: Z = 1). */
void oracle_linear3d_f64(const double* restrict u, double* restrict out, i64 Z, i64 Y, i64 X, int ntaps,
                         const int* restrict offs, const double* restrict w) {
#pragma omp parallel for schedule(static)
    for (i64 z = 0; z < Z; ++z)
        for (i64 y = 0; y < Y; ++y)
            for (i64 x = 0; x < X; ++x) {
                double acc = 0.0;
                for (int k = 0; k < ntaps; ++k) {
                    const i64 zz = z + offs[3 * k], yy = y + offs[3 * k + 1], xx = x + offs[3 * k + 2];
                    if (IN(zz, Z) && IN(yy, Y) && IN(xx, X)) acc += w[k] * u[(zz * Y + yy) * X + xx];
                }
                out[(z * Y + y) * X + x] = acc;
            }
}

static inline float h2f(uint16_t h) {
    uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1f, m = h & 0x3ff, u;
    if (e == 0) {
        if (m == 0) u = s;
        else { e = 127 - 14; while (!(m & 0x400)) { m <<= 1; --e; } m &= 0x3ff; u = s | (e << 23) | (m << 13); }
    } else if (e == 31) u = s | 0x7f800000u | (m << 13);
    else u = s | ((e + 112) << 23) | (m << 13);
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* 27-point stencil, float16 storage, float32 arithmetic, float32 result (rounded by the caller). */
void oracle_stencil27_f16(const uint16_t* restrict u, float* restrict out, i64 Z, i64 Y, i64 X,
                          const float* restrict w /* 27, C order over (dz,dy,dx) in {-1,0,1}^3 */) {
#pragma omp parallel for schedule(static)
    for (i64 z = 0; z < Z; ++z)
        for (i64 y = 0; y < Y; ++y)
            for (i64 x = 0; x < X; ++x) {
                float acc = 0.0f;
                int k = 0;
                for (int dz = -1; dz <= 1; ++dz)
                    for (int dy = -1; dy <= 1; ++dy)
                        for (int dx = -1; dx <= 1; ++dx, ++k) {
                            const i64 zz = z + dz, yy = y + dy, xx = x + dx;
                            const float v = (IN(zz, Z) && IN(yy, Y) && IN(xx, X)) ? h2f(u[(zz * Y + yy) * X + xx]) : 0.0f;
                            acc += w[k] * v;
                        }
                out[(z * Y + y) * X + x] = acc;
            }
}

/* README op z = x*log(x*y) and its adjoint, float32. */
void oracle_readme_fwd_f32(const float* restrict x, const float* restrict y, float* restrict z, i64 n) {
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < n; ++i) z[i] = x[i] * logf(x[i] * y[i]);
}

void oracle_readme_bwd_f32(const float* restrict x, const float* restrict y, const float* restrict dz,
                           float* restrict dx, float* restrict dy, i64 n) {
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < n; ++i) {
        dx[i] = dz[i] * (logf(x[i] * y[i]) + 1.0f);
        dy[i] = dz[i] * x[i] / y[i];
    }
}

int oracle_abi_version(void) { return 1; }
