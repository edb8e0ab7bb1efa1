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
#include <stdlib.h>
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

#ifdef __F16C__
#include <immintrin.h>
#endif

/* IEEE binary16 -> binary32: the hardware conversion (F16C, in every x86-64-v3 host) when compiled for
 * it, else the bit-level restatement. */
static inline float h2f(uint16_t h) {
#ifdef __F16C__
    return _cvtsh_ss(h);
#else
    uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1f, m = h & 0x3ff, u;
    if (e == 0) {
        if (m == 0) u = s;
        else { e = 127 - 14; while (!(m & 0x400)) { m <<= 1; --e; } m &= 0x3ff; u = s | (e << 23) | (m << 13); }
    } else if (e == 31) u = s | 0x7f800000u | (m << 13);
    else u = s | ((e + 112) << 23) | (m << 13);
    float f;
    memcpy(&f, &u, 4);
    return f;
#endif
}

/* One row of binary16 values -> binary32, eight at a time with F16C. */
static void h2f_row(const uint16_t* restrict src, float* restrict dst, i64 n) {
    i64 i = 0;
#ifdef __F16C__
    for (; i + 8 <= n; i += 8)
        _mm256_storeu_ps(dst + i, _mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(src + i))));
#endif
    for (; i < n; ++i) dst[i] = h2f(src[i]);
}

/* 27-point stencil, float16 storage, float32 arithmetic, float32 result (rounded by the caller).
 * Per output row the nine input rows (dz, dy) are converted once into zero-padded float32 rows (the
 * 'zeros' boundary), then the 27 taps run as a vectorisable float loop; the taps are summed in the same
 * (dz, dy, dx) order as the per-tap restatement, so the results are identical. */
void oracle_stencil27_f16(const uint16_t* restrict u, float* restrict out, i64 Z, i64 Y, i64 X,
                          const float* restrict w /* 27, C order over (dz,dy,dx) in {-1,0,1}^3 */) {
#pragma omp parallel
    {
        float* rows = (float*)malloc(sizeof(float) * 9 * (size_t)(X + 2));
#pragma omp for schedule(static)
        for (i64 z = 0; z < Z; ++z)
            for (i64 y = 0; y < Y; ++y) {
                for (int r = 0; r < 9; ++r) {
                    const i64 zz = z + r / 3 - 1, yy = y + r % 3 - 1;
                    float* row = rows + r * (X + 2);
                    row[0] = row[X + 1] = 0.0f;
                    if (IN(zz, Z) && IN(yy, Y)) h2f_row(u + (zz * Y + yy) * X, row + 1, X);
                    else memset(row + 1, 0, sizeof(float) * (size_t)X);
                }
                float* restrict o = out + (z * Y + y) * X;
                for (i64 x = 0; x < X; ++x) o[x] = 0.0f;
                for (int k = 0; k < 27; ++k) {        /* tap-major: each cell still sums k = 0..26 in order */
                    const float wk = w[k];
                    const float* restrict row = rows + (k / 3) * (X + 2) + k % 3;
                    for (i64 x = 0; x < X; ++x) o[x] += wk * row[x];
                }
            }
        free(rows);
    }
}

#ifdef _OPENMP
#include <omp.h>
#endif

/* Thread count of the OpenMP loops above (1 = the reference's default CPU kernel, cpu_openmp off,
 * _autodiff.py:487-489); returns the count in effect. */
int oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
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
