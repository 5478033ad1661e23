// philox_normal.h -- counter-based Gaussian noise for the multicolour Gibbs sweeps.
//
// The reference draws its noise from one shared std::mt19937_64 through a
// std::normal_distribution per sampler object (sampler/sampler.hh:31-34, :69-71;
// sampler/sor_sampler.cc:42-46).  That stream is inherently sequential, so the device path
// replaces it with a counter-based generator: every normal is a pure function of
//   key     = (lo32(seed), lo32(chain) ^ hi32(seed))
//   counter = (pair id, sweep tag, lo32(sample), hi32(sample))
// (Philox4x32-10, Salmon et al. SC'11) followed by a Box-Muller transform whose log / sin / cos
// are evaluated with a fixed sequence of IEEE-754 double operations (explicit fma, correctly
// rounded sqrt, a literal 64-entry log reduction table).  The same bits therefore come out of gfx950 and of a host compiler with
// -ffp-contract=off, which is what lets the CPU oracle replay the device chain exactly.
//
// Pair id: points (i, i+1) with i odd share one Philox call (cos branch for i odd, sin branch
// for i even), pair = row * (nx/2) + (i-1)/2 with row the lexicographic index of (j,k).
#pragma once
#include <math.h>
#include <stdint.h>

#include "log_table.h"

#if defined(__HIPCC__)
#define MGMC_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define MGMC_HD static inline
#endif

namespace mgmc {

struct Philox4 {
    uint32_t v[4];
};

// a ^ b ^ k with k wave-uniform (the Philox key): one v_bitop3_b32 (truth table 0x96 = 3-input xor)
MGMC_HD uint32_t xor3_key(uint32_t a, uint32_t b, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "s"(k));
    return d;
#else
    return a ^ b ^ k;
#endif
}

// fma(a, b, c) with c a literal constant: on the device one v_fma_f64 with c in SGPRs (the
// compiler otherwise keeps such constants in VGPRs and copies them into a tied v_fmac accumulator)
MGMC_HD double fma_k(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
#else
    return fma(a, b, c);
#endif
}

MGMC_HD Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c0;
        const uint64_t p1 = (uint64_t)M1 * c2;
        const uint32_t n0 = xor3_key((uint32_t)(p1 >> 32), c1, k0);
        const uint32_t n1 = (uint32_t)p1;
        const uint32_t n2 = xor3_key((uint32_t)(p0 >> 32), c3, k1);
        const uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += W0; k1 += W1;
    }
    Philox4 out;
    out.v[0] = c0; out.v[1] = c1; out.v[2] = c2; out.v[3] = c3;
    return out;
}

MGMC_HD double as_double(uint64_t b) {
    union { uint64_t u; double d; } c;
    c.u = b;
    return c.d;
}
MGMC_HD uint64_t as_bits(double d) {
    union { uint64_t u; double d; } c;
    c.d = d;
    return c.u;
}

// Uniforms are built exactly from 52 random mantissa bits: v = 1.m in [1,2) (bit pattern), then
// u1 = 2 - v in (0,1] and u2 = v - 1 in [0,1) -- both subtractions are exact.
MGMC_HD uint64_t bits52(uint32_t a, uint32_t b) { return ((uint64_t)a << 20) | (uint64_t)(b >> 12); }

// natural log of u in [2^-52, 1], division free: u = 2^e m, m in [1,2), table point
// rc_i ~ 1/m (top 6 mantissa bits), r = m rc_i - 1 (|r| < 1/128, one fma), log1p(r) by a
// degree-8 polynomial, plus the tabulated -log(rc_i) = hi + lo (log_table.h).  Absolute error
// ~1e-17; the caller clamps -2 log(u) at 0.
MGMC_HD double log_unit(double u, const double* rct, const double* hit, const double* lot) {
    const uint64_t b = as_bits(u);
    const int e = (int)((b >> 52) & 0x7ff) - 1023;
    const uint64_t mant = b & 0x000fffffffffffffull;
    const int idx = (int)(mant >> 46);
    const double m = as_double(mant | 0x3ff0000000000000ull);
    const double r = fma(m, rct[idx], -1.0);
    double q = -1.0 / 8.0;
    q = fma_k(q, r, 1.0 / 7.0);
    q = fma_k(q, r, -1.0 / 6.0);
    q = fma_k(q, r, 1.0 / 5.0);
    q = fma_k(q, r, -1.0 / 4.0);
    q = fma_k(q, r, 1.0 / 3.0);
    q = fma(q, r, -0.5);
    const double p = fma(r * r, q, r);  // log1p(r)
    const double de = (double)e;
    const double LN2_HI = 6.93147180369123816490e-01;  // 0x3fe62e42fee00000
    const double LN2_LO = 1.90821492927058770002e-10;  // 0x3dea39ef35793c76
    return fma(de, LN2_HI, hit[idx]) + (fma(de, LN2_LO, lot[idx]) + p);
}

// (cos(2 pi t), sin(2 pi t)) for t in [0,1) with at most 52 fractional bits.  t = k/64 + r with
// k = round(64 t) in [0,64] and r exact (|r| <= 1/128); theta = 2 pi r, |theta| <= pi/64;
// sin theta to degree 9 and cos theta - 1 to degree 8 (truncation < 1e-19), then the addition
// theorem with the literal table sct[2k], sct[2k+1] = cos, sin(2 pi k/64) (log_table.h).
MGMC_HD void sincos_2pi(double t, const double* sct, double* c_out, double* s_out) {
    const int k = (int)fma(t, 64.0, 0.5);                // exact argument, k in [0, 64]
    const double r = fma((double)(-k), 0.015625, t);     // exact
    const double th = r * 6.28318530717958647692;
    const double t2 = th * th;
    double ps = 1.0 / 362880.0;
    ps = fma_k(ps, t2, -1.0 / 5040.0);
    ps = fma_k(ps, t2, 1.0 / 120.0);
    ps = fma_k(ps, t2, -1.0 / 6.0);
    const double sn = fma(th * t2, ps, th);              // sin theta
    double pc = 1.0 / 40320.0;
    pc = fma_k(pc, t2, -1.0 / 720.0);
    pc = fma_k(pc, t2, 1.0 / 24.0);
    pc = fma(pc, t2, -0.5);
    const double w = pc * t2;                            // cos theta - 1
    const double C = sct[2 * k], S = sct[2 * k + 1];
    *c_out = fma(C, w, fma(-S, sn, C));
    *s_out = fma(S, w, fma(C, sn, S));
}

// sqrt(x) for x = 0 or x >= 2^-700, correctly rounded: on the device the rsq + Newton sequence of
// the compiler's IEEE sqrt lowering without its denormal-range scaling (never taken here), so the
// bits equal the host's sqrt.
MGMC_HD double sqrt_rad(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = 0.5 * y;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    g = fma(d, h, g);
    return x > 0.0 ? g : 0.0;
#else
    return x > 0.0 ? sqrt(x) : 0.0;
#endif
}

// Box-Muller pair from one Philox block: (z_cos, z_sin)
MGMC_HD void normal_pair_t(const Philox4& r, double* z0, double* z1, const double* rct, const double* hit,
                           const double* lot, const double* sct) {
    const double v1 = as_double(0x3ff0000000000000ull | bits52(r.v[0], r.v[1]));
    const double v2 = as_double(0x3ff0000000000000ull | bits52(r.v[2], r.v[3]));
    const double u1 = 2.0 - v1;  // (0,1]
    const double u2 = v2 - 1.0;  // [0,1)
    const double rad = sqrt_rad(-2.0 * log_unit(u1, rct, hit, lot));
    double c, s;
    sincos_2pi(u2, sct, &c, &s);
    *z0 = rad * c;
    *z1 = rad * s;
}

struct RngKey {
    uint32_t k0, k1;
};

MGMC_HD RngKey make_key(uint64_t seed, uint64_t chain) {
    RngKey k;
    k.k0 = (uint32_t)seed;
    k.k1 = (uint32_t)chain ^ (uint32_t)(seed >> 32);
    return k;
}

MGMC_HD void normal_pair(const Philox4& r, double* z0, double* z1) {
    normal_pair_t(r, z0, z1, LOGTAB_RC, LOGTAB_HI, LOGTAB_LO, SINCOS_TAB);
}

// one normal for the point whose pair id is `pair`; cos_branch selects the first of the two
MGMC_HD double point_normal(RngKey key, uint32_t pair, bool cos_branch, uint32_t tag, uint64_t sample) {
    const Philox4 r = philox4x32_10(pair, tag, (uint32_t)sample, (uint32_t)(sample >> 32), key.k0, key.k1);
    double z0, z1;
    normal_pair(r, &z0, &z1);
    return cos_branch ? z0 : z1;
}

}  // namespace mgmc
