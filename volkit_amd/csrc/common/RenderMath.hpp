// RenderMath.hpp -- deterministic float math and RNG for the renderer (host and device).
//
// The reference renderer (src/vkt/Render_kernel.hpp) uses visionaray's libm wrappers and
// random_generator; visionaray is not vendored, so its exact sequences
// are unpinned.  Here every transcendental is a fixed sequence of IEEE float operations
// (range reduction + polynomial; no FMA contraction, correctly rounded division and sqrt),
// so the gfx950 kernel and the CPU oracle (oracle/vkt_oracle.c restates the same sequences)
// produce bit-identical images.  Accuracy: ~2 ulp for ln / exp / sin / cos on the ranges used.
#pragma once

#include <cstdint>
#include <hip/hip_runtime.h>

#define VKT_RHD __host__ __device__ __forceinline__

namespace vkt
{
namespace rmath
{
    VKT_RHD uint32_t f2u(float f)
    {
        union { float f; uint32_t u; } c;
        c.f = f;
        return c.u;
    }

    VKT_RHD float u2f(uint32_t u)
    {
        union { uint32_t u; float f; } c;
        c.u = u;
        return c.f;
    }

    // natural log for x > 0 (0 -> -inf, negative / NaN -> NaN)
    VKT_RHD float ln(float x)
    {
        if (!(x > 0.f))
            return x == 0.f ? -u2f(0x7F800000u) : u2f(0x7FC00000u);
        if (x == u2f(0x7F800000u))
            return x;
        int32_t e = 0;
        if (x < 1.17549435e-38f)   // denormal: scale into the normal range
        {
            x = x * 16777216.f;
            e = -24;
        }
        uint32_t b = f2u(x);
        e += static_cast<int32_t>((b >> 23) & 0xFFu) - 127;
        float m = u2f((b & 0x007FFFFFu) | 0x3F800000u);   // [1, 2)
        if (m > 1.41421356f)
        {
            m = m * 0.5f;
            e += 1;
        }
        float const f = m - 1.f;
        float const s = f / (2.f + f);
        float const z = s * s;
        float p = 0.111111111f;          // 2s * (1 + z/3 + z^2/5 + z^3/7 + z^4/9)
        p = p * z + 0.142857143f;
        p = p * z + 0.2f;
        p = p * z + 0.333333333f;
        p = p * z + 1.f;
        float const lnm = 2.f * s * p;
        float const ef = static_cast<float>(e);
        return ef * 0.693145752f + (lnm + ef * 1.42860677e-06f);   // ln2 = hi + lo
    }

    // e^x (over/underflow saturate to inf / 0)
    VKT_RHD float exp(float x)
    {
        if (x != x)
            return x;
        if (x > 88.7228394f)
            return u2f(0x7F800000u);
        if (x < -87.3365479f)
            return 0.f;
        float const kf = floorf(x * 1.44269504f + 0.5f);
        float const r = (x - kf * 0.693145752f) - kf * 1.42860677e-06f;
        float p = 1.98412698e-04f;       // 1/5040 .. Taylor to r^7
        p = p * r + 1.38888889e-03f;
        p = p * r + 8.33333333e-03f;
        p = p * r + 4.16666667e-02f;
        p = p * r + 1.66666667e-01f;
        p = p * r + 0.5f;
        p = p * r + 1.f;
        p = p * r + 1.f;
        int32_t k = static_cast<int32_t>(kf);
        // 2^k in two steps so that k down to -126 - 23 stays representable
        if (k < -126)
        {
            p = p * u2f(static_cast<uint32_t>(k + 126 + 127) << 23);
            return p * 1.17549435e-38f;
        }
        if (k > 127)
            return u2f(0x7F800000u);
        return p * u2f(static_cast<uint32_t>(k + 127) << 23);
    }

    // x^y for x >= 0
    VKT_RHD float pow(float x, float y)
    {
        if (x == 0.f)
            return y > 0.f ? 0.f : (y == 0.f ? 1.f : u2f(0x7F800000u));
        if (x == 1.f || y == 0.f)
            return 1.f;
        return exp(y * ln(x));
    }

    // sin and cos of a in [-4pi, 4pi] (quadrant reduction, polynomials on [-pi/4, pi/4])
    VKT_RHD void sincos(float a, float& s, float& c)
    {
        float const kf = floorf(a * 0.636619772f + 0.5f);          // a / (pi/2)
        float const r = (a - kf * 1.57079601f) - kf * 3.13916473e-07f;
        float const z = r * r;
        float ps = -1.98412698e-04f;
        ps = ps * z + 8.33333333e-03f;
        ps = ps * z - 1.66666667e-01f;
        float const sr = r + r * z * ps;
        float pc = 2.48015873e-05f;
        pc = pc * z - 1.38888889e-03f;
        pc = pc * z + 4.16666667e-02f;
        float const cr = (1.f - 0.5f * z) + z * z * pc;
        int32_t const q = static_cast<int32_t>(kf) & 3;
        if (q == 0) { s = sr; c = cr; }
        else if (q == 1) { s = cr; c = -sr; }
        else if (q == 2) { s = -sr; c = -cr; }
        else { s = -cr; c = sr; }
    }

    VKT_RHD uint64_t splitmix64(uint64_t x)
    {
        x += 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        return x ^ (x >> 31);
    }

    // PCG32 (XSH RR), one stream per (pixel, frame)
    struct Rng
    {
        uint64_t state, inc;

        VKT_RHD Rng(uint32_t pixel, uint32_t frame)
        {
            inc = (splitmix64(static_cast<uint64_t>(pixel) ^ 0xD1B54A32D192ED03ull) << 1) | 1ull;
            state = splitmix64((static_cast<uint64_t>(frame) << 32) ^ pixel);
        }

        VKT_RHD uint32_t nextU32()
        {
            uint64_t const old = state;
            state = old * 6364136223846793005ull + inc;
            uint32_t const x = static_cast<uint32_t>(((old >> 18) ^ old) >> 27);
            uint32_t const rot = static_cast<uint32_t>(old >> 59);
            return (x >> rot) | (x << ((32u - rot) & 31u));
        }

        // uniform in [0, 1) with 24 random bits
        VKT_RHD float next() { return static_cast<float>(nextU32() >> 8) * 5.96046448e-08f; }
    };

} // rmath
} // vkt
