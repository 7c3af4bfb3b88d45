/*
 * vkt_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the volkit reference's
 * serial StructuredVolume path (see vkt_oracle.h for the pinning status).
 *
 * Structure deliberately follows the reference: per-voxel accessors (get_value /
 * set_value / get_bytes / set_bytes, reference src/vkt/StructuredVolume.cpp:155-296)
 * driven by z->y->x loops with `!=` bounds (src/vkt/for_each.hpp:23-39), so that the
 * timed CPU baseline keeps the reference's loop order and per-voxel call structure.
 * The reference's migrate()/policy-lookup overhead per access is NOT reproduced.
 *
 * Build: gcc -O2 -fPIC -shared -ffp-contract=off (oracle/Makefile); no -march, like the
 * reference's CMake build (which sets no flags).
 */
#include "vkt_oracle.h"

#include <float.h>
#include <math.h>
#include <string.h>

/* ---- helpers: src/vkt/linalg.hpp:18-41 ------------------------------------------ */
static float r_min(float a, float b) { return b < a ? b : a; }
static float r_max(float a, float b) { return a < b ? b : a; }
static float r_clamp(float x, float lo, float hi) { return r_max(lo, r_min(x, hi)); }
static int32_t i_clamp(int32_t x, int32_t lo, int32_t hi)
{
    int32_t m = hi < x ? hi : x; /* clamp = max(lo, min(x, hi)) */
    return lo < m ? m : lo;
}
static float r_lerp(float a, float b, float t) { return (1.0f - t) * a + t * b; }

/* x86 cvttss2si semantics, as the reference's float->int16/int8 assignments compile
 * (SURVEY.md Appendix A.1). */
static int32_t cvtt_i32(float f)
{
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int32_t)f : INT32_MIN;
}
static int64_t cvtt_i64(float f)
{
    return (f >= -9223372036854775808.0f && f < 9223372036854775808.0f) ? (int64_t)f : INT64_MIN;
}

/* src/vkt/DataFormatInfo.hpp:34-47 */
uint32_t vko_bytes_per_voxel(int32_t fmt)
{
    switch (fmt) {
    case 1: case 4: return 1;
    case 2: case 5: return 2;
    case 3: case 6: case 7: return 4;
    default: return 255;
    }
}

/* MapVoxelImpl, src/vkt/VoxelMapping.hpp:15-95 (little endian). */
void vko_map(uint8_t* dst, float value, int32_t fmt, float lo, float hi)
{
    value -= lo;
    value /= hi - lo;
    switch (fmt) {
    case 2: { /* Int16, :28-38 */
        uint32_t c = (uint32_t)cvtt_i32(value * 65535.999f - 32767.f);
        dst[0] = (uint8_t)c;
        dst[1] = (uint8_t)(c >> 8);
        break;
    }
    case 4: /* UInt8, :41-46 */
        dst[0] = (uint8_t)cvtt_i32(value * 255.999f);
        break;
    case 5: { /* UInt16, :48-59 */
        uint32_t c = (uint32_t)cvtt_i32(value * 65535.999f);
        dst[0] = (uint8_t)c;
        dst[1] = (uint8_t)(c >> 8);
        break;
    }
    case 6: { /* UInt32, :62-76 */
        uint32_t c = (uint32_t)(uint64_t)cvtt_i64(value * 4294967295.999f);
        dst[0] = (uint8_t)c;
        dst[1] = (uint8_t)(c >> 8);
        dst[2] = (uint8_t)(c >> 16);
        dst[3] = (uint8_t)(c >> 24);
        break;
    }
    case 7: { /* Float32, :79-94 */
        uint32_t c;
        memcpy(&c, &value, 4);
        dst[0] = (uint8_t)c;
        dst[1] = (uint8_t)(c >> 8);
        dst[2] = (uint8_t)(c >> 16);
        dst[3] = (uint8_t)(c >> 24);
        break;
    }
    default: /* Int8, Int32, Unspecified: no case in the reference switch */
        break;
    }
}

/* UnmapVoxelImpl, src/vkt/VoxelMapping.hpp:98-177 (little endian); leaves *value
 * untouched for formats without a case. */
void vko_unmap(float* value, const uint8_t* src, int32_t fmt, float lo, float hi)
{
    switch (fmt) {
    case 2: { /* :107-119 */
        int16_t iv = (int16_t)(uint16_t)(src[0] | (src[1] << 8));
        float f = (float)iv;
        *value = r_lerp(lo, hi, (f + 32767.f) / 65535.999f);
        break;
    }
    case 4: /* :122-127 */
        *value = r_lerp(lo, hi, (float)src[0] / 255.999f);
        break;
    case 5: { /* :130-142 */
        uint16_t iv = (uint16_t)(src[0] | (src[1] << 8));
        *value = r_lerp(lo, hi, (float)iv / 65535.999f);
        break;
    }
    case 6: { /* :145-160 */
        uint32_t iv = (uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16) |
                      ((uint32_t)src[3] << 24);
        *value = r_lerp(lo, hi, (float)iv / 4294967295.999f);
        break;
    }
    case 7: { /* :163-175 */
        uint32_t iv = (uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16) |
                      ((uint32_t)src[3] << 24);
        memcpy(value, &iv, 4);
        break;
    }
    default:
        break;
    }
}

/* ---- per-voxel accessors: src/vkt/StructuredVolume.cpp:155-317 -------------------- */
static size_t lin_index(const vko_volume* v, int32_t x, int32_t y, int32_t z)
{
    size_t idx = (size_t)z * (size_t)v->dims[0] * (size_t)v->dims[1] + (size_t)y * (size_t)v->dims[0] + (size_t)x;
    return idx * vko_bytes_per_voxel(v->fmt);
}

static float get_value(const vko_volume* v, int32_t x, int32_t y, int32_t z)
{
    float value = 0.f; /* StructuredVolume.cpp:196 */
    vko_unmap(&value, v->data + lin_index(v, x, y, z), v->fmt, v->lo, v->hi);
    return value;
}

static void set_value(vko_volume* v, int32_t x, int32_t y, int32_t z, float value)
{
    vko_map(v->data + lin_index(v, x, y, z), value, v->fmt, v->lo, v->hi);
}

static void get_bytes(const vko_volume* v, int32_t x, int32_t y, int32_t z, uint8_t* out)
{
    uint32_t bpv = vko_bytes_per_voxel(v->fmt);
    size_t idx = lin_index(v, x, y, z);
    for (uint32_t i = 0; i < bpv; ++i)
        out[i] = v->data[idx + i];
}

static void set_bytes(vko_volume* v, int32_t x, int32_t y, int32_t z, const uint8_t* in)
{
    uint32_t bpv = vko_bytes_per_voxel(v->fmt);
    size_t idx = lin_index(v, x, y, z);
    for (uint32_t i = 0; i < bpv; ++i)
        v->data[idx + i] = in[i];
}

/* Flat-index read used by sampleLinear's unclamped hi.x neighbour
 * (src/vkt/StructuredVolumeView.hpp:93-107): the reference reads one voxel past the
 * end of the buffer there (undefined); both this oracle and the HIP kernel clamp that
 * single read to the last voxel. */
static float get_value_flat(const vko_volume* v, size_t voxel)
{
    uint32_t bpv = vko_bytes_per_voxel(v->fmt);
    size_t nvox = v->nbytes / bpv;
    if (voxel >= nvox)
        voxel = nvox - 1;
    float value = 0.f;
    vko_unmap(&value, v->data + voxel * bpv, v->fmt, v->lo, v->hi);
    return value;
}

/* ---- FillRange_serial, src/vkt/Fill_serial.hpp:20-26 ----------------------------- */
void vko_fill_range(vko_volume* v, const int32_t first[3], const int32_t last[3], float value)
{
    for (int32_t z = first[2]; z != last[2]; ++z)
        for (int32_t y = first[1]; y != last[1]; ++y)
            for (int32_t x = first[0]; x != last[0]; ++x)
                set_value(v, x, y, z, value);
}

/* ---- CopyRange_serial, src/vkt/Copy_serial.hpp:13-82 ----------------------------- */
void vko_copy_range(vko_volume* dst, vko_volume* src, const int32_t first[3], const int32_t last[3],
                    const int32_t off[3])
{
    int bytewise = dst->fmt == src->fmt && dst->lo == src->lo && dst->hi == src->hi; /* :21-22 */
    uint8_t voxel[8];
    for (int32_t z = first[2]; z != last[2]; ++z)
        for (int32_t y = first[1]; y != last[1]; ++y)
            for (int32_t x = first[0]; x != last[0]; ++x) {
                int32_t sx = i_clamp(x, 0, src->dims[0] - 1);
                int32_t sy = i_clamp(y, 0, src->dims[1] - 1);
                int32_t sz = i_clamp(z, 0, src->dims[2] - 1);
                int32_t dx = x - first[0] + off[0];
                int32_t dy = y - first[1] + off[1];
                int32_t dz = z - first[2] + off[2];
                /* the reference repeats this per byte of the voxel (:34,:63); idempotent */
                if (bytewise) {
                    get_bytes(src, sx, sy, sz, voxel);
                    set_bytes(dst, dx, dy, dz, voxel);
                } else {
                    set_value(dst, dx, dy, dz, get_value(src, sx, sy, sz));
                }
            }
}

/* ---- ArithmeticOp + lambdas, src/vkt/Arithmetic_serial.hpp:15-258 ---------------- */
static float apply_op(int32_t op, float f1, float f2, float lo, float hi)
{
    switch (op) {
    case 0: return f1 + f2;                                /* :63 */
    case 1: return f1 - f2;                                /* :83 */
    case 2: return f1 * f2;                                /* :103 */
    case 3: return f1 / f2;                                /* :123 */
    case 4: return fabsf(f1 - f2);                         /* :143 */
    case 5: return r_clamp(f1 + f2, lo, hi);               /* :156-166 */
    case 6: return r_clamp(f1 - f2, lo, hi);
    case 7: return r_clamp(f1 * f2, lo, hi);
    case 8: return r_clamp(f1 / f2, lo, hi);
    case 9: return r_clamp(fabsf(f1 - f2), lo, hi);
    default: return 0.f;
    }
}

void vko_arith_range(int32_t op, vko_volume* dst, vko_volume* s1, vko_volume* s2, const int32_t first[3],
                     const int32_t last[3], const int32_t off[3])
{
    float lo = dst->lo, hi = dst->hi;
    for (int32_t z = first[2]; z != last[2]; ++z)
        for (int32_t y = first[1]; y != last[1]; ++y)
            for (int32_t x = first[0]; x != last[0]; ++x) {
                float v1 = get_value(s1, x, y, z);
                float v2 = get_value(s2, x, y, z);
                set_value(dst, x + off[0], y + off[1], z + off[2], apply_op(op, v1, v2, lo, hi));
            }
}

/* ---- Resample_serial (SV->SV), src/vkt/Resample_serial.hpp:26-71 ----------------- */
static int32_t src_index(int32_t d, int32_t dd, int32_t sd)
{
    /* :60-62 then the implicit int32 conversion of sampleLinear's parameters (:65) or
     * the explicit (int32_t) cast (:67): f32 divide, f32 multiply, truncate. */
    float s = (float)d / (float)dd * (float)sd;
    return (int32_t)s;
}

/* sampleLinear(int32_t,int32_t,int32_t), src/vkt/StructuredVolumeView.hpp:80-119, with
 * z given in slab-local planes (local = global - src_z0). */
static float sample_linear(const vko_volume* src, int32_t x, int32_t y, int32_t zg, int32_t src_gdz,
                           int32_t src_z0)
{
    float xf1 = x - 0.f, yf1 = y - 0.f, zf1 = zg - 0.f;
    float xf2 = x + 1.f, yf2 = y + 1.f, zf2 = zg + 1.f;
    int32_t lox = (int32_t)xf1, loy = (int32_t)yf1, loz = (int32_t)zf1;
    int32_t hix = (int32_t)xf2, hiy = (int32_t)yf2, hiz = (int32_t)zf2;
    lox = i_clamp(lox, 0, src->dims[0] - 1); /* :93-99: lo.x, lo.y, hi.y, hi.z only */
    loy = i_clamp(loy, 0, src->dims[1] - 1);
    hiy = i_clamp(hiy, 0, src->dims[1] - 1);
    hiz = i_clamp(hiz, 0, src_gdz - 1);
    float fx = xf1 - lox, fy = yf1 - loy, fz = zf1 - loz;
    size_t dx = (size_t)src->dims[0], plane = dx * (size_t)src->dims[1];
    size_t zl0 = (size_t)(loz - src_z0), zl1 = (size_t)(hiz - src_z0);
#define FLAT(X, Y, Z) get_value_flat(src, (Z) * plane + (size_t)(Y) * dx + (size_t)(X))
    float v0 = FLAT(lox, loy, zl0), v1 = FLAT(hix, loy, zl0);
    float v2 = FLAT(lox, hiy, zl0), v3 = FLAT(hix, hiy, zl0);
    float v4 = FLAT(lox, loy, zl1), v5 = FLAT(hix, loy, zl1);
    float v6 = FLAT(lox, hiy, zl1), v7 = FLAT(hix, hiy, zl1);
#undef FLAT
    return r_lerp(r_lerp(r_lerp(v0, v1, fx), r_lerp(v2, v3, fx), fy),
                  r_lerp(r_lerp(v4, v5, fx), r_lerp(v6, v7, fx), fy), fz);
}

void vko_resample_slab(vko_volume* dst, vko_volume* src, int32_t filter, int32_t dst_gdz, int32_t dst_z0,
                       int32_t src_gdz, int32_t src_z0)
{
    int32_t ddx = dst->dims[0], ddy = dst->dims[1];
    int32_t sdx = src->dims[0], sdy = src->dims[1];
    if (ddx == sdx && ddy == sdy && dst_gdz == src_gdz) {
        /* same-dims branch, :32-48: per-voxel re-encode, no index math */
        for (int32_t z = 0; z != dst->dims[2]; ++z)
            for (int32_t y = 0; y != ddy; ++y)
                for (int32_t x = 0; x != ddx; ++x)
                    set_value(dst, x, y, z, get_value(src, x, y, z + dst_z0 - src_z0));
        return;
    }
    for (int32_t z = 0; z != dst->dims[2]; ++z) {
        int32_t sz = src_index(z + dst_z0, dst_gdz, src_gdz);
        for (int32_t y = 0; y != ddy; ++y) {
            int32_t sy = src_index(y, ddy, sdy);
            for (int32_t x = 0; x != ddx; ++x) {
                int32_t sx = src_index(x, ddx, sdx);
                float value;
                if (filter == 1)
                    value = sample_linear(src, sx, sy, sz, src_gdz, src_z0);
                else
                    value = get_value(src, sx, sy, sz - src_z0);
                set_value(dst, x, y, z, value);
            }
        }
    }
}

void vko_resample(vko_volume* dst, vko_volume* src, int32_t filter)
{
    vko_resample_slab(dst, src, filter, dst->dims[2], 0, src->dims[2], 0);
}

/* ---- TransformRange_serial, src/vkt/Transform_serial.hpp:15-101 ------------------ */
void vko_transform_range1(vko_volume* v, const int32_t first[3], const int32_t last[3], vko_unary_op op)
{
    for (int32_t z = first[2]; z != last[2]; ++z)
        for (int32_t y = first[1]; y != last[1]; ++y)
            for (int32_t x = first[0]; x != last[0]; ++x) {
                uint8_t bytes[8];
                memset(bytes, 0, sizeof(bytes));
                get_bytes(v, x, y, z, bytes);
                op(x, y, z, bytes, v->fmt, v->lo, v->hi);
                set_bytes(v, x, y, z, bytes);
            }
}

void vko_transform_range2(vko_volume* v1, vko_volume* v2, const int32_t first[3], const int32_t last[3],
                          const int32_t off[3], vko_binary_op op)
{
    for (int32_t z = first[2]; z != last[2]; ++z)
        for (int32_t y = first[1]; y != last[1]; ++y)
            for (int32_t x = first[0]; x != last[0]; ++x) {
                uint8_t b1[8], b2[8];
                memset(b1, 0, sizeof(b1));
                memset(b2, 0, sizeof(b2));
                get_bytes(v1, x, y, z, b1);
                get_bytes(v2, x + off[0], y + off[1], z + off[2], b2);
                op(x, y, z, b1, v1->fmt, v1->lo, v1->hi, b2, v2->fmt, v2->lo, v2->hi);
                set_bytes(v1, x, y, z, b1);
                set_bytes(v2, x + off[0], y + off[1], z + off[2], b2);
            }
}

/* ---- ComputeAggregatesRange_serial, src/vkt/Aggregates_serial.hpp:20-83 ---------- */
void vko_aggregates_range(const vko_volume* v, const int32_t first[3], const int32_t last[3], vko_aggregates* a)
{
    memset(a, 0, sizeof(*a)); /* :27 */
    a->min = FLT_MAX;         /* :29-31 */
    a->max = -FLT_MAX;
    a->prod = 1.f;
    for (int32_t z = first[2]; z != last[2]; ++z)
        for (int32_t y = first[1]; y != last[1]; ++y)
            for (int32_t x = first[0]; x != last[0]; ++x) {
                float val = get_value(v, x, y, z);
                if (val < a->min) { /* :41-45 */
                    a->min = val;
                    a->argmin[0] = x; a->argmin[1] = y; a->argmin[2] = z;
                }
                if (val > a->max) { /* :47-51 */
                    a->max = val;
                    a->argmax[0] = x; a->argmax[1] = y; a->argmax[2] = z;
                }
                a->mean += val;     /* :53 */
                a->sum += val;      /* :55 */
                a->prod *= val;     /* :56 */
            }
    size_t num = (size_t)v->dims[0] * (size_t)v->dims[1] * (size_t)v->dims[2]; /* :61 */
    a->mean = (float)(a->mean / (double)num);                                   /* :63 */
    for (int32_t z = first[2]; z != last[2]; ++z)                                /* :68-80 */
        for (int32_t y = first[1]; y != last[1]; ++y)
            for (int32_t x = first[0]; x != last[0]; ++x) {
                float val = get_value(v, x, y, z);
                a->var += (val - a->mean) * (val - a->mean);
            }
    a->var = (float)(a->var / (double)num); /* :81 */
    a->stddev = sqrtf(a->var);              /* :82 */
}

/* ---- ComputeHistogramRange_serial, src/vkt/Histogram_serial.hpp:20-50 ------------- */
uint64_t vko_histogram_range(const vko_volume* v, const int32_t first[3], const int32_t last[3], uint64_t* bins,
                             uint64_t num_bins)
{
    float lo = v->lo, hi = v->hi;
    uint64_t skipped = 0;
    float scale = (float)num_bins / (hi - lo); /* numBins / (hi - lo): size_t -> float */
    memset(bins, 0, num_bins * sizeof(uint64_t));
    for (int32_t z = first[2]; z != last[2]; ++z)
        for (int32_t y = first[1]; y != last[1]; ++y)
            for (int32_t x = first[0]; x != last[0]; ++x) {
                float val = get_value(v, x, y, z);
                float f = (val - lo) * scale;
                /* (size_t)f: x86-64 truncation; (-1, 0) -> 0; the rest would index out of bounds */
                if (!(f > -1.0f) || !(f < 9.2233720e18f)) {
                    ++skipped;
                    continue;
                }
                uint64_t bin = (uint64_t)(int64_t)f;
                if (bin >= num_bins) {
                    ++skipped;
                    continue;
                }
                bins[bin]++;
            }
    return skipped;
}

/* ---- renderers, reference src/vkt/Render_kernel.hpp:80-418 -------------------------- */
/* deterministic math restated from common/RenderMath.hpp (same float operation sequences) */
static uint32_t r_f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float r_u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static float r_ln(float x)
{
    if (!(x > 0.f))
        return x == 0.f ? -r_u2f(0x7F800000u) : r_u2f(0x7FC00000u);
    if (x == r_u2f(0x7F800000u))
        return x;
    int32_t e = 0;
    if (x < 1.17549435e-38f) { x = x * 16777216.f; e = -24; }
    uint32_t b = r_f2u(x);
    e += (int32_t)((b >> 23) & 0xFFu) - 127;
    float m = r_u2f((b & 0x007FFFFFu) | 0x3F800000u);
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    float f = m - 1.f, s = f / (2.f + f), z = s * s;
    float q = 0.111111111f;
    q = q * z + 0.142857143f;
    q = q * z + 0.2f;
    q = q * z + 0.333333333f;
    q = q * z + 1.f;
    float lnm = 2.f * s * q, ef = (float)e;
    return ef * 0.693145752f + (lnm + ef * 1.42860677e-06f);
}

static float r_exp(float x)
{
    if (x != x) return x;
    if (x > 88.7228394f) return r_u2f(0x7F800000u);
    if (x < -87.3365479f) return 0.f;
    float kf = floorf(x * 1.44269504f + 0.5f);
    float r = (x - kf * 0.693145752f) - kf * 1.42860677e-06f;
    float q = 1.98412698e-04f;
    q = q * r + 1.38888889e-03f;
    q = q * r + 8.33333333e-03f;
    q = q * r + 4.16666667e-02f;
    q = q * r + 1.66666667e-01f;
    q = q * r + 0.5f;
    q = q * r + 1.f;
    q = q * r + 1.f;
    int32_t k = (int32_t)kf;
    if (k < -126) { q = q * r_u2f((uint32_t)(k + 126 + 127) << 23); return q * 1.17549435e-38f; }
    if (k > 127) return r_u2f(0x7F800000u);
    return q * r_u2f((uint32_t)(k + 127) << 23);
}

static float r_pow(float x, float y)
{
    if (x == 0.f) return y > 0.f ? 0.f : (y == 0.f ? 1.f : r_u2f(0x7F800000u));
    if (x == 1.f || y == 0.f) return 1.f;
    return r_exp(y * r_ln(x));
}

static void r_sincos(float a, float* s, float* c)
{
    float kf = floorf(a * 0.636619772f + 0.5f);
    float r = (a - kf * 1.57079601f) - kf * 3.13916473e-07f;
    float z = r * r;
    float ps = -1.98412698e-04f;
    ps = ps * z + 8.33333333e-03f;
    ps = ps * z - 1.66666667e-01f;
    float sr = r + r * z * ps;
    float pc = 2.48015873e-05f;
    pc = pc * z - 1.38888889e-03f;
    pc = pc * z + 4.16666667e-02f;
    float cr = (1.f - 0.5f * z) + z * z * pc;
    int32_t q = (int32_t)kf & 3;
    if (q == 0) { *s = sr; *c = cr; }
    else if (q == 1) { *s = cr; *c = -sr; }
    else if (q == 2) { *s = -sr; *c = -cr; }
    else { *s = -cr; *c = sr; }
}

typedef struct { uint64_t state, inc; } r_rng;
static r_rng r_rng_make(uint32_t pixel, uint32_t frame)
{
    r_rng g;
    g.inc = (vko_splitmix64((uint64_t)pixel ^ 0xD1B54A32D192ED03ull) << 1) | 1ull;
    g.state = vko_splitmix64(((uint64_t)frame << 32) ^ pixel);
    return g;
}
static uint32_t r_rng_u32(r_rng* g)
{
    uint64_t old = g->state;
    g->state = old * 6364136223846793005ull + g->inc;
    uint32_t x = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (x >> rot) | (x << ((32u - rot) & 31u));
}
static float r_rng_next(r_rng* g) { return (float)(r_rng_u32(g) >> 8) * 5.96046448e-08f; }

typedef struct { float x, y, z; } r_v3;
static r_v3 rv(float x, float y, float z) { r_v3 r = {x, y, z}; return r; }
static r_v3 rv_add(r_v3 a, r_v3 b) { return rv(a.x + b.x, a.y + b.y, a.z + b.z); }
static r_v3 rv_sub(r_v3 a, r_v3 b) { return rv(a.x - b.x, a.y - b.y, a.z - b.z); }
static r_v3 rv_scale(r_v3 a, float s) { return rv(a.x * s, a.y * s, a.z * s); }
static r_v3 rv_mul(r_v3 a, r_v3 b) { return rv(a.x * b.x, a.y * b.y, a.z * b.z); }
static r_v3 rv_div(r_v3 a, r_v3 b) { return rv(a.x / b.x, a.y / b.y, a.z / b.z); }
static float rv_dot(r_v3 a, r_v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static r_v3 rv_norm(r_v3 a) { return rv_scale(a, 1.f / sqrtf(rv_dot(a, a))); }
static r_v3 rv_arr(const float* a) { return rv(a[0], a[1], a[2]); }

typedef struct { float tnear, tfar; int hit; } r_hit;
static r_hit r_intersect(r_v3 ori, r_v3 dir, r_v3 box)
{
    r_v3 inv = rv(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    r_v3 t1 = rv_mul(rv(0.f - ori.x, 0.f - ori.y, 0.f - ori.z), inv);
    r_v3 t2 = rv_mul(rv_sub(box, ori), inv);
    r_hit h;
    h.tnear = fmaxf(fmaxf(fminf(t1.x, t2.x), fminf(t1.y, t2.y)), fminf(t1.z, t2.z));
    h.tfar = fminf(fminf(fmaxf(t1.x, t2.x), fmaxf(t1.y, t2.y)), fmaxf(t1.z, t2.z));
    h.hit = h.tnear <= h.tfar;
    return h;
}

/* texture_ref filter Nearest, address Clamp (Render.cpp:446-447) */
static int32_t r_tex_index(float c, int32_t n)
{
    float f = c * (float)n;
    if (!(f >= 0.f)) f = 0.f;
    float hi = (float)(n - 1);
    if (f > hi) f = hi;
    return (int32_t)floorf(f);
}

static float r_texel(const vko_volume* v, r_v3 c)
{
    size_t i = ((size_t)r_tex_index(c.z, v->dims[2]) * (size_t)v->dims[1] + (size_t)r_tex_index(c.y, v->dims[1])) *
                   (size_t)v->dims[0] + (size_t)r_tex_index(c.x, v->dims[0]);
    if (v->fmt == 4) return (float)v->data[i] / 255.f;   /* unorm<8> */
    if (v->fmt == 5) { uint16_t u; memcpy(&u, v->data + 2 * i, 2); return (float)u / 65535.f; }
    float f; memcpy(&f, v->data + 4 * i, 4);
    return (f - v->lo) / (v->hi - v->lo);
}

static void r_lut(const vko_render_params* p, float val, float out[4])
{
    int32_t i = r_tex_index(val, p->lut_size);
    for (int k = 0; k < 4; ++k) out[k] = p->lut[4 * i + k];
}

static float r_srgb(float x) { return x <= 0.0031308f ? 12.92f * x : 1.055f * r_pow(x, 1.f / 2.4f) - 0.055f; }

static void r_sample(const vko_volume* v, const vko_render_params* p, int32_t x, int32_t y, uint32_t frame, float out[4])
{
    r_rng gen = r_rng_make((uint32_t)y * (uint32_t)p->width + (uint32_t)x, frame);
    float jx = r_rng_next(&gen), jy = r_rng_next(&gen);
    float sx = 2.f * ((float)x + jx) / (float)p->width - 1.f;
    float sy = 2.f * ((float)y + jy) / (float)p->height - 1.f;
    r_v3 W = rv_arr(p->W);
    r_v3 dir = rv_norm(rv_add(rv_add(W, rv_scale(rv_arr(p->U), sx)), rv_scale(rv_arr(p->V), sy)));
    r_v3 ori = rv_arr(p->eye);
    float lu = r_rng_next(&gen), lv = r_rng_next(&gen);
    if (p->lens_radius > 0.f) {
        r_v3 focus = rv_add(ori, rv_scale(dir, p->focal_distance / rv_dot(dir, W)));
        float r = p->lens_radius * sqrtf(lu), s, c;
        r_sincos(6.28318531f * lv, &s, &c);
        ori = rv_add(rv_add(ori, rv_scale(rv_arr(p->right), r * c)), rv_scale(rv_arr(p->up), r * s));
        dir = rv_norm(rv_sub(focus, ori));
    }
    r_v3 box = rv_arr(p->bbox);
    r_hit h = r_intersect(ori, dir, box);
    out[0] = out[1] = out[2] = out[3] = 0.f;
    if (p->algo == 0) { /* RayMarchingKernel, :80-158 */
        float t = h.tnear;
        r_v3 tc = rv_div(rv_add(ori, rv_scale(dir, t)), box);
        r_v3 inc = rv_div(rv_scale(dir, p->dt_ray_marching), box);
        float dst[4] = {0.f, 0.f, 0.f, 0.f};
        while (t < h.tfar) {
            float voxel = r_texel(v, tc), col[4];
            if (p->lut) r_lut(p, voxel, col); else col[0] = col[1] = col[2] = col[3] = voxel;
            col[3] = 1.f - r_pow(1.f - col[3], p->dt_ray_marching);
            col[0] *= col[3]; col[1] *= col[3]; col[2] *= col[3];
            float rem = 1.f - dst[3];
            for (int k = 0; k < 4; ++k) dst[k] += col[k] * rem;
            if (dst[3] == 1.f) break;
            tc = rv_add(tc, inc);
            t += p->dt_ray_marching;
        }
        for (int k = 0; k < 4; ++k) out[k] = dst[k];
        return;
    }
    if (p->algo == 1) { /* ImplicitIsoKernel, :164-268 */
        float t = h.tnear, last = -1e20f, isoT = -1e20f;
        r_v3 tc = rv_div(rv_add(ori, rv_scale(dir, t)), box);
        r_v3 inc = rv_div(rv_scale(dir, p->dt_implicit_iso), box);
        float dst[4] = {0.f, 0.f, 0.f, 0.f};
        while (t < h.tfar) {
            float voxel = r_texel(v, tc);
            if (last >= -1e10f) {
                for (int32_t i = 0; i < p->num_iso; ++i) {
                    float iso = p->iso[i];
                    if ((last <= iso && voxel >= iso) || (last >= iso && voxel <= iso)) {
                        float col[4], d = 0.01f;
                        if (p->lut) r_lut(p, voxel, col); else col[0] = col[1] = col[2] = col[3] = voxel;
                        isoT = t;
                        r_v3 s1 = rv(r_texel(v, rv_add(tc, rv(d, 0.f, 0.f))), r_texel(v, rv_add(tc, rv(0.f, d, 0.f))),
                                     r_texel(v, rv_add(tc, rv(0.f, 0.f, d))));
                        r_v3 s2 = rv(r_texel(v, rv_sub(tc, rv(d, 0.f, 0.f))), r_texel(v, rv_sub(tc, rv(0.f, d, 0.f))),
                                     r_texel(v, rv_sub(tc, rv(0.f, 0.f, d))));
                        r_v3 N = rv_norm(rv_sub(s2, s1));
                        float kd = fmaxf(0.f, rv_dot(N, rv(-dir.x, -dir.y, -dir.z))) * voxel;
                        dst[0] = 0.2f + col[0] * kd;
                        dst[1] = 0.2f + col[1] * kd;
                        dst[2] = 0.2f + col[2] * kd;
                        dst[3] = 1.f;
                    }
                }
            }
            if (isoT >= -1e10f) break;
            tc = rv_add(tc, inc);
            t += p->dt_implicit_iso;
            last = voxel;
        }
        for (int k = 0; k < 4; ++k) out[k] = dst[k];
        return;
    }
    /* MultiScatteringKernel, :276-418 */
    r_v3 thr = rv(1.f, 1.f, 1.f);
    float mu_ = p->majorant;
    if (h.hit) {
        ori = rv_add(ori, rv_scale(dir, h.tnear));
        h.tfar -= h.tnear;
        uint32_t bounce = 0;
        for (;;) {
            float t = 0.f;
            r_v3 pos;
            int interact;
            for (;;) { /* sample_interaction, :320-341 */
                t -= r_ln(1.f - r_rng_next(&gen)) / mu_;
                pos = rv_add(ori, rv_scale(dir, t));
                if (t >= h.tfar) { interact = 0; break; }
                float voxel = r_texel(v, rv_div(pos, box)), mu;
                if (p->lut) { float col[4]; r_lut(p, voxel, col); mu = col[3]; } else mu = voxel;
                if (!(mu < r_rng_next(&gen) * mu_)) { interact = 1; break; }
            }
            if (!interact) break;
            ori = pos;
            if (bounce++ >= 1024) { thr = rv(0.f, 0.f, 0.f); break; }
            float voxel = r_texel(v, rv_div(ori, box));
            r_v3 alb;
            if (p->lut) { float col[4]; r_lut(p, voxel, col); alb = rv(col[0], col[1], col[2]); }
            else alb = rv(voxel, voxel, voxel);
            thr = rv_mul(thr, alb);
            float prob = fmaxf(fmaxf(thr.x, thr.y), thr.z);
            if (prob < 0.2f) {
                if (r_rng_next(&gen) > prob) { thr = rv(0.f, 0.f, 0.f); break; }
                thr = rv(thr.x / prob, thr.y / prob, thr.z / prob);
            }
            float cz = 1.f - 2.f * r_rng_next(&gen);
            float sr = sqrtf(fmaxf(0.f, 1.f - cz * cz)), s, c;
            r_sincos(6.28318531f * r_rng_next(&gen), &s, &c);
            dir = rv(sr * c, sr * s, cz);
            h = r_intersect(ori, dir, box);
        }
    }
    float ty = (float)y / (float)p->height;
    out[0] = ((1.f - ty) * 1.f + ty * 0.5f) * thr.x;
    out[1] = ((1.f - ty) * 1.f + ty * 0.7f) * thr.y;
    out[2] = ((1.f - ty) * 1.f + ty * 1.0f) * thr.z;
    out[3] = 1.f;
}

/* Pixels [x0, x1) x [y0, y1) only (accum / color keep the full-viewport layout): full-size
 * frames (config 5, 1024^2) are checked on windows -- every pixel is independent (its own
 * random sequence, Render_kernel.hpp per-pixel kernels), so a window equals the same pixels of
 * the full frame. */
void vko_render_window(const vko_volume* v, const vko_render_params* p, float* accum, float* color,
                       int32_t num_frames, int32_t x0, int32_t y0, int32_t x1, int32_t y1)
{
    if (x0 < 0) x0 = 0;
    if (y0 < 0) y0 = 0;
    if (x1 > p->width) x1 = p->width;
    if (y1 > p->height) y1 = p->height;
    for (int32_t y = y0; y < y1; ++y)
        for (int32_t x = x0; x < x1; ++x) {
            size_t pix = (size_t)y * (size_t)p->width + (size_t)x;
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            if (p->frame_begin > 0)
                for (int k = 0; k < 4; ++k) acc[k] = accum[4 * pix + k];
            for (int32_t f = 1; f <= num_frames; ++f) {
                uint32_t frame = p->frame_begin + (uint32_t)f;
                float s[4];
                r_sample(v, p, x, y, frame, s);
                float alpha = 1.f / (float)frame; /* AccumulationKernel::accum */
                for (int k = 0; k < 4; ++k) acc[k] = (1.f - alpha) * acc[k] + alpha * s[k];
            }
            for (int k = 0; k < 4; ++k) accum[4 * pix + k] = acc[k];
            if (color) {
                for (int k = 0; k < 3; ++k) color[4 * pix + k] = p->srgb ? r_srgb(acc[k]) : acc[k];
                color[4 * pix + 3] = acc[3];
            }
        }
}

void vko_render(const vko_volume* v, const vko_render_params* p, float* accum, float* color, int32_t num_frames)
{
    vko_render_window(v, p, accum, color, num_frames, 0, 0, p->width, p->height);
}

/* ---- synthetic input -------------------------------------------------------------- */
uint64_t vko_splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void vko_synth(uint8_t* data, size_t nbytes, uint64_t seed)
{
    size_t words = nbytes / 8;
    for (size_t w = 0; w < words; ++w) {
        uint64_t r = vko_splitmix64(seed + w);
        memcpy(data + 8 * w, &r, 8);
    }
    if (nbytes % 8) {
        uint64_t r = vko_splitmix64(seed + words);
        memcpy(data + 8 * words, &r, nbytes % 8);
    }
}
