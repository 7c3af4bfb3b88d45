/*
 * vkt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the volkit reference's *serial CPU* path for the
 * StructuredVolume core algorithms.  It is the parity checker for the HIP backend and
 * the timed CPU baseline in bench.py ("kind": "port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library never links it.
 *
 * Parity pinning: the reference cannot be built here without writing a stand-in for its
 * CMake-generated vkt/config.h (included by src/vkt/macros.hpp:4), which this project's
 * rules forbid, and the reference ships no tests or fixtures.  This restatement is pinned
 * by the known-answer vectors that the survey recorded from the compiled reference
 * (transcribed into tests/golden/reference_kat.json), i.e. parity
 * is only partially pinned -- see DESIGN.md §3.
 */
#ifndef VKT_ORACLE_H
#define VKT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One dense x-fastest volume (reference src/vkt/StructuredVolume.cpp:311-317). */
typedef struct {
    uint8_t* data;
    int32_t dims[3];
    int32_t fmt;         /* vktDataFormat value */
    float lo, hi;        /* voxel mapping */
    size_t nbytes;       /* size of data; reads past the end are clamped to the last voxel */
} vko_volume;

typedef void (*vko_unary_op)(int32_t x, int32_t y, int32_t z, uint8_t* bytes, int32_t fmt, float lo, float hi);
typedef void (*vko_binary_op)(int32_t x, int32_t y, int32_t z, uint8_t* bytes1, int32_t fmt1, float lo1,
                              float hi1, uint8_t* bytes2, int32_t fmt2, float lo2, float hi2);

uint32_t vko_bytes_per_voxel(int32_t fmt);
void vko_map(uint8_t* dst, float value, int32_t fmt, float lo, float hi);
void vko_unmap(float* value, const uint8_t* src, int32_t fmt, float lo, float hi);

void vko_fill_range(vko_volume* v, const int32_t first[3], const int32_t last[3], float value);
void vko_copy_range(vko_volume* dst, vko_volume* src, const int32_t first[3], const int32_t last[3],
                    const int32_t dst_offset[3]);
/* op: 0 Sum, 1 Diff, 2 Prod, 3 Quot, 4 AbsDiff, 5..9 the Safe variants */
void vko_arith_range(int32_t op, vko_volume* dst, vko_volume* s1, vko_volume* s2, const int32_t first[3],
                     const int32_t last[3], const int32_t dst_offset[3]);
/* filter: 0 Nearest, 1 Linear */
void vko_resample(vko_volume* dst, vko_volume* src, int32_t filter);
/* Z-slab form used to check the multi-GPU path: dst holds global planes [dst_z0, ...) of a
 * volume of depth dst_gdz; src holds global planes [src_z0, ...) of depth src_gdz. */
void vko_resample_slab(vko_volume* dst, vko_volume* src, int32_t filter, int32_t dst_gdz, int32_t dst_z0,
                       int32_t src_gdz, int32_t src_z0);
void vko_transform_range1(vko_volume* v, const int32_t first[3], const int32_t last[3], vko_unary_op op);
void vko_transform_range2(vko_volume* v1, vko_volume* v2, const int32_t first[3], const int32_t last[3],
                          const int32_t v2_offset[3], vko_binary_op op);

/* ComputeAggregatesRange_serial, reference src/vkt/Aggregates_serial.hpp:20-83 (float
 * accumulation in z->y->x order, mean/var divided by the WHOLE volume's voxel count). */
typedef struct {
    float min, max, mean, stddev, var, sum, prod;
    int32_t argmin[3], argmax[3];
} vko_aggregates;
void vko_aggregates_range(const vko_volume* v, const int32_t first[3], const int32_t last[3], vko_aggregates* out);
/* ComputeHistogramRange_serial, reference src/vkt/Histogram_serial.hpp:20-50.  Voxels whose
 * bin index the reference would write out of bounds (UB) are not counted; their number is
 * returned. */
uint64_t vko_histogram_range(const vko_volume* v, const int32_t first[3], const int32_t last[3], uint64_t* bins,
                             uint64_t num_bins);

/* Renderers of reference src/vkt/Render_kernel.hpp:80-418 (RayMarching, ImplicitIso,
 * MultiScattering), one sample per pixel and frame, accumulated like AccumulationKernel::accum.
 * Layout of the parameter block = vktHipRenderParams_t (include/volkit_hip.h).  Camera rays,
 * RNG (PCG32 per pixel and frame) and ln/exp/pow/sincos are restated from this project's
 * common/RenderMath.hpp: the visionaray sequences of the reference are unpinned. */
typedef struct {
    int32_t algo, width, height;
    uint32_t frame_begin;
    float eye[3], U[3], V[3], W[3], right[3], up[3];
    float lens_radius, focal_distance;
    float bbox[3];
    float dt_ray_marching, dt_implicit_iso, majorant;
    int32_t num_iso;
    float iso[10];
    int32_t srgb;
    const float* lut;
    int32_t lut_size;
} vko_render_params;
/* accum / color: width*height*4 floats (row 0 = bottom); accum read when frame_begin > 0 */
void vko_render(const vko_volume* v, const vko_render_params* p, float* accum, float* color, int32_t num_frames);
void vko_render_window(const vko_volume* v, const vko_render_params* p, float* accum, float* color,
                       int32_t num_frames, int32_t x0, int32_t y0, int32_t x1, int32_t y1);

/* Synthetic input shared with the GPU generator (include/volkit_hip.h vktHipSynthesize). */
uint64_t vko_splitmix64(uint64_t x);
void vko_synth(uint8_t* data, size_t nbytes, uint64_t seed);

#ifdef __cplusplus
}
#endif

#endif
