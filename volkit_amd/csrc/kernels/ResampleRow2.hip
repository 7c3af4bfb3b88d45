// ResampleRow2.hip -- row kernel instantiations, MODE 2 (Float32 source, lerp chain).
#include "ResampleRow.hpp"

namespace vkt
{
namespace hipk
{
    void launchRowMode2(ResampleArgs const& a, int32_t k, uint32_t bpvd, unsigned grid, int32_t instrPerRow,
                        hipStream_t s)
    {
        if (bpvd == 4)
            launchRowK<4, 4, 2, codec::FmtFloat32, -1>(a, k, grid, instrPerRow, s);
        else if (bpvd == 2)
            launchRowK<4, 2, 2, codec::FmtFloat32, -1>(a, k, grid, instrPerRow, s);
        else
            launchRowK<4, 1, 2, codec::FmtFloat32, -1>(a, k, grid, instrPerRow, s);
    }
    __global__ __launch_bounds__(256) void resampleFixupScanKernel(ResampleArgs a, uint32_t* list)
    {
        uint32_t const nY = static_cast<uint32_t>(a.nRunsY), nZ = static_cast<uint32_t>(a.nRunsZ);
        uint32_t const t = blockIdx.x * blockDim.x + threadIdx.x;
        if (t >= nY * nZ)
            return;
        uint32_t const iz = t / nY, iy = t - iz * nY;
        if (taskFlagged(a, runY(a, iy), runZ(a, iz)))
        {
            uint32_t const slot = atomicAdd(&list[0], 1u);
            list[1 + slot] = t;
        }
    }

    void launchLinearOptimistic(ResampleArgs const& a, int32_t k, uint32_t bpvd, int32_t instrPerRow, uint32_t* list,
                                hipStream_t s)
    {
        uint64_t const tasks = static_cast<uint64_t>(a.dnz) * a.nRunsY * static_cast<uint64_t>(instrPerRow);
        uint64_t const fixTasks = static_cast<uint64_t>(a.nRunsY) * a.nRunsZ;
        unsigned const gs = static_cast<unsigned>((fixTasks + 255) / 256);
        unsigned const gf = 2048;   // drains the work list (exits at once when it is empty)
#define VKT_OPT_F(B, K, FD)                                                                                     \
    do {                                                                                                        \
        planeChunks(a, tasks, [&](ResampleArgs const& c, unsigned g) {                                         \
            hipLaunchKernelGGL((resamplePlaneKernel<4, B, K, 3, codec::FmtFloat32, FD>), dim3(g), dim3(64), 0, s, c); \
        });                                                                                                     \
        hipLaunchKernelGGL(resampleFixupScanKernel, dim3(gs), dim3(256), 0, s, a, list);                     \
        hipLaunchKernelGGL((resampleFixupKernel<B, K>), dim3(gf), dim3(64), 0, s, a, list);                   \
    } while (0)
    // Float32 destinations (config 3) get the encode with the format fixed at compile time
#define VKT_OPT(B, K)                                                                                           \
    do {                                                                                                        \
        if (B == 4 && a.fd == codec::FmtFloat32) VKT_OPT_F(B, K, codec::FmtFloat32);                            \
        else VKT_OPT_F(B, K, -1);                                                                               \
    } while (0)
#define VKT_OPT_K(B)                            \
    do {                                        \
        if (k == 1) { if constexpr (16 / B >= 1 && (16 / B) * 4 <= 32) VKT_OPT(B, 1); } \
        else if (k == 2) VKT_OPT(B, 2);         \
        else VKT_OPT(B, 4);                     \
    } while (0)
        if (bpvd == 4)
            VKT_OPT_K(4);
        else if (bpvd == 2)
            VKT_OPT_K(2);
        else
            VKT_OPT_K(1);
#undef VKT_OPT_K
#undef VKT_OPT
#undef VKT_OPT_F
    }
} // hipk
} // vkt
