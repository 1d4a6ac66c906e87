// Grid helpers shared by the 2D graph-search engines (astar2d.hip, astar2d_mq.hip): the occupancy
// bit of a cell and Theta* / Lazy Theta*'s Bresenham line of sight (theta_star.py:110-171).
#pragma once
#include <cstdint>

namespace grid2d {

// ThetaStar.lineOfSight (theta_star.py:110-171): Bresenham from (x1, y1) to (x2, y2) over the bit
// grid; tau = (d_y - d_x) / 2 is compared as 2e against d_y - d_x.  Both endpoints are in the grid
// (they are cells the search reached), so the line stays inside its bounding box.  The step bound
// is never reached by the reference's loop; it only guarantees termination.
__device__ __forceinline__ bool occ_bit(const uint32_t* occ, int H, int x, int y)
{
    const uint32_t ci = (uint32_t)x * (uint32_t)H + (uint32_t)y;
    return ((occ[ci >> 5] >> (ci & 31u)) & 1u) != 0u;
}
__device__ inline bool los2d(const uint32_t* occ, int H, int x1, int y1, int x2, int y2)
{
    if (occ_bit(occ, H, x1, y1) || occ_bit(occ, H, x2, y2)) return false;
    const int dx = abs(x2 - x1), dy = abs(y2 - y1);
    const int sx = x2 > x1 ? 1 : (x2 < x1 ? -1 : 0), sy = y2 > y1 ? 1 : (y2 < y1 ? -1 : 0);
    int x = x1, y = y1, e = 0;
    const bool xmaj = dx > dy;
    const int T = xmaj ? dy - dx : dx - dy;
    const int du = xmaj ? dx : dy, dv = xmaj ? dy : dx;  // major / minor deltas
    // The cells a line visits do not depend on the grid, so 8 steps are generated first and their
    // 8 bit loads issued as one round (one memory latency per 8 cells instead of per cell); the
    // first blocked cell in step order decides, as in the reference's loop.
    constexpr int kB = 8;
    for (int it = 0; it <= dx + dy + 1; it += kB) {
        uint32_t ci[kB];
        int nv = 0;
#pragma unroll
        for (int j = 0; j < kB; j++) {
            const bool go = !(xmaj ? x == x2 : y == y2);
            if (go) {
                const bool maj = 2 * e >= T, mino = 2 * e <= T;  // e > tau: major; e < tau: minor; equal: both
                if (maj) {
                    if (xmaj) x += sx; else y += sy;
                }
                if (mino) {
                    if (xmaj) y += sy; else x += sx;
                }
                e += (maj ? -dv : 0) + (mino ? du : 0);
                nv++;
            }
            ci[j] = go ? (uint32_t)x * (uint32_t)H + (uint32_t)y : ~0u;
        }
        uint32_t wv[kB];
#pragma unroll
        for (int j = 0; j < kB; j++) wv[j] = ci[j] != ~0u ? occ[ci[j] >> 5] : 0u;
#pragma unroll
        for (int j = 0; j < kB; j++)
            if (ci[j] != ~0u && ((wv[j] >> (ci[j] & 31u)) & 1u)) return false;
        if (nv < kB || (xmaj ? x == x2 : y == y2)) return true;
    }
    return false;
}

}  // namespace grid2d
