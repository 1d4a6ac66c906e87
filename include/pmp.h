/*
 * pmp.h -- C-ABI of libpmp_hip.so, the MI355X (gfx950) batched motion-planning core.
 *
 * The reference (Slenderman00/python_motion_planning, pure Python) has no FFI of its own; the
 * boundary it exposes for the hot path is the Planner plug-in API:
 *     Planner.plan() (utils/planner/planner.py:28-33), SearchFactory (search_factory.py:13-51),
 *     ControlFactory (control_factory.py:13-27) and one iteration of LocalPlanner.plan loops.
 * Each entry point below replaces the inner loop of one reference call; the Python host package
 * python_motion_planning_amd binds them with ctypes.
 *
 * Conventions
 *  - Every array pointer is a DEVICE pointer owned by the caller (e.g. torch tensor.data_ptr()),
 *    contiguous, with the dtype written in the signature.  The library never frees caller memory
 *    and allocates only grow-only scratch inside its pmp_ctx.
 *  - Calls are asynchronous on `stream` (a hipStream_t; NULL = default stream).
 *  - Return value: 0 = OK, PMP_EINVAL / PMP_ENOMEM / PMP_EHIP < 0; text via pmp_last_error().
 *  - Per-query status: 0 found, 1 no path, 2 path_cap overflow, 3 heap/expand/capacity overflow,
 *    4 "the reference raises" (D* unreachable -> AttributeError at d_star.py:234).
 *  - Grid cells: occupancy bit-packed x-major, cell id c = x*H + y, bit c at word c>>5, bit c&31
 *    (utils/environment/env.py:41-80 stores obstacles as (x, y) tuples).
 *  - A pmp_ctx must not be used by two host threads at once.
 */
#ifndef PMP_H
#define PMP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PMP_OK 0
#define PMP_EINVAL (-1)
#define PMP_ENOMEM (-2)
#define PMP_EHIP (-3)

#define PMP_FOUND 0
#define PMP_NO_PATH 1
#define PMP_PATH_OVERFLOW 2
#define PMP_CAP_OVERFLOW 3
#define PMP_REF_RAISES 4

typedef struct pmp_ctx pmp_ctx;

/* Create a context bound to HIP device `device`; NULL on failure. */
pmp_ctx* pmp_create(int device);
void pmp_destroy(pmp_ctx* ctx);
const char* pmp_last_error(pmp_ctx* ctx);
/* Library version string (static). */
const char* pmp_version(void);

/*
 * Batched 2D A*.  Replaces AStar.plan (global_planner/graph_search/a_star.py:39-83) with its
 * getNeighbor (:85-96), GraphSearcher.h / isCollision (graph_search.py:30-87), CPython heapq
 * ordered by Node.__lt__ (utils/environment/node.py:51-54) and extractPath (:98-117).
 *   occ_bits   [ceil(W*H/32)] u32   shared occupancy of the Grid
 *   heuristic  0 euclidean, 1 manhattan
 *   start_xy, goal_xy  [nq][2] i32
 *   cost       [nq] f64             path cost (sum of hypot, goal->start order)
 *   path_len   [nq] i32             number of cells on the path (goal->start, reference order)
 *   path       [nq][path_cap] u32   cell ids, goal first
 *   n_expanded [nq] i32             len(CLOSED) == len(expand) of the reference
 *   expand     [nq][expand_cap] u32 nullable; CLOSED in insertion order, cell | parent_dir<<28
 *              (parent_dir = motion index of env.py:52-55 that reached the cell, 8 = start)
 *   counters   [nq][4] i64          nullable; pushes, pops, expansions, max heap size
 *   status     [nq] i32
 * W, H <= 8192.  Cells outside [0,W)x[0,H) are blocked (the reference relies on boundary walls).
 */
int pmp_astar2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                      const int32_t* start_xy, const int32_t* goal_xy, int nq, double* cost,
                      int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded,
                      uint32_t* expand, int expand_cap, int64_t* counters, int32_t* status);

/* Pre-size the A* scratch (heap of heap_cap entries per concurrent query, up to max_slots
 * concurrent queries) so that later batch calls allocate nothing (hipGraph-capturable). */
int pmp_astar2d_reserve(pmp_ctx* ctx, int W, int H, int max_slots, int heap_cap);

#ifdef __cplusplus
}
#endif
#endif /* PMP_H */
