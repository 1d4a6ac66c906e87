// Internal helpers shared by the gfx950 kernels of libpmp_hip.so (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/pmp.h"

struct pmp_ctx {
    int device = 0;
    std::string err;
    // A* scratch geometry (pmp_astar2d_reserve)
    int astar_W = 0, astar_H = 0, astar_workers = 0, astar_heap_cap = 0, astar_lds_cap = 0;
    // optional launch-span recording (pmp_set_timing): device u64[2] = {min start, max end}
    unsigned long long* span = nullptr;
    // optional work counters (pmp_set_stats): device i64, [0] += MPC QP solves of track launches
    unsigned long long* stats = nullptr;
    // A* 2D query scheduling: 1 = longest (start-goal distance) first, 0 = input order
    int astar_lpt = 1;
    // longest-first only: how many of the first (longest) queries run at raised wave priority
    int astar_prio_n = 64;
    // A* 2D workers resident per CU over all concurrent launches (0 = ceil(workers / 256)): sets the LDS heap share
    int astar_resident_per_cu = 0;
    // one-wave-per-query planners (3D A* family, D*): persistent workers per CU (0 = each one's default)
    int workers_per_cu = 0;
    // D* 2D: the first pass's heap / entry capacity (0 = one per cell + 64; pmp_dstar_set_first_cap)
    int dstar_first_cap = 0;
    // ... and the workers resident per CU over all concurrent launches, which sets their LDS share
    // (0 = this launch's own workers per CU; pmp_set_resident_per_cu)
    int resident_per_cu = 0;
    // A* 2D engine: 2 = several queries per wave (astar2d_mq.hip) for A* / Dijkstra / GBFS whose heaps fit
    // its capacity, 1 = that for large batches on large grids and the single-query engine
    // (astar2d_sq.hip) for batches of at most 256, 3 = the single-query engine whenever it holds the
    // heap, 0 = one query per wave (astar2d.hip) always (pmp_astar2d_set_engine); the multi-query engine's tier-2
    // direction bits in LDS (1) or HBM (0); the geometry its per-slot epochs were written for
    int astar_engine = 1;
    int astar_mq_t2lds = 0;
    int astar_heap_cap_wave = 0;  // heap capacity of one-query-per-wave launches on a multi-query reservation
    int astar_cap_explicit = 0;   // the reservation's heap capacity was asked for (not the default)
    int astar_reserved_mq = 0;  // the current reservation (pmp_astar2d_reserve) is the multi-query engine's
    int astar_auto = 0;         // ... and was made by a launch (not the host): it grows with the batches
    size_t astar_mq_epoch_slots = 0, astar_mq_cst_bytes = 0;
    // grow-only scratch arena, one buffer per use
    void* buf[24] = {nullptr};
    size_t cap[24] = {0};
    // DWA k-split (dwa.hip): the per-agent arrival counters in SCR_DWA were zeroed for this buffer
    void* dwa_zeroed = nullptr;
    int dwa_zeroed_n = 0;
    // DWA parts per agent (pmp_dwa_set_split): 0 auto, 1 off, k
    int dwa_split = 0;
    int cus = 0;  // compute units of the device (0 = not queried yet)
};

enum ScratchSlot { SCR_HEAP = 0, SCR_CLOSED = 1, SCR_PDIR = 2, SCR_G = 3, SCR_AUX0 = 4, SCR_AUX1 = 5, SCR_AUX2 = 6, SCR_AUX3 = 7,
                   SCR_BITS = 8, SCR_AUX4 = 9, SCR_PAR = 10, SCR_MQ_SPILL = 11, SCR_MQ_CST = 12, SCR_MQ_G = 13,
                   SCR_MQ_T2 = 14, SCR_MQ_EPOCH = 15, SCR_DWA = 16, SCR_MQ_PC = 17, SCR_DSTAR_OVF = 18, SCR_NSLOTS = 19 };

int pmp_set_err(pmp_ctx* ctx, int code, const std::string& msg);
// Workers per CU whose LDS shares a launch of `per_cu` workers per CU must fit beside
inline int pmp_lds_share(const pmp_ctx* ctx, int per_cu) { return ctx->resident_per_cu > per_cu ? ctx->resident_per_cu : per_cu; }
// Heap positions kept in LDS (a multiple of 16) when each of the `pmp_lds_share` workers of a CU
// gets an equal share of its 160 KiB and `fixed_bytes` of that share hold other LDS data (occupancy
// bits, ...).  Below kMinLdsHeap the share cannot hold the kernel's fixed LDS needs: the caller
// moves the fixed data to HBM or refuses the launch (never a negative size: the dynamic LDS size
// would wrap and the kernel would address outside its allocation).
constexpr int kMinLdsHeap = 16;
inline int pmp_heap_lds_cap(const pmp_ctx* ctx, int per_cu, int fixed_bytes, int entry_bytes)
{
    const int bytes = (160 * 1024) / pmp_lds_share(ctx, per_cu) - 256 - fixed_bytes;
    return bytes < kMinLdsHeap * entry_bytes ? 0 : (bytes / entry_bytes) & ~15;
}
// Ensure scratch buffer `slot` holds at least `bytes`; returns device pointer or nullptr (error set).
void* pmp_scratch(pmp_ctx* ctx, int slot, size_t bytes);

// Longest-first order of a 3D batch (descending start-goal distance, counting sort on `s`) in the
// context's SCR_PDIR scratch; *order = nullptr when the schedule is off or every query has its own
// worker (nq <= workers).  Shared by the one-wave-per-query 3D planners (astar3d.hip).
int pmp_lpt_order3d(pmp_ctx* ctx, hipStream_t s, const int32_t* start_xyz, const int32_t* goal_xyz, int nq, int X,
                    int Y, int Z, int workers, int32_t** order);

// The multi-query A* 2D engine (astar2d_mq.hip), driven by pmp_graph2d_batch (astar2d.hip).
int pmp_astar2d_mq_launch(pmp_ctx* ctx, hipStream_t s, int algo, const uint32_t* occ_bits, int W, int H, int heuristic,
                          const int32_t* start_xy, const int32_t* goal_xy, const int32_t* order, int nq, double* cost,
                          int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded, uint32_t* expand,
                          int expand_cap, int64_t* counters, int32_t* status, int* queue);
int pmp_astar2d_mq_lds_cap(int per_cu, bool t2lds);
// the multi-query engine keeps 3-4x more queries in flight (9.5 MB of cell state, g and heap spill
// each at 1024^2; Theta* another 4 MB of CLOSED parents): its per-context scratch budget
constexpr size_t kScratchBudgetMq = (size_t)160 << 30;
int pmp_astar2d_slot_scratch(pmp_ctx* ctx, hipStream_t s, size_t slots, int W, int H, uint8_t** cst, size_t* cst_bytes,
                             double** G, uint32_t** ep);
// The single-query A* 2D engine (astar2d_sq.hip): one query per workgroup, the CU's LDS its heap.
// Returns the heap capacity it can hold for this grid (0: not this engine's grid) / launches.
extern "C" int pmp_astar2d_sq_cap(int W, int H);
int pmp_astar2d_sq_launch(pmp_ctx* ctx, hipStream_t s, int algo, const uint32_t* occ_bits, int W, int H, int heuristic,
                          const int32_t* start_xy, const int32_t* goal_xy, int nq, int heap_cap, double* cost,
                          int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded, uint32_t* expand,
                          int expand_cap, int64_t* counters, int32_t* status);
int pmp_astar2d_mq_cap(bool t2lds);

#define PMP_HIP_CHECK(ctx, call)                                                                     \
    do {                                                                                             \
        hipError_t _e = (call);                                                                      \
        if (_e != hipSuccess) return pmp_set_err((ctx), PMP_EHIP, std::string(#call) + ": " + hipGetErrorString(_e)); \
    } while (0)

// ---------------------------------------------------------------------------------------------
// wave64 helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ uint32_t rl_u32(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ double rl_f64(double v, int lane) {
    uint64_t b = __double_as_longlong(v);
    uint32_t lo = rl_u32((uint32_t)b, lane), hi = rl_u32((uint32_t)(b >> 32), lane);
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Next index from a persistent-worker queue, wave-uniform.  The workgroup barrier is a convergence
// point (free for one-wave workgroups): without it the compiler may let lanes run ahead into the
// next iteration while lane 0 is still in a lane-0-only block, and then readfirstlane would read a
// lane that never fetched the index.
__device__ __forceinline__ int next_query(int* queue, int lane)
{
    __syncthreads();
    int qi = 0;
    if (lane == 0) qi = atomicAdd(queue, 1);
    return __builtin_amdgcn_readfirstlane(qi);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// Per-lane bools kept as the wave's 64-bit lane mask (SGPR pair): a select between two divergent
// bools written as `c ? a : b` is lowered through 0/1 VGPRs and v_cndmask (five VALU instructions);
// as masks it is three scalar ops.  lm() of a compare is the compare itself (its SGPR result).
typedef unsigned long long lmask;
__device__ __forceinline__ lmask lm(bool c) { return __builtin_amdgcn_ballot_w64(c); }
__device__ __forceinline__ bool lb(lmask m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

// Per-slot A* 2D cell-state bytes (astar2d_mq.hip / astar2d_sq.hip) in tiles of 8 (x) x 16 (y)
// cells: a tile is one 128-B line, so the 3x3 round of an expansion touches ~1.4 lines on average
// instead of one per grid row x-1, x, x+1 (the row-major layout, x * H + y), and an A* front's
// cells share lines in both directions.  tH = tiles along y.
#ifndef PMP_CST_TX
#define PMP_CST_TX 3  // log2 tile width along x
#endif
#ifndef PMP_CST_TY
#define PMP_CST_TY 4  // log2 tile height along y
#endif
constexpr int kCstTx = PMP_CST_TX, kCstTy = PMP_CST_TY;
__host__ __device__ inline size_t cst_tiled_bytes(int W, int H)
{
    return (size_t)((W + (1 << kCstTx) - 1) >> kCstTx) * (size_t)((H + (1 << kCstTy) - 1) >> kCstTy) *
           ((size_t)1 << (kCstTx + kCstTy));
}
__device__ __forceinline__ uint32_t cst_tiles_y(int H) { return (uint32_t)(H + (1 << kCstTy) - 1) >> kCstTy; }
__device__ __forceinline__ uint32_t cst_idx(int x, int y, uint32_t tH)
{
    return ((((uint32_t)x >> kCstTx) * tH + ((uint32_t)y >> kCstTy)) << (kCstTx + kCstTy)) +
           (((uint32_t)x & ((1u << kCstTx) - 1u)) << kCstTy) + ((uint32_t)y & ((1u << kCstTy) - 1u));
}

// Per-slot G (f64) of the multi-query engine in tiles of 4 (x) x 4 (y) cells, one 128-B line: the
// pusher's G (read at every pop) and the node's (written at its expansion) are neighbours, in one line
// for most motions (the row-major layout puts every x +- 1 neighbour in another line).  The slot stride
// (cells) covers the padded tiles; the single-query engine keeps row-major G inside the same stride.
#ifndef PMP_G_TX
#define PMP_G_TX 2  // log2 tile width along x
#endif
#ifndef PMP_G_TY
#define PMP_G_TY 2  // log2 tile height along y
#endif
constexpr int kGTx = PMP_G_TX, kGTy = PMP_G_TY;
__host__ __device__ inline size_t g_slot_cells(int W, int H)
{
    return (size_t)((W + (1 << kGTx) - 1) >> kGTx) * (size_t)((H + (1 << kGTy) - 1) >> kGTy) * ((size_t)1 << (kGTx + kGTy));
}
__device__ __forceinline__ uint32_t g_tiles_y(int H) { return (uint32_t)(H + (1 << kGTy) - 1) >> kGTy; }
__device__ __forceinline__ uint32_t g_idx(int x, int y, uint32_t tHg)
{
    return ((((uint32_t)x >> kGTx) * tHg + ((uint32_t)y >> kGTy)) << (kGTx + kGTy)) +
           (((uint32_t)x & ((1u << kGTx) - 1u)) << kGTy) + ((uint32_t)y & ((1u << kGTy) - 1u));
}

// Correctly rounded sqrt of an integer 0 <= k < 2^31: the operation sequence of LLVM's f64 sqrt
// lowering for gfx9 (rsq, two Newton-Raphson corrections of (s, h = y/2), two residual corrections),
// without its input scaling (only for x < 2^-767) and its 0 / inf class test (0 handled here), so the
// bits equal __dsqrt_rn((double)k) in 12 instead of 20 VALU instructions.
__device__ __forceinline__ double sqrt_int_rn(uint32_t k)
{
    const double x = (double)k;
    const double y = __builtin_amdgcn_rsq(x);
    const double s0 = x * y, h0 = y * 0.5;
    const double r0 = __builtin_fma(-h0, s0, 0.5);
    const double h1 = __builtin_fma(h0, r0, h0);
    const double s1 = __builtin_fma(s0, r0, s0);
    const double d0 = __builtin_fma(-s1, s1, x);
    const double s2 = __builtin_fma(d0, h1, s1);
    const double d1 = __builtin_fma(-s2, s2, x);
    const double s3 = __builtin_fma(d1, h1, s2);
    return k == 0u ? 0.0 : s3;
}

// launch-span stamps (pmp_set_timing): each worker's lane 0 folds its start / end wall-clock tick
__device__ __forceinline__ void span_begin(unsigned long long* span)
{
    if (span && lane_id() == 0) atomicMin(&span[0], (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void span_end(unsigned long long* span)
{
    if (span && lane_id() == 0) atomicMax(&span[1], (unsigned long long)wall_clock64());
}
