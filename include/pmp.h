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

/* Planners that share the AStar loop (2D: a_star.py:39-83; 3D: a_star3d.py:33-78). */
enum { PMP_ALGO_ASTAR = 0, PMP_ALGO_DIJKSTRA = 1, PMP_ALGO_GBFS = 2, PMP_ALGO_THETA = 3, PMP_ALGO_LAZY_THETA = 4 };

/*
 * Batched 2D AStar / Dijkstra / GBFS.  algo = PMP_ALGO_ASTAR is pmp_astar2d_batch;
 * PMP_ALGO_DIJKSTRA replaces Dijkstra.plan (global_planner/graph_search/dijkstra.py:36-85: node_n.h
 * = 0, so `heuristic` is unused); PMP_ALGO_GBFS replaces GBFS.plan (gbfs.py:36-86: node_n.g = 0,
 * ordered by h).  PMP_ALGO_THETA replaces ThetaStar.plan (theta_star.py:44-171: updateVertex with
 * the Bresenham lineOfSight) and PMP_ALGO_LAZY_THETA LazyThetaStar.plan (lazy_theta_star.py:38-114:
 * the line of sight at the pop); both need H <= 4096, and their expand records are
 * cell | code << 26 (code 0-7 path 1 via motion d, 8 start, 16+d path 2, 24+d Lazy Theta*'s
 * re-parenting to the CLOSED neighbour in motion d, +32 g = inf).  Same loop, CPython heap ties,
 * goal -> start path and arguments as pmp_astar2d_batch; cost is extractPath's (a_star.py:98-117).
 */
int pmp_graph2d_batch(pmp_ctx* ctx, void* stream, int algo, const uint32_t* occ_bits, int W, int H, int heuristic,
                      const int32_t* start_xy, const int32_t* goal_xy, int nq, double* cost,
                      int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded,
                      uint32_t* expand, int expand_cap, int64_t* counters, int32_t* status);

/*
 * Batched 3D A*.  Replaces AStar3D.plan (global_planner/graph_search/a_star3d.py:33-106) with
 * GraphSearcher3D.h / isCollision (graph_search_3d.py:30-107) over Grid3D's 26 motions
 * (utils/environment/env3d.py:56-70) and the (f, h, counter) tuple heap.
 *   occ_bits  per_query ? [nq][ceil(X*Y*Z/32)] : [ceil(X*Y*Z/32)] u32, cell (x*Y + y)*Z + z
 *   start_xyz, goal_xyz [nq][3] i32;  X, Y, Z <= 256
 *   cost      [nq] f64   inf when unreachable (a_star3d.py:77-78)
 *   path      [nq][path_cap] u32 cells start -> goal;  n_expanded = len(CLOSED) (distinct cells)
 *   expand    nullable [nq][expand_cap] u32 cells in first-insertion order of CLOSED
 *   counters  nullable [nq][4] i64 pushes, pops, expansions (incl. re-expansions), max heap size
 */
int pmp_astar3d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int per_query, int X, int Y, int Z,
                      int heuristic, const int32_t* start_xyz, const int32_t* goal_xyz, int nq, double* cost,
                      int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded, uint32_t* expand,
                      int expand_cap, int64_t* counters, int32_t* status);

/*
 * Batched 3D AStar3D / Dijkstra3D / GBFS3D.  algo = PMP_ALGO_ASTAR is pmp_astar3d_batch;
 * PMP_ALGO_DIJKSTRA replaces Dijkstra3D.plan (global_planner/graph_search/dijkstra3d.py:39-87: key
 * (g, 0.0, counter), `heuristic` unused; its getNeighbor (:89-126) equals isCollision plus an
 * in-bounds test, and cells outside the grid are blocked here); PMP_ALGO_GBFS replaces
 * GBFS3D.plan (gbfs3d.py:34-82: key (h, counter), CLOSED membership tests); PMP_ALGO_THETA
 * replaces ThetaStar3D.plan (theta_star3d.py:38-110: at each push, the expanding node's CLOSED
 * parent becomes the neighbour's parent when lineOfSight(neighbour, parent) (Bresenham, :139-213)
 * holds and it is cheaper); PMP_ALGO_LAZY_THETA replaces LazyThetaStar3D.plan
 * (lazy_theta_star3d.py:41-128: that update without the test, the test deferred to the pop, where
 * a failed line of sight re-parents the node to its best CLOSED neighbour).  Same arguments as
 * pmp_astar3d_batch; cost is extractPath's (Planner3D.dist along the path) for all five; any-voxel
 * parents make paths shorter than their cell counts suggest.
 */
int pmp_graph3d_batch(pmp_ctx* ctx, void* stream, int algo, const uint32_t* occ_bits, int per_query, int X, int Y,
                      int Z, int heuristic, const int32_t* start_xyz, const int32_t* goal_xyz, int nq, double* cost,
                      int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded, uint32_t* expand,
                      int expand_cap, int64_t* counters, int32_t* status);

/* LocalPlanner.params (local_planner/local_planner.py:39-55), same names and units. */
typedef struct {
    double dt;             /* TIME_STEP */
    double lookahead_time; /* LOOKAHEAD_TIME */
    double max_lookahead;  /* MAX_LOOKAHEAD_DIST */
    double min_lookahead;  /* MIN_LOOKAHEAD_DIST */
    double max_v_inc, min_v_inc, max_v, min_v;
    double max_w_inc, min_w_inc, max_w, min_w;
    double goal_dist_tol, rotate_tol;
} pmp_lp_params;

/* DWA constructor parameters (local_planner/dwa.py:45-56). nv, nw > 0 fix the number of (v, w)
 * samples instead of int((v1 - v0) / v_resolution) (used for the 64 x 64 = 4096-sample bench). */
typedef struct {
    double heading_weight, obstacle_weight, velocity_weight;
    double predict_time;   /* horizon H = int(predict_time / dt) */
    double inflation;      /* obstacle_inflation_radius */
    double v_resolution, w_resolution;
    int32_t nv, nw;
} pmp_dwa_params;

/*
 * Batched DWA control steps.  Replaces `iters` iterations of DWA.plan (local_planner/dwa.py:72-93):
 * reachGoal, getLookaheadPoint (local_planner.py:103-170), calDynamicWin (dwa.py:111-135),
 * evaluation (dwa.py:137-190: H-step Robot.lookforward rollout of every (v, w) sample, heading /
 * obstacle (cdist, capped at the inflation radius) / velocity, numpy pairwise-sum normalisation,
 * eval_win @ factor, first-index argmax) and Robot.kinematic (utils/agent/agent.py:68-116).
 * One workgroup per agent, or -- with fewer agents than CUs and a fixed window (nv, nw > 0) -- k
 * workgroups per agent, each on a leaf-aligned part of numpy's pairwise-sum tree over the samples,
 * the last to finish combining the leaf sums in the tree's order and taking the argmax (the same bits
 * as one workgroup; pmp_dwa_set_split).  Agents never interact.
 *   occ_bits [ceil(W*H/32)] u32  obstacle cells, cell (ox + i, oy + j) at bit i*H + j
 *   state    [na][5] f64  in/out  x, y, theta, v, w
 *   goal     [na][3] f64          goal pose
 *   path_xy  [*][2] f64, path_off [na+1] i32   global path of each agent (start -> goal)
 *   u        [na][2] f64          last applied (v, w)
 *   best     [na] i32             argmax sample index of the last step
 *   status   [na] i32             0 stepped (not at goal), 1 goal reached, 4 the reference raises
 *   n_steps  [na] i32             steps taken in this call
 *   hist_pose [na][iters][3] f64  nullable; robot pose before each step (Robot.history_pose)
 *   eval     [na][4096][3] f64    nullable; eval_win @ factor of the last step, row c = sample c
 *                                  (c < N = nv*nw <= 4096; v outer, w inner as itertools.product)
 *   best_traj [na][iters][H][5] f64 nullable; traj_win[argmax] of every step (history_traj)
 */
int pmp_dwa_step_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int ox, int oy, int W, int H,
                       const pmp_lp_params* lp, const pmp_dwa_params* dp, int na, double* state,
                       const double* goal, const double* path_xy, const int32_t* path_off, int iters,
                       double* u, int32_t* best, int32_t* status, int32_t* n_steps, double* hist_pose,
                       double* eval, double* best_traj);

/*
 * Batched D* static plans.  Replaces DStar.plan (global_planner/graph_search/d_star.py:75-291):
 * __init__ (every cell NEW, insert(goal, 0)), processState until start is CLOSED, extractPath.
 * OPEN keeps the reference's list semantics exactly (append-always insert, first-minimal-k
 * min_state, first-occurrence remove).  One wave64 per query; queries never interact.
 *   occ_bits as pmp_astar2d_batch; start_xy, goal_xy [nq][2] i32
 *   cost [nq] f64        extractPath cost (sum of GraphSearcher.cost along the path)
 *   path [nq][path_cap]  cells x*H + y, start -> goal; path_len [nq]
 *   n_process [nq] i64   processState calls (len(DStar.EXPAND))
 *   status [nq]          0 found, 2 path_cap overflow, 3 capacity / max_process exceeded,
 *                        4 the reference raises (OPEN empties: AttributeError at d_star.py:234;
 *                        path_len -2: processState reached a node on the grid's border, whose
 *                        getNeighbor looks up an out-of-grid key -- KeyError, d_star.py:276-291 --
 *                        and path[0] is that node's cell)
 *   max_process          0 = unbounded, else stop with status 3 after that many processState calls
 * Grids built by Grid.init have obstacle borders, so the border KeyError never happens for them.
 */
int pmp_dstar2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, const int32_t* start_xy,
                      const int32_t* goal_xy, int nq, double* cost, int32_t* path_len, int32_t* path, int path_cap,
                      int64_t* n_process, int32_t* status, int64_t max_process);

/*
 * Batched D* with OnPress replanning.  Replaces DStar.plan followed by npress DStar.OnPress(event)
 * calls (d_star.py:102-134) without the figure: an in-grid press on a free cell adds the obstacle,
 * walks from the start along the parents (the walk's path excludes the goal, as there) and runs
 * modify() (:262-274) -- processState on the kept OPEN / cell states -- where an edge collides.
 *   presses [nq][npress][2]       the pressed cells (x, y)
 *   cost, path_len, n_process, status [nq][npress + 1]; path [nq][npress + 1][path_cap]
 *       round 0 = plan() as pmp_dstar2d_batch; round r: the walk's cost / cells / len(EXPAND);
 *       status 0 walked to the goal, 1 the press changed nothing (off the grid or already an
 *       obstacle: len(EXPAND) is kept), 2 path_cap overflow, 3 a cap or a loop the reference never
 *       leaves (4*W*H+4 steps, or modify() on an empty OPEN), 4 the reference raises (a parentless
 *       node: KeyError, reported with path_len -1; a border node processed: KeyError, path_len -2
 *       and path[r][0] = its cell; OPEN emptied: AttributeError), -1 not run (an earlier call
 *       raised or capped)
 * pmp_dstar2d_batch is this call with npress = 0.
 */
int pmp_dstar2d_onpress_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H,
                              const int32_t* start_xy, const int32_t* goal_xy, int nq, const int32_t* presses, int npress,
                              double* cost, int32_t* path_len, int32_t* path, int path_cap, int64_t* n_process,
                              int32_t* status, int64_t max_process);

/*
 * Batched 3D D* with dynamic obstacles.  Replaces DStar3D (global_planner/graph_search/d_star3d.py:60-281):
 * plan() (:100-109: processState until OPEN empties or the start is CLOSED, then extractPath
 * :153-166) followed by nrounds apply_dynamic_obstacles(newly_blocked) calls (:115-149: block the
 * voxels, walk from the start along the parents, modify() + processState where an edge collides).
 * OPEN keeps the reference's list semantics (append when absent, first-minimal k), so every round's
 * len(EXPAND), cost and path are bit-exact, including the inf costs of the asymmetric isCollision.
 *   occ_bits, per_query, X, Y, Z, start_xyz, goal_xyz as pmp_graph3d_batch (X, Y, Z <= 256)
 *   blocks [nq][nrounds][nblk][3]  voxels newly blocked per round (outside the grid: ignored); may be
 *                                  NULL when nrounds == 0 or nblk == 0
 *   cost, path_len, n_process, status [nq][nrounds + 1]  per round, 0 = plan(): cost (may be inf),
 *                                  len(EXPAND) of that call, status 0 reached the goal, 1 the walk met
 *                                  a parentless voxel (plan: unreachable; the reference returns the
 *                                  partial path), 2 path_cap overflow, 3 cap (max_process, heap, or the
 *                                  4*X*Y*Z+4 walk bound the reference lacks), 4 endpoints off the grid
 *   path [nq][nrounds + 1][path_cap]  voxel ids (x*Y + y)*Z + z, start -> goal (round 0: extractPath's
 *                                  path; rounds: apply_dynamic_obstacles' path, the goal appended when
 *                                  reached)
 *   expand [nq][expand_cap]        nullable: plan()'s EXPAND as voxel ids, in order (duplicates kept)
 *   max_process                    0 = unbounded, else a processState cap per round
 */
int pmp_dstar3d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int per_query, int X, int Y, int Z,
                      const int32_t* start_xyz, const int32_t* goal_xyz, int nq, const int32_t* blocks, int nrounds,
                      int nblk, double* cost, int32_t* path_len, int32_t* path, int path_cap, int64_t* n_process,
                      int32_t* status, int32_t* expand, int expand_cap, int64_t max_process);

/*
 * Batched 3D LPA* with apply_change rounds.  Replaces LPAStar3D (global_planner/graph_search/
 * lpa_star3d.py:40-225): plan() (:78-82: computeShortestPath :127-145, extractPath :185-225, the
 * greedy min-g walk from the goal that gives (cost, []) when stuck or after 100000 steps) followed by
 * nr apply_change(coord, blocked) calls (:93-124), each re-planning on the kept g / rhs / U.  U keeps
 * the reference's list semantics, so every call's len(EXPAND), cost and path are bit-exact.
 *   occ_bits, per_query, X, Y, Z, heuristic, start_xyz, goal_xyz as pmp_graph3d_batch
 *   changes [nq][nr][4]      (x, y, z, mode): mode 0 = blocked None (toggle), 1 = True, 2 = False
 *   cost, path_len, n_expanded, status [nq][nr + 1]; path [nq][nr + 1][path_cap] (voxels, start -> goal)
 *       status 0 path, 1 the reference's empty path (cost kept), 2 path_cap overflow, 3 max_expansions
 *       (0 = unbounded) hit, 4 endpoints off the grid, -1 not run (an earlier call hit a cap)
 *   counters [nq][4] nullable: U pushes, expansions (all calls), 0, max |U|
 */
int pmp_lpastar3d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int per_query, int X, int Y, int Z,
                        int heuristic, const int32_t* start_xyz, const int32_t* goal_xyz, int nq, const int32_t* changes,
                        int nr, double* cost, int32_t* path_len, int32_t* path, int path_cap, int64_t* n_expanded,
                        int32_t* status, int64_t* counters, int64_t max_expansions);

/*
 * Batched LPA*.  Replaces LPAStar.plan (global_planner/graph_search/lpa_star.py:78-87): the initial
 * computeShortestPath (:139-160) with updateVertex (:162-179), and extractPath (:209-230).  U keeps
 * the reference's Python-list semantics (first-minimal `min(U, key)`, shifting `U.remove`,
 * `heapq.heappush` on the list), so the expansion order, len(EXPAND) and costs are bit-exact.
 *   occ_bits, heuristic, start_xy, goal_xy as pmp_astar2d_batch
 *   cost [nq] f64        extractPath cost; also kept when extractPath gives up after 1000 steps
 *   path [nq][path_cap]  cells x*H + y, start -> goal (path_cap >= 1001 covers every result)
 *   n_expanded [nq]      len(EXPAND) of computeShortestPath
 *   counters nullable [nq][4] i64: pushes, expansions, extractPath steps, max |U|
 *   status [nq]          0 found, 1 extractPath gave up (1000 steps: the reference returns
 *                        (cost, [], None)), 2 path_cap overflow, 4 the reference raises (U empties:
 *                        ValueError from min(); a neighbour off the grid: KeyError; start == goal
 *                        ends that way too, the goal node being detached from the map)
 */
int pmp_lpastar2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                        const int32_t* start_xy, const int32_t* goal_xy, int nq, double* cost, int32_t* path_len,
                        uint32_t* path, int path_cap, int32_t* n_expanded, int64_t* counters, int32_t* status);

/*
 * Batched D* Lite.  Replaces DStarLite.plan (global_planner/graph_search/d_star_lite.py:14-187; plan()
 * is LPAStar's): the same list-semantics U, searched from the goal (rhs = 0) toward the start with
 * keys min(g, rhs) + h(node, start) + km (km = 0), outdated keys re-keyed at the pop (:104-106), and
 * extractPath from the start to the goal (:156-187).  Arguments, outputs and statuses as
 * pmp_lpastar2d_batch; start == goal raises in the reference (status 4 after one expansion).
 */
int pmp_dstarlite2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                          const int32_t* start_xy, const int32_t* goal_xy, int nq, double* cost, int32_t* path_len,
                          uint32_t* path, int path_cap, int32_t* n_expanded, int64_t* counters, int32_t* status);

/*
 * Batched LPA* incremental replanning: LPAStar.plan() followed by nt LPAStar.OnPress edits
 * (global_planner/graph_search/lpa_star.py:101-137) without the figure.  Edit p toggles the
 * obstacle at toggles[q][p] (in-grid cells): a freed cell gets updateVertex, then its free
 * neighbours do, and plan() runs again on the kept g / rhs / U (len(EXPAND) restarts per plan).
 * Each worker edits its own copy of the grid; the shared occ_bits are not written.
 *   toggles   [nq][nt][2] i32 (nt >= 1)
 *   cost, n_expanded, status  [nq][nt + 1]: every plan's result, status as pmp_lpastar2d_batch,
 *             -1 = not run (an earlier plan raised, which ends OnPress in the reference)
 *   path_len [nq], path [nq][path_cap]: the last plan's path (start -> goal)
 *   counters  nullable [nq][4] i64, cumulative over the plans (pushes, last plan's expansions and
 *             extractPath steps, max |U|)
 */
int pmp_lpastar2d_replan_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                               const int32_t* start_xy, const int32_t* goal_xy, int nq, const int32_t* toggles, int nt,
                               double* cost, int32_t* n_expanded, int32_t* status, int32_t* path_len, uint32_t* path,
                               int path_cap, int64_t* counters);

/*
 * Batched D* Lite incremental replanning: DStarLite.plan() followed by nt DStarLite.OnPress calls
 * (global_planner/graph_search/d_star_lite.py:61-97) without the figure: walk from the start along
 * min-g neighbours; after the first step set km = h(step, start), apply the edit as
 * pmp_lpastar2d_replan_batch does, computeShortestPath on the kept state, and walk on to the goal.
 * cost[q][p] is the walk's cost and path the last walk (start -> goal); the walk has no step limit
 * in the reference (it can loop forever), so here it stops with status 3 after 4 W H + 4 steps.
 * Arguments and outputs otherwise as pmp_lpastar2d_replan_batch.
 */
int pmp_dstarlite2d_replan_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                                 const int32_t* start_xy, const int32_t* goal_xy, int nq, const int32_t* toggles,
                                 int nt, double* cost, int32_t* n_expanded, int32_t* status, int32_t* path_len,
                                 uint32_t* path, int path_cap, int64_t* counters);

/* LQR settings (local_planner/lqr.py:35-38): diag Q, diag R, Riccati iteration cap and the
 * signed exit threshold of lqr.py:134.  Reference defaults: q = 1,1,1  r = 1,1  iters 100  eps 0.1. */
typedef struct {
    double q[3], r[2];
    int32_t iters;
    double eps;
} pmp_lqr_params;

/* MPC settings: horizons and weights of mpc.py:37-40 (p = prediction horizon, m = control horizon
 * <= 8, Q = diag q, R = diag r), then the ADMM settings of the QP solve that replaces OSQP
 * (mpc.py:196-203): rho, sigma, relaxation alpha, eps_abs / eps_rel on the inf-norm residuals,
 * max_iter, termination checked every check_every iterations, rho adapted every adaptive_every
 * iterations (0 = never) when the residual-ratio estimate leaves [rho/adaptive_tol, rho*adaptive_tol]. */
typedef struct {
    int32_t p, m;
    double q[3], r[2];
    double rho, sigma, alpha, eps_abs, eps_rel, adaptive_tol;
    int32_t max_iter, check_every, adaptive_every, reserved;
} pmp_mpc_params;

/*
 * Batched LQR.lqrControl (local_planner/lqr.py:103-145), one thread per call:
 *   s, s_d [n][3]   current and desired (x, y, theta)      u_r [n][2]  reference (v, w)
 *   robot_vw [n][2] the robot's current (v, w) for linear/angularRegularization (local_planner.py:172-206)
 *   u [n][2]        regularised control
 */
/* Workgroups per agent of pmp_dwa_step_batch: 0 (default) = auto (the device's CUs over the agents,
 * at most 16, only for fixed windows nv, nw > 0), 1 = one workgroup per agent, k = k parts (reduced
 * to the sample tree's leaf count; a part holds at most 1024 samples).  Results are identical for
 * every setting. */
int pmp_dwa_set_split(pmp_ctx* ctx, int parts);

int pmp_lqr_control_batch(pmp_ctx* ctx, void* stream, const pmp_lp_params* lp, const pmp_lqr_params* lq, int n,
                          const double* s, const double* s_d, const double* u_r, const double* robot_vw, double* u);

/*
 * Batched MPC.mpcControl (local_planner/mpc.py:111-214), four calls per wave64 (one per 16-lane
 * row): QP assembly (S_u'QS_u on the f64 MFMA 16x16x4, one pass per row's agent), ADMM solve on the
 * row (DPP broadcasts and scans), u = du0 + u_p + u_r, regularisation.
 *   u_p [n][2] in/out  carried control error (returned as u - u_r, before regularisation)
 *   qp_H [n][2m][2m], qp_g [n][2m], qp_lu [n][2][4m], du [n][2m]   nullable: the assembled QP and its solution
 *   admm_iters, admm_status [n] i32  nullable: iterations, 0 converged / 1 iteration limit
 */
int pmp_mpc_control_batch(pmp_ctx* ctx, void* stream, const pmp_lp_params* lp, const pmp_mpc_params* mp, int n,
                          const double* s, const double* s_d, const double* u_r, double* u_p, const double* robot_vw,
                          double* u, double* qp_H, double* qp_g, double* qp_lu, double* du, int32_t* admm_iters,
                          int32_t* admm_status);

#define PMP_TRACK_LQR 0
#define PMP_TRACK_MPC 1
/*
 * Batched tracking-controller plan iterations: `iters` iterations of LQR.plan (lqr.py:58-86,
 * kind PMP_TRACK_LQR) or MPC.plan (mpc.py:66-94, kind PMP_TRACK_MPC) per agent, four agents per
 * wave64 (one per 16-lane row): reachGoal, getLookaheadPoint, the rotate/move branch, lqrControl / mpcControl,
 * Robot.kinematic.  Arrays as pmp_dwa_step_batch, plus
 *   u_p [na][2] f64 in/out   MPC's carried u_p (start a plan with zeros); unused for LQR
 *   admm_iters [na] i32      nullable; ADMM iterations summed over this call's steps
 */
int pmp_track_step_batch(pmp_ctx* ctx, void* stream, int kind, const pmp_lp_params* lp, const pmp_lqr_params* lq,
                         const pmp_mpc_params* mp, int na, double* state, double* u_p, const double* goal,
                         const double* path_xy, const int32_t* path_off, int iters, double* u, int32_t* status,
                         int32_t* n_steps, double* hist_pose, int32_t* admm_iters);

/* RRT / RRT* settings: Map size (utils/environment/env.py:92), inflation delta (sample_search.py:22),
 * max_dist, sample_num, goal_sample_rate (rrt.py:36-44), radius r (rrt_star.py:34-38). */
typedef struct {
    double x_range, y_range, delta;
    double max_dist, radius, goal_sample_rate;
    int32_t sample_num;
    int32_t star;          /* 1 = RRTStar.getNearest (choose parent + rewire), 0 = RRT */
} pmp_rrt_params;

/*
 * Batched RRT / RRT*.  Replaces RRT.plan (global_planner/sample_search/rrt.py:49-151) with
 * SampleSearcher.isCollision (sample_search.py:27-135) and RRTStar.getNearest (rrt_star.py:43-76).
 * One workgroup per query; queries never interact.  All arrays are device pointers.
 *   rect [nr][4] (x, y, w, h), circ [nc][3] (x, y, r), bnd [nb][4]   the Map's obs_rect, obs_circ, boundary
 *   start_xy, goal_xy [nq][2]
 *   rnd [nq][rnd_stride]  each query's np.random double stream, in RandomState.random_sample order
 *                         (generateRandomNode draws one double, then two uniforms if it exceeds
 *                         goal_sample_rate); 3*sample_num+1 doubles always suffice
 *   tree_xy [nq][tree_cap][2], tree_g [nq][tree_cap], tree_parent [nq][tree_cap]   out: sample_list in
 *                         insertion order (the start is node 0 and its own parent; the goal is last when found)
 *   n_nodes [nq]          out: len(sample_list)
 *   cost [nq]             out: goal.g, 0 when not found
 *   path_len [nq], path_xy [nq][path_cap][2]   out: extractPath goal -> start
 *   draws [nq] i64        out: doubles consumed from rnd (advance the caller's RNG by this many)
 *   status [nq]           0 found, 1 not found (returns (0, None, nodes)), 2 path_cap overflow,
 *                         3 tree_cap / stream / candidate-list overflow, 4 parent cycle (reference hangs)
 *   counters [nq][4] i64  nullable: iterations, nodes scanned (nearest + radius passes), in-radius
 *                         candidates, segment collision tests
 * A new RRT* node that lands exactly on an existing one replaces it (dict semantics); plain RRT does
 * not check for that (a measure-zero event).
 */
int pmp_rrt_batch(pmp_ctx* ctx, void* stream, const pmp_rrt_params* p, const double* rect, int nr,
                  const double* circ, int nc, const double* bnd, int nb, const double* start_xy,
                  const double* goal_xy, int nq, const double* rnd, int64_t rnd_stride, int tree_cap,
                  double* tree_xy, double* tree_g, int32_t* tree_parent, int32_t* n_nodes, double* cost,
                  int32_t* path_len, double* path_xy, int path_cap, int64_t* draws, int32_t* status,
                  int64_t* counters);

/* TrajectoryConstraints (trajectory/trajectory_base.py:30-45) and TimeOptimalTrajectory3D's
 * path_resolution (trajectory/time_optimal_trajectory.py:17-29) */
typedef struct {
    double max_velocity[3];
    double max_acceleration[3];
    double min_time_step;
    double path_resolution;
} pmp_totp_params;

/*
 * Batched time-optimal trajectories (config 5's step after 3D planning, examples/3d_example.py:93-128).
 * Replaces TimeOptimalTrajectory3D(path, constraints, path_resolution).generate()
 * (trajectory/time_optimal_trajectory.py:260-302): arc-length parameterisation with scipy's
 * not-a-knot CubicSpline per axis (:41-74), forward / backward velocity integration (:162-226, the
 * reference's sign handling for q' < 0 included), s_ddot and time profiles (:228-258), sampling at
 * t = 0, dt, ... (+ total_time) through interp1d (:304-335), yaw / yaw rate
 * (trajectory_base.py:245-261).  Values match the reference to rounding.
 *   path_xyz [sum n][3] f64, path_off [nq + 1] i32   waypoints per path (reference order)
 *   max_waypoints  >= every path's n (sizes LDS; <= 480)
 *   s_values, s_dot, s_ddot, time_profile [nq][sample_cap]; n_samples [nq] = max(int(L / res), 100)
 *   points [nq][point_cap][12]: time, position[3], velocity[3], acceleration[3], yaw, yaw rate
 *       (NaN where the reference leaves None); n_points [nq]; total_time [nq]
 *   status [nq]  0 ok, 2 sample_cap or point_cap too small (the counts are still reported),
 *                3 path longer than max_waypoints, 4 the reference raises (< 2 waypoints, or
 *                repeated consecutive waypoints: scipy needs strictly increasing knots)
 *   eval_t [n_eval] nullable: instead of generate()'s sampling, evaluate(t) (:304-335) at these times
 *       (yaw / yaw rate NaN, as evaluate leaves them)
 */
int pmp_totp3d_batch(pmp_ctx* ctx, void* stream, const pmp_totp_params* prm, int nq, const double* path_xyz,
                     const int32_t* path_off, int max_waypoints, int sample_cap, double* s_values, double* s_dot,
                     double* s_ddot, double* time_profile, int32_t* n_samples, int point_cap, double* points,
                     int32_t* n_points, double* total_time, int32_t* status, const double* eval_t, int n_eval);

/* Launch-span recording for profiling: while set, every A* 2D launch of this context folds its
 * workers' first start and last end wall-clock ticks into span[0] (atomic min) and span[1] (atomic
 * max); the caller initialises span to {UINT64_MAX, 0}.  NULL switches it off. */
int pmp_set_timing(pmp_ctx* ctx, uint64_t* span);
/* Work counters for profiling: while set, every MPC pmp_track_step_batch launch of this context adds
 * the number of QP solves it ran (agent-iterations whose MPC.plan branch called mpcControl,
 * mpc.py:85-91) into stats[0] (atomic add; the caller zeroes it).  The matrix-core work of a launch
 * is that count x ceil(3p / 16) x 10 v_mfma_f64_16x16x4 instructions.  NULL switches it off. */
int pmp_set_stats(pmp_ctx* ctx, int64_t* stats);
/* Rate of the wall-clock ticks above, in kHz. */
int pmp_wall_clock_khz(pmp_ctx* ctx, int* khz);
/* A* 2D query scheduling across the persistent workers: 1 (default) = longest start-goal distance
 * first (the expansion count grows with it, so long queries stop forming a tail), 0 = input order.
 * Results are identical either way; only which worker runs which query changes. */
int pmp_astar2d_set_schedule(pmp_ctx* ctx, int longest_first);
/* With the longest-first schedule, the first n_high queries (the longest) run at raised wave
 * priority, so they finish sooner and the short queries fill the issue slots they leave idle.
 * Default 64; 0 switches it off.  Results are identical for any value. */
int pmp_astar2d_set_priority(pmp_ctx* ctx, int n_high);
/* A* 2D queries resident per CU across all the launches that run at once, in [0, 128] (default 0 =
 * this context's own launch alone: ceil(max_slots / 256) of pmp_astar2d_reserve).  The LDS share of
 * each query's heap is 160 KiB / per_cu, so several batches in flight with fewer queries each (e.g.
 * 6 contexts x 2048 queries on the multi-query engine) set 48 here to stay resident together: every
 * batch's longest queries then start at once instead of behind the earlier batches.  A share too
 * small for the engine's fixed LDS needs is refused (PMP_EINVAL).  Re-sizes the reserved scratch
 * (call after pmp_astar2d_reserve).  Results are identical for any accepted value. */
int pmp_astar2d_set_residency(pmp_ctx* ctx, int per_cu);

/* A* 2D engine of the context (replaces nothing in the reference: a scheduling knob of
 * AStar.plan / Dijkstra.plan / GBFS.plan, a_star.py:39-83).  engine 2: four queries per wave, one
 * per 16-lane row, for A* / Dijkstra / GBFS whose heaps stay within 32,767 entries (a query that
 * outgrows it reports PMP_CAP_OVERFLOW; re-reserving with a larger heap_cap selects engine 0);
 * t2_lds = keep its level-10..14 heap direction bits in LDS (1) or HBM (0).  engine 0: one query per
 * wave (also Theta* / Lazy Theta*, and heaps of any size); on grids whose occupancy, cell state and
 * g fit in a wave's LDS share beside its heap (the README grid: 14 KB) all of them live in LDS.
 * engine 3: one query per workgroup with the CU's whole LDS as its heap (pmp_astar2d_sq_cap entries:
 * 13,632 beside no grid; a query that outgrows it reports PMP_CAP_OVERFLOW) and the heap's choice bits in
 * registers -- a single query's latency (the drop-in AStar.plan).  engine 1 (default): engine 3 for
 * batches of <= 256 queries whose heap capacity it holds, engine 2 for batches of >= 1024 queries on
 * grids too large for engine 0's LDS grid block, engine 0 otherwise.  Results are identical.
 * Applies to the next launch (re-reserves the scratch geometry when one is set). */
int pmp_astar2d_set_engine(pmp_ctx* ctx, int engine, int t2_lds);
/* Heap entries engine 3 holds for a W x H grid (its LDS beside the grid block it keeps in LDS on
 * small grids); 0 = the grid leaves too little for the engine.  No device call. */
int pmp_astar2d_sq_cap(int W, int H);

/* Persistent workers (one wave each) per CU of the one-wave-per-query planners: pmp_graph3d_batch,
 * pmp_dstar2d_batch / pmp_dstar2d_onpress_batch, pmp_dstar3d_batch and pmp_lpastar3d_batch (default 16
 * each), and the LPA* / D* Lite 2D entry points (default 24); 0 = the default.
 * Each launch caps it at ceil(nq / 256), so a small batch gets fewer workers with a larger LDS share
 * each.  Fewer workers leave each a larger LDS share of its heap (fewer spilled positions), more
 * workers hide more latency.  The longest-first schedule and its raised priority
 * (pmp_astar2d_set_schedule, pmp_astar2d_set_priority) apply to these planners as well.  Results are
 * identical for any value. */
int pmp_set_workers_per_cu(pmp_ctx* ctx, int per_cu);
/* pmp_dstar2d_batch / pmp_dstar2d_onpress_batch run in two passes: the first with a heap and entry
 * capacity of `entries` per query (0 = the default, W*H + 64: a smaller per-worker scratch, so more
 * workers fit the scratch budget), the second, on the same stream, re-runs every query whose heap or
 * entry list outgrew it with the bound (4 W*H + 64) on a few workers.  Results are identical for any
 * value. */
int pmp_dstar_set_first_cap(pmp_ctx* ctx, int entries);
/* Workers resident per CU over all the launches that run at once, for pmp_graph3d_batch,
 * pmp_dstar2d_batch / pmp_dstar2d_onpress_batch and pmp_dstar3d_batch: each worker's LDS heap share
 * is sized for max(this, the launch's own workers per CU), so several batches in flight with few
 * workers each stay resident together (as pmp_astar2d_set_residency for A* 2D); 0 = the launch's own
 * count.  pmp_rrt_batch sizes each query's LDS copy of its tree for this many workgroups per CU, at
 * least 2 (its 256-thread workgroups run two per CU) and at most 4.  Results are identical for any
 * value. */
int pmp_set_resident_per_cu(pmp_ctx* ctx, int per_cu);

/* Pre-size the A* scratch (heap of heap_cap entries per concurrent query, up to max_slots
 * concurrent queries) so that later batch calls allocate nothing (hipGraph-capturable). */
int pmp_astar2d_reserve(pmp_ctx* ctx, int W, int H, int max_slots, int heap_cap);
/* The A* 2D scratch geometry in force: out[0..5] = {W, H, max_slots, heap_cap in force, flags,
 * sized by the launches (1) or by pmp_astar2d_reserve (0)}; all 0 before any.  flags: bit 0 the
 * multi-query engine is reserved, bit 1 heap_cap was the caller's own (pmp_astar2d_reserve's
 * heap_cap > 0) -- without it the geometry is restored with heap_cap = 0 (the default, which the
 * engine may cut to its limit). */
int pmp_astar2d_geometry(pmp_ctx* ctx, int32_t* out6);
/* Forget the host's pmp_astar2d_reserve geometry: the next launch sizes the scratch for its own
 * batch and later larger batches grow it, as on a fresh context (allocated scratch is kept). */
int pmp_astar2d_reserve_auto(pmp_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* PMP_H */
